// cpl/CentroidalPlanner.hpp — host facade of the MI355X engine.
//
// Mirrors include/CentroidalPlanner/CentroidalPlanner.h and CoMPlanner.h of the reference (same
// public methods, argument meaning, validation and exception types; src/CentroidalPlanner.cpp,
// src/CoMPlanner.cpp).  The reference's solver member is an ifopt::IpoptSolver
// (CentroidalPlanner.h:232); IPOPT is not part of this build, so the solver is the NlpSolver
// interface below: any NLP solver that drives a CplTNLP (an Ipopt::TNLP forwarding adapter, see
// INTEGRATION.md §1), by default the native engine (NativeSolver: IPOPT's interior-point method on
// the GPU, csrc/cpl_solver.hip, with IFOPT's IpoptSolver defaults — limited-memory Hessian,
// max_iter 3000, tol 1e-8).  Like IFOPT's solver, a solve that ends unconverged does not throw
// (LastSolveSucceeded() tells); a HIP failure throws std::runtime_error.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "cpl/CplProblem.hpp"

namespace cpl {

namespace solver {
class NlpSolver {
 public:
  typedef std::shared_ptr<NlpSolver> Ptr;
  virtual ~NlpSolver() = default;
  // runs the solve; must call nlp.finalize_solution with the final iterate.  true on success.
  virtual bool Solve(CplTNLP& nlp) = 0;
};

// The native engine's options (cpl_solve_options), IFOPT's IpoptSolver defaults: limited-memory
// Hessian (src/CentroidalPlanner.cpp:22-29 keeps IFOPT's setting), max_iter 3000, tol 1e-8.
struct SolveOptions : cpl_solve_options {
  SolveOptions() {
    cpl_solve_options_default(this);
    hessian = CPL_HESSIAN_LIMITED_MEMORY;
  }
  // src/CentroidalPlanner.cpp:26 SetOption("derivative_test", "first-order"): IPOPT's first-order
  // derivative checker at the start point of every solve (cpl_derivative_test); NativeSolver keeps
  // the report.  IPOPT's defaults for the perturbation and the tolerance.
  bool derivative_test = true;
  double derivative_test_perturbation = 1e-8;
  double derivative_test_tol = 1e-4;
};

// Many instances of one problem template solved at once on the GPU by the native engine
// (cpl_solver_*): host arrays in and out, device buffers and the captured iteration kept between
// solves.  x0 / x: [batch * n] (vector order of CplProblem), mass: [batch] or nullptr (the
// template's), outputs may be nullptr.  Throws std::runtime_error on a HIP / engine failure.
class BatchSolver {
 public:
  BatchSolver(CplProblem::Ptr problem, int64_t batch, const SolveOptions& opt = SolveOptions());
  ~BatchSolver();
  BatchSolver(const BatchSolver&) = delete;
  BatchSolver& operator=(const BatchSolver&) = delete;

  void Solve(const double* x0, const double* mass, double* x, double* y = nullptr, int32_t* status = nullptr,
             int32_t* iterations = nullptr, double* objective = nullptr, double* primal_inf = nullptr);
  int64_t batch() const { return _batch; }
  int32_t iterations_run() const { return _iterations_run; }
  bool graph_captured() const;
  // per instance, the NaN Jacobian entries the last Solve met at its start point (taken as 0):
  // counts [batch] on the host (cpl_solver_nan_jacobian)
  void NanJacobian(int32_t* counts) const;

 private:
  void release();  // frees every device resource (idempotent: pointers nulled)
  CplProblem::Ptr _problem;
  int64_t _batch;
  cpl_solver* _solver = nullptr;
  void* _stream = nullptr;
  double *_dx0 = nullptr, *_dmass = nullptr, *_dx = nullptr, *_dy = nullptr, *_dobj = nullptr, *_dpinf = nullptr;
  int32_t *_dstatus = nullptr, *_diters = nullptr;
  int32_t* _dnan = nullptr;  // [batch] NaN Jacobian counts (NanJacobian), allocated with the others
  int32_t _iterations_run = 0;
};

// CentroidalPlanner's default solver: the native engine on a batch of one, from the problem's
// current variables (x = 0 initially, src/Variable3D.cpp:8-10), finalize_solution with the result.
class NativeSolver : public NlpSolver {
 public:
  explicit NativeSolver(const SolveOptions& opt = SolveOptions()) : _opt(opt) {}
  bool Solve(CplTNLP& nlp) override;
  int32_t status() const { return _status; }        // CPL_SOLVE_*
  int32_t iterations() const { return _iterations; }
  double primal_inf() const { return _primal_inf; }
  // the derivative checker's report of the last Solve (n_checked == 0 when it did not run)
  const cpl_derivative_report& derivative_report() const { return _dreport; }
  // Jacobian entries that were NaN at the last Solve's start point (FrictionCone's 0/0 where the
  // tangential force is 0, src/Constraints/FrictionCone.cpp:85-87 — e.g. at x = 0): IPOPT would
  // receive them as NaN; the engine takes them as 0 (a subgradient).  0: no substitution happened.
  int32_t nan_jacobian_at_start() const { return _nan_jac_start; }

 private:
  SolveOptions _opt;
  std::unique_ptr<BatchSolver> _bs;  // kept between solves of the same template (_bs_desc)
  const CplProblem* _bs_problem = nullptr;
  cpl_problem_desc _bs_desc{};
  int32_t _status = -1, _iterations = 0, _nan_jac_start = 0;
  double _primal_inf = 0.0;
  cpl_derivative_report _dreport{};
};
}  // namespace solver

class CentroidalPlanner {
 public:
  typedef std::shared_ptr<CentroidalPlanner> Ptr;

  // throws std::invalid_argument("Invalid robot mass") if robot_mass <= 0 (src/CentroidalPlanner.cpp:12-15)
  CentroidalPlanner(std::vector<std::string> contact_names, double robot_mass, env::EnvironmentClass::Ptr env);

  solver::Solution Solve();
  void SetSolver(solver::NlpSolver::Ptr s) { _cpl_solver = std::move(s); }
  bool LastSolveSucceeded() const { return _last_ok; }

  void SetManipulationWrench(const VectorXd& wrench_manip);
  VectorXd GetManipulationWrench() const;

  void SetForceBounds(std::string contact_name, const Vector3d& force_lb, const Vector3d& force_ub);
  void GetForceBounds(std::string contact_name, Vector3d& force_lb, Vector3d& force_ub) const;
  void SetPosBounds(std::string contact_name, const Vector3d& pos_lb, const Vector3d& pos_ub);
  void GetPosBounds(std::string contact_name, Vector3d& pos_lb, Vector3d& pos_ub) const;
  void GetNormalBounds(std::string contact_name, Vector3d& normal_lb, Vector3d& normal_ub) const;

  void SetPosRef(std::string contact_name, const Vector3d& pos_ref);
  Vector3d GetPosRef(std::string contact_name) const;
  void SetForceRef(std::string contact_name, const Vector3d& force_ref);
  Vector3d GetForceRef(std::string contact_name) const;
  void SetCoMRef(const Vector3d& com_ref);
  Vector3d GetCoMRef() const;

  void SetCoMWeight(double W_CoM);
  double GetCoMWeight() const;
  void SetPosWeight(double W_p);
  std::map<std::string, double> GetPosWeight() const;
  void SetContactPosWeight(std::string contact_name, double W_p);
  double GetContactPosWeight(std::string contact_name) const;
  void SetForceWeight(double W_F);
  std::map<std::string, double> GetForceWeight() const;
  void SetContactForceWeight(std::string contact_name, double W_F);
  double GetContactForceWeight(std::string contact_name) const;

  double GetMu() const;

  void SetForceThreshold(std::string contact_name, double F_thr);
  double GetForceThreshold(std::string contact_name) const;

  virtual ~CentroidalPlanner() = default;

 protected:
  void SetNormalBounds(std::string contact_name, const Vector3d& normal_lb, const Vector3d& normal_ub);
  bool HasContact(const std::string& contact_name) const;
  solver::CplProblem::Ptr GetCplProblem() const { return _cpl_problem; }

 private:
  void CheckContact(const std::string& contact_name) const;

  std::vector<std::string> _contact_names;
  double _robot_mass;
  env::EnvironmentClass::Ptr _env;
  solver::NlpSolver::Ptr _cpl_solver;
  solver::CplProblem::Ptr _cpl_problem;
  bool _last_ok = false;
};

// include/CentroidalPlanner/CoMPlanner.h (private inheritance, env = nullptr)
class CoMPlanner : private CentroidalPlanner {
 public:
  typedef std::shared_ptr<CoMPlanner> Ptr;

  CoMPlanner(std::vector<std::string> contact_names, double robot_mass);

  void SetLiftingContact(std::string contact_name);
  std::vector<std::string> GetLiftingContacts() const;
  void ResetLiftingContact(std::string contact_name);
  void SetContactPosition(std::string contact_name, const Vector3d& pos_ref);
  Vector3d GetContactPosition(std::string contact_name) const;
  void SetContactNormal(std::string contact_name, const Vector3d& n_ref);
  Vector3d GetContactNormal(std::string contact_name) const;
  void SetMu(double mu);

  using CentroidalPlanner::GetCoMRef;
  using CentroidalPlanner::GetCoMWeight;
  using CentroidalPlanner::GetForceThreshold;
  using CentroidalPlanner::GetForceWeight;
  using CentroidalPlanner::GetMu;
  using CentroidalPlanner::GetPosWeight;
  using CentroidalPlanner::LastSolveSucceeded;
  using CentroidalPlanner::SetCoMRef;
  using CentroidalPlanner::SetCoMWeight;
  using CentroidalPlanner::SetForceThreshold;
  using CentroidalPlanner::SetForceWeight;
  using CentroidalPlanner::SetPosWeight;
  using CentroidalPlanner::SetSolver;
  using CentroidalPlanner::Solve;

 protected:
  bool IsLiftingContact(const std::string& contact_name) const;

 private:
  std::vector<std::string> _contact_names;
  std::map<std::string, double> _F_thr_map;
};

}  // namespace cpl
