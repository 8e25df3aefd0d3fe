// cpl/CplProblem.hpp — host-side problem template, solution types and the IPOPT TNLP hooks.
//
// Mirrors include/CentroidalPlanner/Ifopt/{CplProblem,Types}.h and src/CplProblem.cpp of the
// reference (names, argument meaning, std::map::at -> std::out_of_range, Variable3D::SetBounds ->
// std::invalid_argument "Inconsistent bounds").  The IFOPT components behind it (Variable3D,
// CentroidalStatics, FrictionCone, EnvironmentConstraint, EnvironmentNormal,
// MinimizeCentroidalVariables) are not host objects: their GetValues / FillJacobianBlock /
// GetCost / gradient run as one fused HIP kernel over a batch of instances (cpl_eval_batch), and
// the problem is the plain-data cpl_problem_desc that kernel reads.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <ostream>
#include <string>
#include <vector>

#include "cpl/Environment.hpp"
#include "cpl_mi355x.h"

namespace cpl {

using VectorXd = std::vector<double>;

// throws the reference's exception type for a failing C-ABI status (cpl_last_error() message)
void ThrowOnError(int32_t status);

namespace solver {

// include/CentroidalPlanner/Ifopt/Types.h:8-21
struct ContactValues {
  Vector3d force_value{};
  Vector3d position_value{};
  Vector3d normal_value{};
};

struct Solution {
  std::map<std::string, ContactValues> contact_values_map;
  Vector3d com_sol{};
  friend std::ostream& operator<<(std::ostream& os, const Solution& sol);  // src/CplProblem.cpp:321-344
};

// src/CplProblem.cpp
class CplProblem {
 public:
  typedef std::shared_ptr<CplProblem> Ptr;

  // env == nullptr: the CoMPlanner problem (FrictionCone only; mu kept by a private Ground,
  // src/CplProblem.cpp:14,63-71)
  CplProblem(std::vector<std::string> contact_names, double robot_mass, env::EnvironmentClass::Ptr env);

  void GetSolution(Solution& sol) const;

  void SetManipulationWrench(const VectorXd& wrench_manip);
  VectorXd GetManipulationWrench() const;

  void SetForceBounds(std::string contact_name, const Vector3d& force_lb, const Vector3d& force_ub);
  void GetForceBounds(std::string contact_name, Vector3d& force_lb, Vector3d& force_ub) const;
  void SetPosBounds(std::string contact_name, const Vector3d& pos_lb, const Vector3d& pos_ub);
  void GetPosBounds(std::string contact_name, Vector3d& pos_lb, Vector3d& pos_ub) const;
  void SetNormalBounds(std::string contact_name, const Vector3d& normal_lb, const Vector3d& normal_ub);
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
  void SetContactPosWeight(std::string contact_name, double W_p);
  double GetContactPosWeight(std::string contact_name) const;
  void SetForceWeight(double W_F);
  void SetContactForceWeight(std::string contact_name, double W_F);
  double GetContactForceWeight(std::string contact_name) const;

  void SetMu(double mu);
  double GetMu() const;
  void SetForceThreshold(std::string contact_name, double F_thr);
  double GetForceThreshold(std::string contact_name) const;

  // ---- engine side ----------------------------------------------------------------------------
  // the problem template with the environment's current state folded in
  const cpl_problem_desc& Desc() const;
  const std::vector<std::string>& ContactNames() const { return _contact_names; }
  int32_t n() const { return _n; }
  int32_t m() const { return _m; }
  int32_t nnz() const { return _nnz; }
  // the persistent variable values (Variable3D, init 0; the warm start of the next Solve)
  const VectorXd& GetVariables() const { return _x; }
  void SetVariables(const VectorXd& x);

 private:
  int32_t Index(const std::string& contact_name) const;  // std::map::at semantics
  void SetBounds(int32_t var, const std::string& contact_name, const Vector3d& lb, const Vector3d& ub);

  std::vector<std::string> _contact_names;
  std::map<std::string, int32_t> _index;
  env::EnvironmentClass::Ptr _env;
  env::Ground::Ptr _ground_fake;
  mutable cpl_problem_desc _desc;
  int32_t _n = 0, _m = 0, _nnz = 0;
  VectorXd _x;
};

// The IPOPT TNLP hooks IFOPT's IpoptAdapter exposes for a CplProblem [IFOPT-ext], with IPOPT's
// argument meaning (C_STYLE indices, inf = 1e20, eval_jac_g(values == NULL) = structure).  Every
// callback of one x runs ONE fused launch on the GPU (g, jac, f and grad together, through
// cpl_eval_batch_host: zero-copy pinned staging at this size) and serves the
// remaining callbacks of that x from the cached results, so IPOPT's eval_f / eval_grad_f /
// eval_g / eval_jac_g sequence costs one launch per iterate.  A maintainer's Ipopt::TNLP
// subclass forwards to these one-to-one.
class CplTNLP {
 public:
  explicit CplTNLP(CplProblem::Ptr problem, int device = -1);
  ~CplTNLP();
  CplTNLP(const CplTNLP&) = delete;
  CplTNLP& operator=(const CplTNLP&) = delete;

  bool get_nlp_info(int32_t& n, int32_t& m, int32_t& nnz_jac_g, int32_t& nnz_h_lag) const;
  bool get_bounds_info(int32_t n, double* x_l, double* x_u, int32_t m, double* g_l, double* g_u) const;
  bool get_starting_point(int32_t n, bool init_x, double* x) const;
  bool eval_f(int32_t n, const double* x, bool new_x, double& obj_value);
  bool eval_grad_f(int32_t n, const double* x, bool new_x, double* grad_f);
  bool eval_g(int32_t n, const double* x, bool new_x, int32_t m, double* g);
  bool eval_jac_g(int32_t n, const double* x, bool new_x, int32_t m, int32_t nele_jac, int32_t* iRow,
                  int32_t* jCol, double* values);
  void finalize_solution(int32_t n, const double* x);  // saves x into the problem's variables

  int64_t launches() const { return _launches; }
  const CplProblem::Ptr& problem() const { return _problem; }

 private:
  bool Evaluate(const double* x, bool new_x);

  CplProblem::Ptr _problem;
  std::vector<double> _hbuf;  // x | g | jac | f | grad of the cached iterate (host)
  std::vector<double> _x_cached;
  bool _valid = false;
  int64_t _launches = 0;
};

}  // namespace solver
}  // namespace cpl
