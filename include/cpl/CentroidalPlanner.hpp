// cpl/CentroidalPlanner.hpp — host facade of the MI355X engine.
//
// Mirrors include/CentroidalPlanner/CentroidalPlanner.h and CoMPlanner.h of the reference (same
// public methods, argument meaning, validation and exception types; src/CentroidalPlanner.cpp,
// src/CoMPlanner.cpp).  The reference's solver member is an ifopt::IpoptSolver
// (CentroidalPlanner.h:232); IPOPT is not part of this build, so the solver is the NlpSolver
// interface below: any NLP solver that drives a CplTNLP (an Ipopt::TNLP forwarding adapter, see
// INTEGRATION.md §1, or a built-in driver).  Solve() without an attached solver throws
// std::runtime_error.
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
