// Host facade: cpl::CentroidalPlanner and cpl::CoMPlanner over the MI355X engine.
// Reference: src/CentroidalPlanner.cpp, src/CoMPlanner.cpp (line numbers cited per method).
#include <algorithm>
#include <stdexcept>

#include "cpl/CentroidalPlanner.hpp"

namespace cpl {

// src/CentroidalPlanner.cpp:5-20
CentroidalPlanner::CentroidalPlanner(std::vector<std::string> contact_names, double robot_mass,
                                     env::EnvironmentClass::Ptr env)
    : _contact_names(std::move(contact_names)), _robot_mass(robot_mass), _env(std::move(env)) {
  if (robot_mass <= 0.0) throw std::invalid_argument("Invalid robot mass");
  _cpl_problem = std::make_shared<solver::CplProblem>(_contact_names, _robot_mass, _env);
}

// src/CentroidalPlanner.cpp:22-34: solve, then read the solution out of the persistent variables
// (the default solver, like the reference's ifopt::IpoptSolver member, is created with the planner's
// first Solve: the native engine with IFOPT's defaults)
solver::Solution CentroidalPlanner::Solve() {
  if (!_cpl_solver) _cpl_solver = std::make_shared<solver::NativeSolver>();
  solver::CplTNLP nlp(_cpl_problem);
  _last_ok = _cpl_solver->Solve(nlp);
  solver::Solution sol;
  _cpl_problem->GetSolution(sol);
  return sol;
}

bool CentroidalPlanner::HasContact(const std::string& c) const {  // :359-370
  return std::find(_contact_names.begin(), _contact_names.end(), c) != _contact_names.end();
}

void CentroidalPlanner::CheckContact(const std::string& c) const {
  if (!HasContact(c)) throw std::invalid_argument("Invalid contact name: '" + c + "'");
}

static void check_weight(double w) {
  if (w < 0.0) throw std::invalid_argument("Invalid weight");
}

void CentroidalPlanner::SetForceBounds(std::string c, const Vector3d& lb, const Vector3d& ub) {  // :37-48
  CheckContact(c);
  _cpl_problem->SetForceBounds(c, lb, ub);
}
void CentroidalPlanner::GetForceBounds(std::string c, Vector3d& lb, Vector3d& ub) const {
  CheckContact(c);
  _cpl_problem->GetForceBounds(c, lb, ub);
}
void CentroidalPlanner::SetPosBounds(std::string c, const Vector3d& lb, const Vector3d& ub) {
  CheckContact(c);
  _cpl_problem->SetPosBounds(c, lb, ub);
}
void CentroidalPlanner::GetPosBounds(std::string c, Vector3d& lb, Vector3d& ub) const {
  CheckContact(c);
  _cpl_problem->GetPosBounds(c, lb, ub);
}
void CentroidalPlanner::SetNormalBounds(std::string c, const Vector3d& lb, const Vector3d& ub) {
  CheckContact(c);
  _cpl_problem->SetNormalBounds(c, lb, ub);
}
void CentroidalPlanner::GetNormalBounds(std::string c, Vector3d& lb, Vector3d& ub) const {
  CheckContact(c);
  _cpl_problem->GetNormalBounds(c, lb, ub);
}

void CentroidalPlanner::SetPosRef(std::string c, const Vector3d& r) {
  CheckContact(c);
  _cpl_problem->SetPosRef(c, r);
}
Vector3d CentroidalPlanner::GetPosRef(std::string c) const {
  CheckContact(c);
  return _cpl_problem->GetPosRef(c);
}
void CentroidalPlanner::SetForceRef(std::string c, const Vector3d& r) {
  CheckContact(c);
  _cpl_problem->SetForceRef(c, r);
}
Vector3d CentroidalPlanner::GetForceRef(std::string c) const {
  CheckContact(c);
  return _cpl_problem->GetForceRef(c);
}
void CentroidalPlanner::SetCoMRef(const Vector3d& r) { _cpl_problem->SetCoMRef(r); }
Vector3d CentroidalPlanner::GetCoMRef() const { return _cpl_problem->GetCoMRef(); }

void CentroidalPlanner::SetCoMWeight(double w) {
  check_weight(w);
  _cpl_problem->SetCoMWeight(w);
}
double CentroidalPlanner::GetCoMWeight() const { return _cpl_problem->GetCoMWeight(); }
void CentroidalPlanner::SetPosWeight(double w) {
  check_weight(w);
  _cpl_problem->SetPosWeight(w);
}
std::map<std::string, double> CentroidalPlanner::GetPosWeight() const {
  std::map<std::string, double> out;
  for (const auto& c : _contact_names) out[c] = _cpl_problem->GetContactPosWeight(c);
  return out;
}
void CentroidalPlanner::SetContactPosWeight(std::string c, double w) {
  CheckContact(c);
  check_weight(w);
  _cpl_problem->SetContactPosWeight(c, w);
}
double CentroidalPlanner::GetContactPosWeight(std::string c) const {
  CheckContact(c);
  return _cpl_problem->GetContactPosWeight(c);
}
void CentroidalPlanner::SetForceWeight(double w) {
  check_weight(w);
  _cpl_problem->SetForceWeight(w);
}
std::map<std::string, double> CentroidalPlanner::GetForceWeight() const {
  std::map<std::string, double> out;
  for (const auto& c : _contact_names) out[c] = _cpl_problem->GetContactForceWeight(c);
  return out;
}
void CentroidalPlanner::SetContactForceWeight(std::string c, double w) {
  CheckContact(c);
  check_weight(w);
  _cpl_problem->SetContactForceWeight(c, w);
}
double CentroidalPlanner::GetContactForceWeight(std::string c) const {
  CheckContact(c);
  return _cpl_problem->GetContactForceWeight(c);
}

void CentroidalPlanner::SetManipulationWrench(const VectorXd& w) { _cpl_problem->SetManipulationWrench(w); }
VectorXd CentroidalPlanner::GetManipulationWrench() const { return _cpl_problem->GetManipulationWrench(); }
double CentroidalPlanner::GetMu() const { return _cpl_problem->GetMu(); }

// src/CentroidalPlanner.cpp:324-346: the threshold is only applied to a contact whose force bounds
// are not both zero (Eigen operator!= : any coefficient differs)
void CentroidalPlanner::SetForceThreshold(std::string c, double F_thr) {
  CheckContact(c);
  if (F_thr < 0.0) throw std::invalid_argument("Invalid force threshold");
  Vector3d lb, ub;
  _cpl_problem->GetForceBounds(c, lb, ub);
  const Vector3d zero{0.0, 0.0, 0.0};
  if (lb != zero && ub != zero) _cpl_problem->SetForceThreshold(c, F_thr);
}
double CentroidalPlanner::GetForceThreshold(std::string c) const {
  CheckContact(c);
  return _cpl_problem->GetForceThreshold(c);
}

// ------------------------------------------------------------------------------------------------
// CoMPlanner (src/CoMPlanner.cpp)
// ------------------------------------------------------------------------------------------------
CoMPlanner::CoMPlanner(std::vector<std::string> contact_names, double robot_mass)  // :5-24
    : CentroidalPlanner(contact_names, robot_mass, nullptr), _contact_names(contact_names) {
  SetPosWeight(0.0);
  SetForceWeight(0.0);
  for (const auto& c : _contact_names) {
    SetContactNormal(c, {0.0, 0.0, 1.0});
    _F_thr_map[c] = GetForceThreshold(c);
  }
}

void CoMPlanner::SetLiftingContact(std::string c) {  // :27-37
  _F_thr_map[c] = GetForceThreshold(c);
  SetForceThreshold(c, 0.0);
  SetForceBounds(c, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0});
}

std::vector<std::string> CoMPlanner::GetLiftingContacts() const {  // :40-56
  std::vector<std::string> out;
  const Vector3d zero{0.0, 0.0, 0.0};
  for (const auto& c : _contact_names) {
    Vector3d lb, ub;
    GetForceBounds(c, lb, ub);
    if (lb == zero && ub == zero) out.push_back(c);
  }
  return out;
}

bool CoMPlanner::IsLiftingContact(const std::string& c) const {  // :59-71
  const auto l = GetLiftingContacts();
  return std::find(l.begin(), l.end(), c) != l.end();
}

void CoMPlanner::ResetLiftingContact(std::string c) {  // :74-88
  if (!IsLiftingContact(c)) throw std::runtime_error("'" + c + "' is not a lifting contact.");
  SetForceBounds(c, {-1e3, -1e3, -1e3}, {1e3, 1e3, 1e3});
  SetForceThreshold(c, _F_thr_map.at(c));
}

void CoMPlanner::SetContactPosition(std::string c, const Vector3d& pos_ref) {  // :91-97
  SetPosBounds(c, pos_ref, pos_ref);
}

Vector3d CoMPlanner::GetContactPosition(std::string c) const {  // :100-111
  Vector3d lb, ub;
  GetPosBounds(c, lb, ub);
  if (lb != ub) throw std::runtime_error("Contact position for '" + c + "' not set");
  return lb;
}

void CoMPlanner::SetContactNormal(std::string c, const Vector3d& n_ref) {  // :114-129
  if (!HasContact(c)) throw std::invalid_argument("Invalid contact name: '" + c + "'");
  SetNormalBounds(c, n_ref, n_ref);
}

Vector3d CoMPlanner::GetContactNormal(std::string c) const {  // :132-143
  Vector3d lb, ub;
  GetNormalBounds(c, lb, ub);
  if (lb != ub) throw std::runtime_error("Contact normal for '" + c + "' not set");
  return lb;
}

void CoMPlanner::SetMu(double mu) {  // :146-156
  if (mu <= 0.0) throw std::invalid_argument("Invalid friction coefficient");
  GetCplProblem()->SetMu(mu);
}

}  // namespace cpl
