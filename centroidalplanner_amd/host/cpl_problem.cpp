// Host problem template, solution printing and the TNLP hooks over the C-ABI.
// Reference: src/CplProblem.cpp, include/CentroidalPlanner/Ifopt/CplProblem.h, Types.h;
// IFOPT IpoptAdapter [IFOPT-ext] for the TNLP argument conventions.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "cpl/CplProblem.hpp"

namespace cpl {

void ThrowOnError(int32_t status) {
  if (status == CPL_OK) return;
  const std::string msg = cpl_last_error();
  switch (status) {
    case CPL_ERR_INVALID_ARGUMENT: throw std::invalid_argument(msg);
    case CPL_ERR_OUT_OF_RANGE: throw std::out_of_range(msg);
    default: throw std::runtime_error(std::string(cpl_status_string(status)) + ": " + msg);
  }
}

namespace env {
void Superquadric::SetParameters(const Vector3d& C, const Vector3d& R, const Vector3d& P) {
  // the validation lives in the C-ABI setter (same messages as src/Superquadric.cpp:16-24)
  cpl_problem_desc probe;
  ThrowOnError(cpl_desc_init(&probe, 1, CPL_ENV_SUPERQUADRIC, 1.0));
  ThrowOnError(cpl_desc_set_superquadric(&probe, C.data(), R.data(), P.data()));
  _C = C;
  _R = R;
  _P = P;
}

void Superquadric::FillDesc(cpl_problem_desc& d) const {
  EnvironmentClass::FillDesc(d);
  for (int j = 0; j < 3; ++j) {
    d.sq_C[j] = _C[j];
    d.sq_R[j] = _R[j];
    d.sq_P[j] = _P[j];
  }
}
}  // namespace env

namespace solver {

namespace {
void put_row(std::ostream& os, const Vector3d& v) {
  // Eigen's transpose() printing of a 3-vector: default IOFormat, precision 6, space separated
  std::ios_base::fmtflags f = os.flags();
  std::streamsize p = os.precision(6);
  for (int j = 0; j < 3; ++j) {
    if (j) os << ' ';
    os << v[j];
  }
  os.precision(p);
  os.flags(f);
}
}  // namespace

std::ostream& operator<<(std::ostream& os, const Solution& sol) {
  os << "CoM: ";
  put_row(os, sol.com_sol);
  os << "\n";
  for (const auto& e : sol.contact_values_map) { os << "F_" + e.first + ": "; put_row(os, e.second.force_value); os << "\n"; }
  for (const auto& e : sol.contact_values_map) { os << "p_" + e.first + ": "; put_row(os, e.second.position_value); os << "\n"; }
  for (const auto& e : sol.contact_values_map) { os << "n_" + e.first + ": "; put_row(os, e.second.normal_value); os << "\n"; }
  return os;
}

// src/CplProblem.cpp:6-82
CplProblem::CplProblem(std::vector<std::string> contact_names, double robot_mass, env::EnvironmentClass::Ptr env)
    : _contact_names(std::move(contact_names)), _env(std::move(env)), _ground_fake(std::make_shared<env::Ground>()) {
  const int32_t N = (int32_t)_contact_names.size();
  ThrowOnError(cpl_desc_init(&_desc, N, _env ? _env->Kind() : CPL_ENV_NONE, robot_mass));
  std::vector<const char*> names(N);
  for (int32_t i = 0; i < N; ++i) {
    names[i] = _contact_names[i].c_str();
    _index[_contact_names[i]] = i;
  }
  ThrowOnError(cpl_desc_set_contact_names(&_desc, names.data(), N));
  ThrowOnError(cpl_dims(&_desc, &_n, &_m, &_nnz));
  _x.assign(_n, 0.0);  // Variable3D init 0 (src/Variable3D.cpp:8-10)
}

int32_t CplProblem::Index(const std::string& contact_name) const {
  auto it = _index.find(contact_name);
  if (it == _index.end()) throw std::out_of_range("map::at");  // std::map::at
  return it->second;
}

const cpl_problem_desc& CplProblem::Desc() const {
  if (_env)
    _env->FillDesc(_desc);
  else
    _desc.mu = _ground_fake->GetMu();
  return _desc;
}

void CplProblem::SetVariables(const VectorXd& x) {
  if ((int32_t)x.size() != _n) throw std::invalid_argument("variable vector has the wrong size");
  _x = x;
}

// src/CplProblem.cpp:84-106, contacts in std::map (name) order
void CplProblem::GetSolution(Solution& sol) const {
  sol.com_sol = {_x[0], _x[1], _x[2]};
  sol.contact_values_map.clear();
  for (const auto& e : _index) {
    const int32_t b = 3 + 9 * e.second;
    ContactValues cv;
    cv.force_value = {_x[b], _x[b + 1], _x[b + 2]};
    cv.position_value = {_x[b + 3], _x[b + 4], _x[b + 5]};
    cv.normal_value = {_x[b + 6], _x[b + 7], _x[b + 8]};
    sol.contact_values_map[e.first] = cv;
  }
}

void CplProblem::SetBounds(int32_t var, const std::string& contact_name, const Vector3d& lb, const Vector3d& ub) {
  ThrowOnError(cpl_desc_set_bounds(&_desc, var, Index(contact_name), lb.data(), ub.data()));
}

#define CPL_GET3(arr, i) Vector3d{arr[i][0], arr[i][1], arr[i][2]}

void CplProblem::SetForceBounds(std::string c, const Vector3d& lb, const Vector3d& ub) { SetBounds(1, c, lb, ub); }
void CplProblem::GetForceBounds(std::string c, Vector3d& lb, Vector3d& ub) const {
  const int32_t i = Index(c);
  lb = CPL_GET3(_desc.F_lb, i);
  ub = CPL_GET3(_desc.F_ub, i);
}
void CplProblem::SetPosBounds(std::string c, const Vector3d& lb, const Vector3d& ub) { SetBounds(2, c, lb, ub); }
void CplProblem::GetPosBounds(std::string c, Vector3d& lb, Vector3d& ub) const {
  const int32_t i = Index(c);
  lb = CPL_GET3(_desc.p_lb, i);
  ub = CPL_GET3(_desc.p_ub, i);
}
void CplProblem::SetNormalBounds(std::string c, const Vector3d& lb, const Vector3d& ub) { SetBounds(3, c, lb, ub); }
void CplProblem::GetNormalBounds(std::string c, Vector3d& lb, Vector3d& ub) const {
  const int32_t i = Index(c);
  lb = CPL_GET3(_desc.n_lb, i);
  ub = CPL_GET3(_desc.n_ub, i);
}

void CplProblem::SetPosRef(std::string c, const Vector3d& r) {
  const int32_t i = Index(c);
  for (int j = 0; j < 3; ++j) _desc.p_ref[i][j] = r[j];
}
Vector3d CplProblem::GetPosRef(std::string c) const { return CPL_GET3(_desc.p_ref, Index(c)); }
void CplProblem::SetForceRef(std::string c, const Vector3d& r) {
  const int32_t i = Index(c);
  for (int j = 0; j < 3; ++j) _desc.F_ref[i][j] = r[j];
}
Vector3d CplProblem::GetForceRef(std::string c) const { return CPL_GET3(_desc.F_ref, Index(c)); }
void CplProblem::SetCoMRef(const Vector3d& r) {
  for (int j = 0; j < 3; ++j) _desc.com_ref[j] = r[j];
}
Vector3d CplProblem::GetCoMRef() const { return {_desc.com_ref[0], _desc.com_ref[1], _desc.com_ref[2]}; }

#undef CPL_GET3

void CplProblem::SetCoMWeight(double w) { _desc.W_com = w; }
double CplProblem::GetCoMWeight() const { return _desc.W_com; }
void CplProblem::SetPosWeight(double w) {
  for (size_t i = 0; i < _contact_names.size(); ++i) _desc.W_p[i] = w;
}
void CplProblem::SetContactPosWeight(std::string c, double w) { _desc.W_p[Index(c)] = w; }
double CplProblem::GetContactPosWeight(std::string c) const { return _desc.W_p[Index(c)]; }
void CplProblem::SetForceWeight(double w) {
  for (size_t i = 0; i < _contact_names.size(); ++i) _desc.W_F[i] = w;
}
void CplProblem::SetContactForceWeight(std::string c, double w) { _desc.W_F[Index(c)] = w; }
double CplProblem::GetContactForceWeight(std::string c) const { return _desc.W_F[Index(c)]; }

void CplProblem::SetManipulationWrench(const VectorXd& w) {
  if (w.size() != 6) throw std::invalid_argument("manipulation wrench must have 6 entries");
  for (int j = 0; j < 6; ++j) _desc.wrench[j] = w[j];
}
VectorXd CplProblem::GetManipulationWrench() const { return VectorXd(_desc.wrench, _desc.wrench + 6); }

// src/CplProblem.cpp:275-301
void CplProblem::SetMu(double mu) {
  if (_env)
    _env->SetMu(mu);
  else
    _ground_fake->SetMu(mu);
}
double CplProblem::GetMu() const { return _env ? _env->GetMu() : _ground_fake->GetMu(); }

void CplProblem::SetForceThreshold(std::string c, double F_thr) { _desc.F_thr[Index(c)] = F_thr; }
double CplProblem::GetForceThreshold(std::string c) const { return _desc.F_thr[Index(c)]; }

// ------------------------------------------------------------------------------------------------
// TNLP hooks
// ------------------------------------------------------------------------------------------------
namespace {
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

CplTNLP::CplTNLP(CplProblem::Ptr problem, int device) : _problem(std::move(problem)) {
  if (!_problem) throw std::invalid_argument("CplTNLP needs a problem");
  if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
  _hbuf.assign((size_t)(_problem->n() + _problem->m() + _problem->nnz() + 1 + _problem->n()), 0.0);
}

CplTNLP::~CplTNLP() = default;

bool CplTNLP::get_nlp_info(int32_t& n, int32_t& m, int32_t& nnz_jac_g, int32_t& nnz_h_lag) const {
  n = _problem->n();
  m = _problem->m();
  nnz_jac_g = _problem->nnz();
  nnz_h_lag = n * n;  // IFOPT reports a dense Hessian structure and uses limited-memory updates
  return true;
}

bool CplTNLP::get_bounds_info(int32_t n, double* x_l, double* x_u, int32_t m, double* g_l, double* g_u) const {
  if (n != _problem->n() || m != _problem->m()) return false;
  return cpl_bounds(&_problem->Desc(), x_l, x_u, g_l, g_u) == CPL_OK;
}

bool CplTNLP::get_starting_point(int32_t n, bool init_x, double* x) const {
  if (n != _problem->n()) return false;
  if (init_x) std::copy(_problem->GetVariables().begin(), _problem->GetVariables().end(), x);
  return true;
}

// one fused launch for every output of x; later callbacks of the same x read the cache
bool CplTNLP::Evaluate(const double* x, bool new_x) {
  const int32_t n = _problem->n(), m = _problem->m(), nnz = _problem->nnz();
  if (!new_x && _valid && std::equal(_x_cached.begin(), _x_cached.end(), x)) return true;
  double* g = _hbuf.data() + n;
  double* jac = g + m;
  double* f = jac + nnz;
  double* grad = f + 1;
  std::copy(x, x + n, _hbuf.data());
  if (cpl_eval_batch_host(&_problem->Desc(), 1, _hbuf.data(), nullptr, nullptr, g, jac, f, grad, nullptr, 0) != CPL_OK)
    return false;
  _x_cached.assign(x, x + n);
  _valid = true;
  ++_launches;
  return true;
}

bool CplTNLP::eval_f(int32_t n, const double* x, bool new_x, double& obj_value) {
  if (n != _problem->n() || !Evaluate(x, new_x)) return false;
  obj_value = _hbuf[n + _problem->m() + _problem->nnz()];
  return true;
}

bool CplTNLP::eval_grad_f(int32_t n, const double* x, bool new_x, double* grad_f) {
  if (n != _problem->n() || !Evaluate(x, new_x)) return false;
  const double* src = _hbuf.data() + n + _problem->m() + _problem->nnz() + 1;
  std::copy(src, src + n, grad_f);
  return true;
}

bool CplTNLP::eval_g(int32_t n, const double* x, bool new_x, int32_t m, double* g) {
  if (n != _problem->n() || m != _problem->m() || !Evaluate(x, new_x)) return false;
  std::copy(_hbuf.data() + n, _hbuf.data() + n + m, g);
  return true;
}

bool CplTNLP::eval_jac_g(int32_t n, const double* x, bool new_x, int32_t m, int32_t nele_jac, int32_t* iRow,
                         int32_t* jCol, double* values) {
  if (n != _problem->n() || m != _problem->m() || nele_jac != _problem->nnz()) return false;
  if (!values) return cpl_structure(&_problem->Desc(), iRow, jCol, nullptr) == CPL_OK;
  if (!Evaluate(x, new_x)) return false;
  const double* src = _hbuf.data() + n + m;
  std::copy(src, src + nele_jac, values);
  return true;
}

void CplTNLP::finalize_solution(int32_t n, const double* x) {
  if (n == _problem->n()) _problem->SetVariables(VectorXd(x, x + n));
}

}  // namespace solver
}  // namespace cpl
