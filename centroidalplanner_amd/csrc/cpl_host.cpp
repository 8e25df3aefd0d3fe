// cpl_host.cpp — host half of the C-ABI: problem template defaults and validating setters,
// problem dimensions, Jacobian structure and bounds export (the IPOPT TNLP metadata hooks).
// Nothing here evaluates the hot path; that lives in cpl_kernels.hip.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "cpl_layout.hpp"
#include "cpl_status.hpp"

namespace cpl {

thread_local std::string g_last_error;

int32_t fail(int32_t status, const std::string& msg) {
  g_last_error = msg;
  return status;
}

int32_t validate_desc(const cpl_problem_desc* d) {
  if (!d) return fail(CPL_ERR_INVALID_ARGUMENT, "null problem descriptor");
  if (d->abi_version != CPL_ABI_VERSION)
    return fail(CPL_ERR_INVALID_ARGUMENT, "problem descriptor ABI version mismatch");
  if (d->n_contacts < 1 || d->n_contacts > CPL_MAX_CONTACTS)
    return fail(CPL_ERR_INVALID_ARGUMENT, "n_contacts out of range [1, CPL_MAX_CONTACTS]");
  if (d->env_kind < CPL_ENV_NONE || d->env_kind > CPL_ENV_MIXED)
    return fail(CPL_ERR_INVALID_ARGUMENT, "unknown environment kind");
  // map_order must be a permutation of 0..N-1
  bool seen[CPL_MAX_CONTACTS] = {false};
  for (int32_t k = 0; k < d->n_contacts; ++k) {
    int32_t i = d->map_order[k];
    if (i < 0 || i >= d->n_contacts || seen[i])
      return fail(CPL_ERR_INVALID_ARGUMENT, "map_order is not a permutation of the contacts");
    seen[i] = true;
  }
  return CPL_OK;
}

}  // namespace cpl

using namespace cpl;

extern "C" {

int32_t cpl_abi_version(void) { return CPL_ABI_VERSION; }
size_t cpl_desc_sizeof(void) { return sizeof(cpl_problem_desc); }
const char* cpl_last_error(void) { return g_last_error.c_str(); }

const char* cpl_status_string(int32_t status) {
  switch (status) {
    case CPL_OK: return "ok";
    case CPL_ERR_INVALID_ARGUMENT: return "invalid argument";
    case CPL_ERR_OUT_OF_RANGE: return "out of range";
    case CPL_ERR_RUNTIME: return "runtime error";
    case CPL_ERR_HIP: return "HIP error";
    case CPL_ERR_UNSUPPORTED: return "unsupported";
    default: return "unknown status";
  }
}

// Defaults of the reference constructors: CentroidalStatics (m, g, wrench)
// src/Constraints/CentroidalStatics.cpp:5-17; FrictionCone F_thr=0 src/Constraints/FrictionCone.cpp:14;
// EnvironmentClass mu=1 Environment.h:46; Ground z=0 src/Ground.cpp:5-8; Superquadric
// src/Superquadric.cpp:5-10; MinimizeCentroidalVariables src/MinimizeCentroidalVariables.cpp:5-27;
// Variable3D bounds src/Variable3D.cpp:5-15.  Mass check: src/CentroidalPlanner.cpp:12-15.
int32_t cpl_desc_init(cpl_problem_desc* d, int32_t n_contacts, int32_t env_kind, double mass) {
  if (!d) return fail(CPL_ERR_INVALID_ARGUMENT, "null problem descriptor");
  if (n_contacts < 1 || n_contacts > CPL_MAX_CONTACTS)
    return fail(CPL_ERR_INVALID_ARGUMENT, "n_contacts out of range [1, CPL_MAX_CONTACTS]");
  if (env_kind < CPL_ENV_NONE || env_kind > CPL_ENV_MIXED)
    return fail(CPL_ERR_INVALID_ARGUMENT, "unknown environment kind");
  if (!(mass > 0.0)) return fail(CPL_ERR_INVALID_ARGUMENT, "Invalid robot mass");
  std::memset(d, 0, sizeof(*d));
  d->abi_version = CPL_ABI_VERSION;
  d->n_contacts = n_contacts;
  d->env_kind = env_kind;
  d->mass = mass;
  d->gravity[0] = 0.0;
  d->gravity[1] = 0.0;
  d->gravity[2] = -9.81;
  d->mu = 1.0;
  d->ground_z = 0.0;
  d->sq_C[0] = 0.0; d->sq_C[1] = 0.0; d->sq_C[2] = 10.0;
  for (int j = 0; j < 3; ++j) { d->sq_R[j] = 10.0; d->sq_P[j] = 10.0; }
  d->W_com = 1.0;
  d->com_ref[0] = 0.0; d->com_ref[1] = 0.0; d->com_ref[2] = 1.0;
  for (int j = 0; j < 3; ++j) { d->com_lb[j] = -1000.0; d->com_ub[j] = 1000.0; }
  for (int i = 0; i < CPL_MAX_CONTACTS; ++i) {
    d->W_p[i] = 1.0;
    d->W_F[i] = 1.0;
    for (int j = 0; j < 3; ++j) {
      d->F_lb[i][j] = d->p_lb[i][j] = d->n_lb[i][j] = -1000.0;
      d->F_ub[i][j] = d->p_ub[i][j] = d->n_ub[i][j] = 1000.0;
    }
  }
  // names "contact1".."contactN": map order is lexicographic over those names
  std::vector<std::string> names;
  for (int32_t i = 0; i < n_contacts; ++i) names.push_back("contact" + std::to_string(i + 1));
  std::vector<const char*> ptrs;
  for (auto& s : names) ptrs.push_back(s.c_str());
  return cpl_desc_set_contact_names(d, ptrs.data(), n_contacts);
}

// std::map<std::string, ContactVars> iterates in std::string operator< order (byte-wise);
// CplProblem builds its constraint sets in that order (src/CplProblem.cpp:42).
int32_t cpl_desc_set_contact_names(cpl_problem_desc* d, const char* const* names, int32_t n) {
  if (!d || !names) return fail(CPL_ERR_INVALID_ARGUMENT, "null argument");
  if (n != d->n_contacts) return fail(CPL_ERR_INVALID_ARGUMENT, "name count differs from n_contacts");
  std::vector<std::string> v;
  for (int32_t i = 0; i < n; ++i) {
    if (!names[i] || !names[i][0]) return fail(CPL_ERR_INVALID_ARGUMENT, "empty contact name");
    v.emplace_back(names[i]);
  }
  std::vector<int32_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return v[a] < v[b]; });
  for (int32_t k = 1; k < n; ++k)
    if (v[idx[k]] == v[idx[k - 1]])
      return fail(CPL_ERR_INVALID_ARGUMENT, "duplicate contact name: '" + v[idx[k]] + "'");
  for (int32_t k = 0; k < n; ++k) d->map_order[k] = idx[k];
  for (int32_t k = n; k < CPL_MAX_CONTACTS; ++k) d->map_order[k] = 0;
  return CPL_OK;
}

// EnvironmentClass::SetMu, include/CentroidalPlanner/Environment/Environment.h:19-26
int32_t cpl_desc_set_mu(cpl_problem_desc* d, double mu) {
  if (!d) return fail(CPL_ERR_INVALID_ARGUMENT, "null problem descriptor");
  if (mu <= 0.0) return fail(CPL_ERR_INVALID_ARGUMENT, "Invalid friction coefficient");
  d->mu = mu;
  return CPL_OK;
}

// Superquadric::SetParameters, src/Superquadric.cpp:12-29
int32_t cpl_desc_set_superquadric(cpl_problem_desc* d, const double C[3], const double R[3], const double P[3]) {
  if (!d || !C || !R || !P) return fail(CPL_ERR_INVALID_ARGUMENT, "null argument");
  if (R[0] <= 0.0 || R[1] <= 0.0 || R[2] <= 0.0)
    return fail(CPL_ERR_INVALID_ARGUMENT, "Invalid superquadric axial radii");
  if (P[0] < 2.0 || P[1] < 2.0 || P[2] < 2.0)
    return fail(CPL_ERR_INVALID_ARGUMENT, "Invalid superquadric axial curvatures: must be >= 2");
  for (int j = 0; j < 3; ++j) { d->sq_C[j] = C[j]; d->sq_R[j] = R[j]; d->sq_P[j] = P[j]; }
  return CPL_OK;
}

// Variable3D::SetBounds, src/Variable3D.cpp:28-40 (the reference stores first, then throws;
// here nothing is stored on failure).
int32_t cpl_desc_set_bounds(cpl_problem_desc* d, int32_t var, int32_t contact, const double lb[3], const double ub[3]) {
  if (!d || !lb || !ub) return fail(CPL_ERR_INVALID_ARGUMENT, "null argument");
  if (var != 0 && (contact < 0 || contact >= d->n_contacts))
    return fail(CPL_ERR_OUT_OF_RANGE, "contact index out of range");
  for (int j = 0; j < 3; ++j)
    if (ub[j] - lb[j] < 0) return fail(CPL_ERR_INVALID_ARGUMENT, "Inconsistent bounds");
  double *L = nullptr, *U = nullptr;
  switch (var) {
    case 0: L = d->com_lb; U = d->com_ub; break;
    case 1: L = d->F_lb[contact]; U = d->F_ub[contact]; break;
    case 2: L = d->p_lb[contact]; U = d->p_ub[contact]; break;
    case 3: L = d->n_lb[contact]; U = d->n_ub[contact]; break;
    default: return fail(CPL_ERR_INVALID_ARGUMENT, "unknown variable set");
  }
  for (int j = 0; j < 3; ++j) { L[j] = lb[j]; U[j] = ub[j]; }
  return CPL_OK;
}

int32_t cpl_dims(const cpl_problem_desc* d, int32_t* n, int32_t* m, int32_t* nnz) {
  int32_t st = validate_desc(d);
  if (st) return st;
  Dims D = dims_of(d->n_contacts, d->env_kind);
  if (n) *n = D.n;
  if (m) *m = D.m;
  if (nnz) *nnz = D.nnz;
  return CPL_OK;
}

// RowMajor CSR structure, closed form of the blocks the constraint sets insert:
//  statics rows 0-2: I3 of every F_i (columns ascending = contact_names order);
//  statics rows 3-5: CoM's [F]x pattern, then per contact F_i's and p_i's cross-product pattern
//    (src/Constraints/CentroidalStatics.cpp:90-136);
//  per contact (map order): env row = p_i (EnvironmentConstraint.cpp:53-60); normal rows r =
//    p_i(3) + n_i[r] (EnvironmentNormal.cpp:63-85); cone rows = F_i(3) + n_i(3) (FrictionCone.cpp:79-101).
int32_t cpl_structure(const cpl_problem_desc* d, int32_t* iRow, int32_t* jCol, int32_t* row_ptr) {
  int32_t st = validate_desc(d);
  if (st) return st;
  const int32_t N = d->n_contacts;
  const bool env = has_env(d->env_kind);
  int32_t k = 0, row = 0;
  auto put = [&](int32_t r, int32_t c) {
    if (iRow) iRow[k] = r;
    if (jCol) jCol[k] = c;
    ++k;
  };
  auto end_row = [&]() {
    ++row;
    if (row_ptr) row_ptr[row] = k;
  };
  if (row_ptr) row_ptr[0] = 0;
  for (int32_t r = 0; r < 3; ++r) {
    for (int32_t i = 0; i < N; ++i) put(r, col_F(i, r));
    end_row();
  }
  // (row, first component, second component) of the skew-symmetric patterns
  static const int32_t skew[3][2] = {{1, 2}, {0, 2}, {0, 1}};
  for (int32_t r = 0; r < 3; ++r) {
    const int32_t a = skew[r][0], b = skew[r][1];
    put(3 + r, col_com(a));
    put(3 + r, col_com(b));
    for (int32_t i = 0; i < N; ++i) {
      put(3 + r, col_F(i, a));
      put(3 + r, col_F(i, b));
      put(3 + r, col_p(i, a));
      put(3 + r, col_p(i, b));
    }
    end_row();
  }
  for (int32_t kk = 0; kk < N; ++kk) {
    const int32_t i = d->map_order[kk];
    if (env) {
      for (int32_t c = 0; c < 3; ++c) put(row, col_p(i, c));
      end_row();
      for (int32_t r = 0; r < 3; ++r) {
        for (int32_t c = 0; c < 3; ++c) put(row, col_p(i, c));
        put(row, col_n(i, r));
        end_row();
      }
    }
    for (int32_t r = 0; r < 2; ++r) {
      for (int32_t c = 0; c < 3; ++c) put(row, col_F(i, c));
      for (int32_t c = 0; c < 3; ++c) put(row, col_n(i, c));
      end_row();
    }
  }
  return CPL_OK;
}

int32_t cpl_jac_fold_info(const cpl_problem_desc* d, int32_t* nnz_folded, int32_t* var_k, int32_t* n_const,
                          int32_t* const_k, double* const_val) {
  int32_t st = validate_desc(d);
  if (st) return st;
  const int32_t N = d->n_contacts;
  const bool env = has_env(d->env_kind);
  const int32_t lvl = fold_level(d->env_kind);
  // the walk of cpl_structure, each CSR position classified as variable or constant
  int32_t k = 0, nv = 0, nc = 0;
  auto var = [&](int32_t count) {
    for (int32_t e = 0; e < count; ++e) {
      if (var_k) var_k[nv] = k;
      ++nv;
      ++k;
    }
  };
  auto cst = [&](double v) {
    if (const_k) const_k[nc] = k;
    if (const_val) const_val[nc] = v;
    ++nc;
    ++k;
  };
  for (int32_t e = 0; e < 3 * N; ++e) cst(1.0);  // force balance: I3 per contact
  var(3 * (2 + 4 * N));                            // torque rows
  for (int32_t kk = 0; kk < N; ++kk) {
    if (env) {
      if (lvl == FOLD_GROUND) {  // Ground gradient (0, 0, 1) and zero normal Jacobian
        cst(0.0); cst(0.0); cst(1.0);
        for (int32_t r = 0; r < 3; ++r) { cst(0.0); cst(0.0); cst(0.0); cst(1.0); }
      } else {
        var(3);
        for (int32_t r = 0; r < 3; ++r) { var(3); cst(1.0); }
      }
    }
    var(12);  // friction cone
  }
  if (nv != folded_nnz(N, d->env_kind) || k != dims_of(N, d->env_kind).nnz)
    return fail(CPL_ERR_RUNTIME, "cpl_jac_fold_info: layout mismatch");
  if (nnz_folded) *nnz_folded = nv;
  if (n_const) *n_const = nc;
  return CPL_OK;
}

int32_t cpl_bounds(const cpl_problem_desc* d, double* x_l, double* x_u, double* g_l, double* g_u) {
  int32_t st = validate_desc(d);
  if (st) return st;
  const int32_t N = d->n_contacts;
  const Dims D = dims_of(N, d->env_kind);
  for (int32_t c = 0; c < 3; ++c) {
    if (x_l) x_l[col_com(c)] = d->com_lb[c];
    if (x_u) x_u[col_com(c)] = d->com_ub[c];
  }
  for (int32_t i = 0; i < N; ++i)
    for (int32_t c = 0; c < 3; ++c) {
      if (x_l) { x_l[col_F(i, c)] = d->F_lb[i][c]; x_l[col_p(i, c)] = d->p_lb[i][c]; x_l[col_n(i, c)] = d->n_lb[i][c]; }
      if (x_u) { x_u[col_F(i, c)] = d->F_ub[i][c]; x_u[col_p(i, c)] = d->p_ub[i][c]; x_u[col_n(i, c)] = d->n_ub[i][c]; }
    }
  for (int32_t r = 0; r < D.m; ++r) {
    bool cone = r >= 6 && ((r - 6) % D.contact_rows) >= D.contact_rows - 2;
    if (g_l) g_l[r] = cone ? -CPL_INF : 0.0;
    if (g_u) g_u[r] = 0.0;
  }
  return CPL_OK;
}

}  // extern "C"
