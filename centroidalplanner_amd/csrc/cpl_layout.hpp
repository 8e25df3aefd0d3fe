// cpl_layout.hpp — the IFOPT layout contract of one CentroidalPlanner instance, shared by the
// host C-ABI (structure / bounds export) and the kernel launcher.
//
// Reference: variable order src/CplProblem.cpp:17-34 (CoM, then F_i p_i n_i in contact_names
// order); constraint order src/CplProblem.cpp:37-75 (statics, then per contact in std::map order
// env / normal / cone, or cone alone without environment); block shapes from the constraint sets'
// FillJacobianBlock (src/Constraints/*.cpp) as assembled by IFOPT into RowMajor CSR.
#pragma once

#include <cstdint>

#include "../../include/cpl_mi355x.h"

namespace cpl {

inline bool has_env(int32_t env_kind) {
  return env_kind == CPL_ENV_GROUND || env_kind == CPL_ENV_SUPERQUADRIC || env_kind == CPL_ENV_MIXED;
}

struct Dims {
  int32_t N, n, m, nnz;
  int32_t statics_nnz;      // 6 + 15N
  int32_t contact_rows;     // 6 (env) or 2
  int32_t contact_nnz;      // 27 (env) or 12
};

inline Dims dims_of(int32_t N, int32_t env_kind) {
  Dims d;
  d.N = N;
  d.n = 3 + 9 * N;
  const bool e = has_env(env_kind);
  d.contact_rows = e ? 6 : 2;
  d.contact_nnz = e ? 27 : 12;
  d.statics_nnz = 6 + 15 * N;
  d.m = 6 + d.contact_rows * N;
  d.nnz = d.statics_nnz + d.contact_nnz * N;
  return d;
}

// Values-only ("folded") Jacobian layout (cpl_eval_batch_ex, CPL_EVAL_JAC_FOLDED): the entries that
// are constant for every x are skipped in the output record, row-major order otherwise kept.
//   FOLD_COMMON (every environment kind but Ground): the I3 blocks of the force-balance rows
//     (src/Constraints/CentroidalStatics.cpp:93-95) and the n_r entry (1) of each normal row
//     (src/Constraints/EnvironmentNormal.cpp:63-70);
//   FOLD_GROUND: also the Ground gradient (0, 0, 1) (src/Ground.cpp:30-35) and the zero normal
//     Jacobian (src/Ground.cpp:46-50) — per contact only the 12 friction-cone entries remain.
enum { FOLD_NONE = 0, FOLD_COMMON = 1, FOLD_GROUND = 2 };

inline int32_t fold_level(int32_t env_kind) { return env_kind == CPL_ENV_GROUND ? FOLD_GROUND : FOLD_COMMON; }

// per-contact entries of a folded record: cone 12, + env 3 + normal 9 (p blocks) with a surface
inline int32_t folded_contact_nnz(int32_t env_kind) {
  if (env_kind == CPL_ENV_GROUND || !has_env(env_kind)) return 12;
  return 24;
}
inline int32_t folded_nnz(int32_t N, int32_t env_kind) { return 6 + 12 * N + folded_contact_nnz(env_kind) * N; }

// Column of component c of a variable set.
inline int32_t col_com(int32_t c) { return c; }
inline int32_t col_F(int32_t i, int32_t c) { return 3 + 9 * i + c; }
inline int32_t col_p(int32_t i, int32_t c) { return 6 + 9 * i + c; }
inline int32_t col_n(int32_t i, int32_t c) { return 9 + 9 * i + c; }

}  // namespace cpl
