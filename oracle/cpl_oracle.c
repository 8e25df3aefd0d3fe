/*
 * cpl_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of CentroidalPlanner's IFOPT
 * evaluation path, used as the parity checker for the HIP kernels and as the bench's
 * `cpu_baseline` ("port").  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library; the product (centroidalplanner_amd) never does.
 *
 * What it restates (all paths relative to /root/reference):
 *   - the constraint sets' GetValues / FillJacobianBlock (src/Constraints/<Set>.cpp),
 *   - the cost term (src/MinimizeCentroidalVariables.cpp),
 *   - the environments (src/Ground.cpp, src/Superquadric.cpp),
 *   - the problem layout (src/CplProblem.cpp:6-82),
 *   - IFOPT's assembly [IFOPT-ext, not in the container]: every constraint set's
 *     FillJacobianBlock is called for EVERY variable set in AddVariableSet order (the block is
 *     cleared with setZero() first), stored entries (explicit zeros included) are shifted by the
 *     set's row / the variable set's column offset and assembled into a RowMajor sparse matrix,
 *     so IPOPT receives the values in row-major / column-ascending order.  Duplicates never
 *     occur on this path, so setFromTriplets' summing is not exercised.
 * The O(N^2) block walk of the reference (each set visits every variable set, the environment
 * Jacobians are recomputed on every visit) is kept on purpose: this is also the CPU baseline.
 *
 * Arithmetic contract (stated with the fixtures):
 *   - IEEE binary64, compiled with -O2 -ffp-contract=off (no FMA contraction);
 *   - Eigen 3.3 Vector3d semantics: dot / squaredNorm = (a0*b0 + a1*b1) + a2*b2 (SSE2 packet
 *     reduction of a 3-vector), norm = sqrt(squaredNorm), cross = Eigen's cross formula;
 *   - glibc pow (the reference calls <cmath> pow).
 *
 * Pinning: the reference cannot be built in this image (it needs Eigen3, IFOPT and IPOPT headers
 * and libraries, none present; building it against stand-in headers is not allowed), and its
 * own tests (tests/TestBasic.cpp) hold no golden vectors.  This oracle is therefore pinned at
 * SOLVE level by the four TestBasic scenarios and their invariants (tests/test_oracle_pinning.py
 * solves them through these callbacks), and at derivative level by central finite differences.
 * Value-level parity against the reference binary itself is UNPINNED.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/cpl_mi355x.h"

/* ---------------------------------------------------------------------------------------- */
/* Eigen 3.3 fixed-size 3-vector arithmetic as the reference sees it                         */
/* ---------------------------------------------------------------------------------------- */
#ifdef CPLO_EIGEN_REDUX_NOVEC
/* Eigen's reduction WITHOUT packet math for a 3-vector (a build without SSE2 vectorisation, or an AVX
 * build, whose 4-double packets are longer than a Vector3d): redux_novec_unroller splits the 3 terms
 * as 1 + 2, i.e. a0 b0 + (a1 b1 + a2 b2).  The reference's Eigen build is unpinned; this variant of the
 * oracle (oracle/_build/libcpl_oracle_novec.so) quantifies how far the two orders lie apart
 * (tests/test_eigen_order.py). */
static double edot(const double* a, const double* b) { return a[0] * b[0] + (a[1] * b[1] + a[2] * b[2]); }
static double esqn(const double* a) { return a[0] * a[0] + (a[1] * a[1] + a[2] * a[2]); }
#else
/* Eigen 3.3 on x86-64 with its default SSE2 packets (2 doubles): the packet (a0 b0, a1 b1) is
 * reduced first, then the tail a2 b2 is added: (a0 b0 + a1 b1) + a2 b2 */
static double edot(const double* a, const double* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static double esqn(const double* a) { return (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]; }
#endif
static double enorm(const double* a) { return sqrt(esqn(a)); }
/* Eigen MatrixBase::cross: (a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0) */
static void ecross(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

/* ---------------------------------------------------------------------------------------- */
/* Sparse block with Eigen SparseMatrix coeffRef semantics (find-or-insert, inserted at 0.0)  */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
  int n;
  int r[24], c[24];
  double v[24];
} blk_t;
static void blk_zero(blk_t* b) { b->n = 0; } /* SparseMatrix::setZero drops every stored entry */
static double* blk_ref(blk_t* b, int r, int c) {
  for (int k = 0; k < b->n; ++k)
    if (b->r[k] == r && b->c[k] == c) return &b->v[k];
  b->r[b->n] = r;
  b->c[b->n] = c;
  b->v[b->n] = 0.0;
  return &b->v[b->n++];
}

/* ---------------------------------------------------------------------------------------- */
/* Variables: x = [CoM | F_i p_i n_i for i in contact_names order]  (src/CplProblem.cpp:17-34) */
/* Variable3D::GetValues returns the 3 stored doubles (src/Variable3D.cpp:42-51).            */
/* ---------------------------------------------------------------------------------------- */
enum { VK_COM = 0, VK_F = 1, VK_P = 2, VK_N = 3 };
typedef struct { int kind, contact; } varset_t;
static varset_t varset_of(int v) { /* AddVariableSet order */
  varset_t s;
  if (v == 0) { s.kind = VK_COM; s.contact = -1; }
  else { s.kind = 1 + (v - 1) % 3; s.contact = (v - 1) / 3; }
  return s;
}
static const double* xcom(const double* x) { return x; }
static const double* xF(const double* x, int i) { return x + 3 + 9 * i; }
static const double* xp(const double* x, int i) { return x + 6 + 9 * i; }
static const double* xn(const double* x, int i) { return x + 9 + 9 * i; }

/* ---------------------------------------------------------------------------------------- */
/* Environments                                                                              */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
  int kind; /* CPL_ENV_GROUND / CPL_ENV_SUPERQUADRIC */
  double z;
  double C[3], R[3], P[3];
} env_t;

/* Ground::GetEnvironmentValue, src/Ground.cpp:23-27 (assigns: overwrites the caller's 0) */
/* Superquadric::GetEnvironmentValue, src/Superquadric.cpp:40-49 (accumulates with +=) */
static void env_value(const env_t* e, const double* p, double* val) {
  if (e->kind == CPL_ENV_GROUND) {
    *val = p[2] - e->z;
  } else {
    for (int i = 0; i < 3; ++i) *val += pow((p[i] - e->C[i]) / e->R[i], e->P[i]);
    *val -= 1.0;
  }
}
/* Ground::GetEnvironmentJacobian src/Ground.cpp:30-35; Superquadric src/Superquadric.cpp:51-57 */
static void env_jacobian(const env_t* e, const double* p, double* j) {
  if (e->kind == CPL_ENV_GROUND) {
    j[0] = 0.0; j[1] = 0.0; j[2] = 0.0;
    j[2] = 1.0;
  } else {
    for (int i = 0; i < 3; ++i)
      j[i] = e->P[i] / pow(e->R[i], e->P[i]) * pow(p[i] - e->C[i], e->P[i] - 1);
  }
}
/* Ground::GetNormalValue src/Ground.cpp:38-43; Superquadric src/Superquadric.cpp:60-69
 * (the norm is recomputed for every component, same value) */
static void env_normal(const env_t* e, const double* p, double* nv) {
  if (e->kind == CPL_ENV_GROUND) {
    nv[0] = 0.0; nv[1] = 0.0; nv[2] = 0.0;
    nv[2] = 1.0;
  } else {
    double j[3];
    env_jacobian(e, p, j);
    nv[0] = -j[0] / enorm(j);
    nv[1] = -j[1] / enorm(j);
    nv[2] = -j[2] / enorm(j);
  }
}
/* Ground::GetNormalJacobian src/Ground.cpp:46-50 (zero 3x3);
 * Superquadric::GetNormalJacobian src/Superquadric.cpp:72-209 — MATLAB-generated expressions
 * restated term by term with the reference's evaluation order (left-to-right * and /,
 * left-to-right + and -).  a[.] / R / P / C index 0,1,2 = x,y,z. */
static void env_normal_jacobian(const env_t* e, const double* p, double J[3][3]) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) J[r][c] = 0.0;
  if (e->kind == CPL_ENV_GROUND) return;
  const double* C = e->C;
  const double* R = e->R;
  const double* P = e->P;
  double t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15, t16, t17, t18, t19, t20;

  /* (0,0)  src/Superquadric.cpp:78-100 */
  t2 = -C[0] + p[0]; t3 = C[0] - p[0]; t4 = 1.0 / (t3 * t3); t6 = P[1] * 2.0; t5 = pow(R[1], -t6);
  t7 = C[1] - p[1]; t8 = 1.0 / (t7 * t7); t10 = P[2] * 2.0; t9 = pow(R[2], -t10);
  t11 = C[2] - p[2]; t12 = 1.0 / (t11 * t11); t13 = P[1] * P[1]; t14 = -C[1] + p[1];
  t15 = pow(t14, t6); t16 = P[2] * P[2]; t17 = -C[2] + p[2]; t18 = pow(t17, t10);
  t19 = pow(R[2], t10); t20 = pow(R[1], t6);
  J[0][0] = P[0] * pow(R[0], -P[0]) * pow(t2, P[0]) * t4 * t5 * t8 * t9 * t12 * (P[0] - 1.0) * 1.0 /
            pow(t5 * t8 * t13 * t15 + t9 * t12 * t16 * t18 +
                    (P[0] * P[0]) * pow(R[0], P[0] * -2.0) * pow(t2, P[0] * 2.0) * t4,
                3.0 / 2.0) *
            ((C[1] * C[1]) * t16 * t18 * t20 + (C[2] * C[2]) * t13 * t15 * t19 +
             (p[1] * p[1]) * t16 * t18 * t20 + (p[2] * p[2]) * t13 * t15 * t19 -
             C[1] * p[1] * t16 * t18 * t20 * 2.0 - C[2] * p[2] * t13 * t15 * t19 * 2.0);

  /* (0,1)  src/Superquadric.cpp:102-110 */
  t2 = P[1] * 2.0; t3 = -C[0] + p[0]; t4 = P[1] * P[1]; t5 = -C[1] + p[1]; t6 = t2 - 2.0;
  t7 = pow(R[1], -t2);
  J[0][1] = P[0] * pow(R[0], -P[0]) * pow(t3, P[0] - 1.0) * t4 * pow(t5, t2 - 3.0) * t6 * t7 * 1.0 /
            pow((P[2] * P[2]) * pow(R[2], P[2] * -2.0) * pow(-C[2] + p[2], P[2] * 2.0 - 2.0) +
                    (P[0] * P[0]) * pow(R[0], P[0] * -2.0) * pow(t3, P[0] * 2.0 - 2.0) +
                    t4 * pow(t5, t6) * t7,
                3.0 / 2.0) *
            (-1.0 / 2.0);

  /* (0,2)  src/Superquadric.cpp:112-120 */
  t2 = P[2] * 2.0; t3 = -C[0] + p[0]; t4 = P[2] * P[2]; t5 = -C[2] + p[2]; t6 = t2 - 2.0;
  t7 = pow(R[2], -t2);
  J[0][2] = P[0] * pow(R[0], -P[0]) * pow(t3, P[0] - 1.0) * t4 * pow(t5, t2 - 3.0) * t6 * t7 * 1.0 /
            pow((P[1] * P[1]) * pow(R[1], P[1] * -2.0) * pow(-C[1] + p[1], P[1] * 2.0 - 2.0) +
                    (P[0] * P[0]) * pow(R[0], P[0] * -2.0) * pow(t3, P[0] * 2.0 - 2.0) +
                    t4 * pow(t5, t6) * t7,
                3.0 / 2.0) *
            (-1.0 / 2.0);

  /* (1,0)  src/Superquadric.cpp:122-130 */
  t2 = P[0] * 2.0; t3 = P[0] * P[0]; t4 = -C[0] + p[0]; t5 = t2 - 2.0; t6 = -C[1] + p[1];
  t7 = pow(R[0], -t2);
  J[1][0] = P[1] * pow(R[1], -P[1]) * t3 * pow(t4, t2 - 3.0) * t5 * pow(t6, P[1] - 1.0) * t7 * 1.0 /
            pow((P[2] * P[2]) * pow(R[2], P[2] * -2.0) * pow(-C[2] + p[2], P[2] * 2.0 - 2.0) +
                    (P[1] * P[1]) * pow(R[1], P[1] * -2.0) * pow(t6, P[1] * 2.0 - 2.0) +
                    t3 * pow(t4, t5) * t7,
                3.0 / 2.0) *
            (-1.0 / 2.0);

  /* (1,1)  src/Superquadric.cpp:132-154 */
  t3 = P[0] * 2.0; t2 = pow(R[0], -t3); t4 = C[0] - p[0]; t5 = 1.0 / (t4 * t4); t6 = -C[1] + p[1];
  t7 = C[1] - p[1]; t8 = 1.0 / (t7 * t7); t10 = P[2] * 2.0; t9 = pow(R[2], -t10);
  t11 = C[2] - p[2]; t12 = 1.0 / (t11 * t11); t13 = P[0] * P[0]; t14 = -C[0] + p[0];
  t15 = pow(t14, t3); t16 = P[2] * P[2]; t17 = -C[2] + p[2]; t18 = pow(t17, t10);
  t19 = pow(R[2], t10); t20 = pow(R[0], t3);
  J[1][1] = P[1] * pow(R[1], -P[1]) * t2 * t5 * pow(t6, P[1]) * t8 * t9 * t12 * (P[1] - 1.0) * 1.0 /
            pow(t2 * t5 * t13 * t15 + t9 * t12 * t16 * t18 +
                    (P[1] * P[1]) * pow(R[1], P[1] * -2.0) * pow(t6, P[1] * 2.0) * t8,
                3.0 / 2.0) *
            ((C[0] * C[0]) * t16 * t18 * t20 + (C[2] * C[2]) * t13 * t15 * t19 +
             (p[0] * p[0]) * t16 * t18 * t20 + (p[2] * p[2]) * t13 * t15 * t19 -
             C[0] * p[0] * t16 * t18 * t20 * 2.0 - C[2] * p[2] * t13 * t15 * t19 * 2.0);

  /* (1,2)  src/Superquadric.cpp:156-164 */
  t2 = P[2] * 2.0; t3 = -C[1] + p[1]; t4 = P[2] * P[2]; t5 = -C[2] + p[2]; t6 = t2 - 2.0;
  t7 = pow(R[2], -t2);
  J[1][2] = P[1] * pow(R[1], -P[1]) * pow(t3, P[1] - 1.0) * t4 * pow(t5, t2 - 3.0) * t6 * t7 * 1.0 /
            pow((P[0] * P[0]) * pow(R[0], P[0] * -2.0) * pow(-C[0] + p[0], P[0] * 2.0 - 2.0) +
                    (P[1] * P[1]) * pow(R[1], P[1] * -2.0) * pow(t3, P[1] * 2.0 - 2.0) +
                    t4 * pow(t5, t6) * t7,
                3.0 / 2.0) *
            (-1.0 / 2.0);

  /* (2,0)  src/Superquadric.cpp:166-174 */
  t2 = P[0] * 2.0; t3 = P[0] * P[0]; t4 = -C[0] + p[0]; t5 = t2 - 2.0; t6 = -C[2] + p[2];
  t7 = pow(R[0], -t2);
  J[2][0] = P[2] * pow(R[2], -P[2]) * t3 * pow(t4, t2 - 3.0) * t5 * pow(t6, P[2] - 1.0) * t7 * 1.0 /
            pow((P[1] * P[1]) * pow(R[1], P[1] * -2.0) * pow(-C[1] + p[1], P[1] * 2.0 - 2.0) +
                    (P[2] * P[2]) * pow(R[2], P[2] * -2.0) * pow(t6, P[2] * 2.0 - 2.0) +
                    t3 * pow(t4, t5) * t7,
                3.0 / 2.0) *
            (-1.0 / 2.0);

  /* (2,1)  src/Superquadric.cpp:176-184 */
  t2 = P[1] * 2.0; t3 = P[1] * P[1]; t4 = -C[1] + p[1]; t5 = t2 - 2.0; t6 = -C[2] + p[2];
  t7 = pow(R[1], -t2);
  J[2][1] = P[2] * pow(R[2], -P[2]) * t3 * pow(t4, t2 - 3.0) * t5 * pow(t6, P[2] - 1.0) * t7 * 1.0 /
            pow((P[0] * P[0]) * pow(R[0], P[0] * -2.0) * pow(-C[0] + p[0], P[0] * 2.0 - 2.0) +
                    (P[2] * P[2]) * pow(R[2], P[2] * -2.0) * pow(t6, P[2] * 2.0 - 2.0) +
                    t3 * pow(t4, t5) * t7,
                3.0 / 2.0) *
            (-1.0 / 2.0);

  /* (2,2)  src/Superquadric.cpp:186-208 */
  t3 = P[0] * 2.0; t2 = pow(R[0], -t3); t4 = C[0] - p[0]; t5 = 1.0 / (t4 * t4); t7 = P[1] * 2.0;
  t6 = pow(R[1], -t7); t8 = C[1] - p[1]; t9 = 1.0 / (t8 * t8); t10 = -C[2] + p[2];
  t11 = C[2] - p[2]; t12 = 1.0 / (t11 * t11); t13 = P[0] * P[0]; t14 = -C[0] + p[0];
  t15 = pow(t14, t3); t16 = P[1] * P[1]; t17 = -C[1] + p[1]; t18 = pow(t17, t7);
  t19 = pow(R[1], t7); t20 = pow(R[0], t3);
  J[2][2] = P[2] * pow(R[2], -P[2]) * t2 * t5 * t6 * t9 * pow(t10, P[2]) * t12 * (P[2] - 1.0) * 1.0 /
            pow(t2 * t5 * t13 * t15 + t6 * t9 * t16 * t18 +
                    (P[2] * P[2]) * pow(R[2], P[2] * -2.0) * pow(t10, P[2] * 2.0) * t12,
                3.0 / 2.0) *
            ((C[0] * C[0]) * t16 * t18 * t20 + (C[1] * C[1]) * t13 * t15 * t19 +
             (p[0] * p[0]) * t16 * t18 * t20 + (p[1] * p[1]) * t13 * t15 * t19 -
             C[0] * p[0] * t16 * t18 * t20 * 2.0 - C[1] * p[1] * t13 * t15 * t19 * 2.0);
}

/* ---------------------------------------------------------------------------------------- */
/* Constraint sets                                                                           */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
  const cpl_problem_desc* d;
  const double* x;
  double mass;
  env_t env;
  int has_env;
} ctx_t;

enum { CS_STATICS = 0, CS_ENV = 1, CS_NORMAL = 2, CS_CONE = 3 };
typedef struct { int kind, contact, rows; } cset_t;

/* CentroidalStatics::GetValues src/Constraints/CentroidalStatics.cpp:37-61 */
static void statics_values(const ctx_t* c, double* v) {
  const cpl_problem_desc* d = c->d;
  for (int r = 0; r < 6; ++r) v[r] = 0.0;
  const double* com = xcom(c->x);
  for (int k = 0; k < d->n_contacts; ++k) { /* std::map order */
    int i = d->map_order[k];
    const double* F = xF(c->x, i);
    const double* p = xp(c->x, i);
    double dp[3] = {p[0] - com[0], p[1] - com[1], p[2] - com[2]};
    double cr[3];
    ecross(dp, F, cr);
    v[0] += F[0]; v[1] += F[1]; v[2] += F[2];
    v[3] += cr[0]; v[4] += cr[1]; v[5] += cr[2];
  }
  for (int r = 0; r < 6; ++r) v[r] -= d->wrench[r];
  double mg[3] = {c->mass * d->gravity[0], c->mass * d->gravity[1], c->mass * d->gravity[2]};
  v[0] += mg[0]; v[1] += mg[1]; v[2] += mg[2];
}

/* CentroidalStatics::FillJacobianBlock src/Constraints/CentroidalStatics.cpp:75-137 */
static void statics_fill(const ctx_t* c, varset_t vs, blk_t* b) {
  const cpl_problem_desc* d = c->d;
  blk_zero(b);
  const double* com = xcom(c->x);
  for (int k = 0; k < d->n_contacts; ++k) {
    int i = d->map_order[k];
    const double* p = xp(c->x, i);
    const double* F = xF(c->x, i);
    if (vs.kind == VK_F && vs.contact == i) {
      *blk_ref(b, 0, 0) = 1.0;
      *blk_ref(b, 1, 1) = 1.0;
      *blk_ref(b, 2, 2) = 1.0;
      *blk_ref(b, 3, 1) = -(p[2] - com[2]);
      *blk_ref(b, 3, 2) = p[1] - com[1];
      *blk_ref(b, 4, 0) = p[2] - com[2];
      *blk_ref(b, 4, 2) = -(p[0] - com[0]);
      *blk_ref(b, 5, 0) = -(p[1] - com[1]);
      *blk_ref(b, 5, 1) = p[0] - com[0];
    }
    if (vs.kind == VK_P && vs.contact == i) {
      *blk_ref(b, 3, 1) = F[2];
      *blk_ref(b, 3, 2) = -F[1];
      *blk_ref(b, 4, 0) = -F[2];
      *blk_ref(b, 4, 2) = F[0];
      *blk_ref(b, 5, 0) = F[1];
      *blk_ref(b, 5, 1) = -F[0];
    }
  }
  if (vs.kind == VK_COM) {
    for (int k = 0; k < d->n_contacts; ++k) {
      const double* F = xF(c->x, d->map_order[k]);
      *blk_ref(b, 3, 1) -= F[2];
      *blk_ref(b, 3, 2) -= -F[1];
      *blk_ref(b, 4, 0) -= -F[2];
      *blk_ref(b, 4, 2) -= F[0];
      *blk_ref(b, 5, 0) -= F[1];
      *blk_ref(b, 5, 1) -= -F[0];
    }
  }
}

/* EnvironmentConstraint::GetValues src/Constraints/EnvironmentConstraint.cpp:16-28 */
static void envc_values(const ctx_t* c, int i, double* v) {
  v[0] = 0.0; /* value.setZero(1) */
  env_value(&c->env, xp(c->x, i), &v[0]);
}
/* EnvironmentConstraint::FillJacobianBlock src/Constraints/EnvironmentConstraint.cpp:42-61
 * (GetEnvironmentJacobian runs for every variable set, before the name test) */
static void envc_fill(const ctx_t* c, int i, varset_t vs, blk_t* b) {
  blk_zero(b);
  double j[3];
  env_jacobian(&c->env, xp(c->x, i), j);
  if (vs.kind == VK_P && vs.contact == i) {
    *blk_ref(b, 0, 0) = j[0];
    *blk_ref(b, 0, 1) = j[1];
    *blk_ref(b, 0, 2) = j[2];
  }
}

/* EnvironmentNormal::GetValues src/Constraints/EnvironmentNormal.cpp:16-33 */
static void envn_values(const ctx_t* c, int i, double* v) {
  double en[3];
  env_normal(&c->env, xp(c->x, i), en);
  const double* n = xn(c->x, i);
  v[0] = n[0] - en[0];
  v[1] = n[1] - en[1];
  v[2] = n[2] - en[2];
}
/* EnvironmentNormal::FillJacobianBlock src/Constraints/EnvironmentNormal.cpp:52-87
 * (GetNormalJacobian runs for every variable set; entered with a plus sign) */
static void envn_fill(const ctx_t* c, int i, varset_t vs, blk_t* b) {
  blk_zero(b);
  double J[3][3];
  env_normal_jacobian(&c->env, xp(c->x, i), J);
  if (vs.kind == VK_N && vs.contact == i) {
    *blk_ref(b, 0, 0) = 1.0;
    *blk_ref(b, 1, 1) = 1.0;
    *blk_ref(b, 2, 2) = 1.0;
  }
  if (vs.kind == VK_P && vs.contact == i) {
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q) *blk_ref(b, r, q) = J[r][q];
  }
}

/* FrictionCone::GetValues src/Constraints/FrictionCone.cpp:30-45
 * mu: the problem's environment, or CplProblem's private Ground when env == nullptr
 * (src/CplProblem.cpp:63-71, SetMu src/CplProblem.cpp:275-287) */
static void cone_values(const ctx_t* c, int i, double* v) {
  const double* F = xF(c->x, i);
  const double* n = xn(c->x, i);
  double mu = c->d->mu;
  v[0] = 0.0; v[1] = 0.0;
  v[0] = -edot(F, n) + c->d->F_thr[i];
  double nF = edot(n, F);
  double tv[3] = {F[0] - nF * n[0], F[1] - nF * n[1], F[2] - nF * n[2]};
  v[1] = enorm(tv) - mu * edot(F, n);
}
/* FrictionCone::FillJacobianBlock src/Constraints/FrictionCone.cpp:60-103 */
static void cone_fill(const ctx_t* c, int i, varset_t vs, blk_t* b) {
  double mu = c->d->mu;
  blk_zero(b);
  const double* F = xF(c->x, i);
  const double* n = xn(c->x, i);
  double t1 = edot(F, n);
  double t2 = F[0] - n[0] * t1;
  double t3 = F[1] - n[1] * t1;
  double t4 = F[2] - n[2] * t1;
  double t5 = F[0] * n[0];
  double t6 = F[1] * n[1];
  double t7 = F[2] * n[2];
  if (vs.kind == VK_F && vs.contact == i) {
    *blk_ref(b, 0, 0) = -n[0];
    *blk_ref(b, 0, 1) = -n[1];
    *blk_ref(b, 0, 2) = -n[2];
    *blk_ref(b, 1, 0) = (t2 * (n[0] * n[0] - 1.0) * 2.0 + n[0] * n[1] * t3 * 2.0 + n[0] * n[2] * t4 * 2.0) *
                            1.0 / sqrt(t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - mu * n[0];
    *blk_ref(b, 1, 1) = (t3 * (n[1] * n[1] - 1.0) * 2.0 + n[0] * n[1] * t2 * 2.0 + n[1] * n[2] * t4 * 2.0) *
                            1.0 / sqrt(t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - mu * n[1];
    *blk_ref(b, 1, 2) = (t4 * (n[2] * n[2] - 1.0) * 2.0 + n[0] * n[2] * t2 * 2.0 + n[1] * n[2] * t3 * 2.0) *
                            1.0 / sqrt(t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - mu * n[2];
  }
  if (vs.kind == VK_N && vs.contact == i) {
    *blk_ref(b, 0, 0) = -F[0];
    *blk_ref(b, 0, 1) = -F[1];
    *blk_ref(b, 0, 2) = -F[2];
    *blk_ref(b, 1, 0) = (t2 * (t6 + t7 + t5 * 2.0) * 2.0 + F[0] * n[1] * t3 * 2.0 + F[0] * n[2] * t4 * 2.0) *
                            1.0 / sqrt(t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - mu * F[0];
    *blk_ref(b, 1, 1) = (t3 * (t5 + t7 + t6 * 2.0) * 2.0 + F[1] * n[0] * t2 * 2.0 + F[1] * n[2] * t4 * 2.0) *
                            1.0 / sqrt(t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - mu * F[1];
    *blk_ref(b, 1, 2) = (t4 * (t5 + t6 + t7 * 2.0) * 2.0 + F[2] * n[0] * t2 * 2.0 + F[2] * n[1] * t3 * 2.0) *
                            1.0 / sqrt(t2 * t2 + t3 * t3 + t4 * t4) * (-1.0 / 2.0) - mu * F[2];
  }
}

/* Constraint-set order of CplProblem's ctor: statics, then per contact in map order
 * env, normal, cone (or cone alone without environment)  src/CplProblem.cpp:37-75 */
static int constraint_sets(const cpl_problem_desc* d, int has_env, cset_t* out) {
  int s = 0;
  out[s].kind = CS_STATICS; out[s].contact = -1; out[s].rows = 6; ++s;
  for (int k = 0; k < d->n_contacts; ++k) {
    int i = d->map_order[k];
    if (has_env) {
      out[s].kind = CS_ENV; out[s].contact = i; out[s].rows = 1; ++s;
      out[s].kind = CS_NORMAL; out[s].contact = i; out[s].rows = 3; ++s;
    }
    out[s].kind = CS_CONE; out[s].contact = i; out[s].rows = 2; ++s;
  }
  return s;
}
static void cset_values(const ctx_t* c, cset_t cs, double* v) {
  switch (cs.kind) {
    case CS_STATICS: statics_values(c, v); break;
    case CS_ENV: envc_values(c, cs.contact, v); break;
    case CS_NORMAL: envn_values(c, cs.contact, v); break;
    default: cone_values(c, cs.contact, v); break;
  }
}
static void cset_fill(const ctx_t* c, cset_t cs, varset_t vs, blk_t* b) {
  switch (cs.kind) {
    case CS_STATICS: statics_fill(c, vs, b); break;
    case CS_ENV: envc_fill(c, cs.contact, vs, b); break;
    case CS_NORMAL: envn_fill(c, cs.contact, vs, b); break;
    default: cone_fill(c, cs.contact, vs, b); break;
  }
}

/* MinimizeCentroidalVariables::GetCost src/MinimizeCentroidalVariables.cpp:124-148 */
static double cost_value(const ctx_t* c) {
  const cpl_problem_desc* d = c->d;
  double value = 0;
  const double* com = xcom(c->x);
  for (int k = 0; k < d->n_contacts; ++k) {
    int i = d->map_order[k];
    const double* F = xF(c->x, i);
    const double* p = xp(c->x, i);
    double dp[3] = {p[0] - d->p_ref[i][0], p[1] - d->p_ref[i][1], p[2] - d->p_ref[i][2]};
    double dF[3] = {F[0] - d->F_ref[i][0], F[1] - d->F_ref[i][1], F[2] - d->F_ref[i][2]};
    value += 0.5 * d->W_p[i] * esqn(dp) + 0.5 * d->W_F[i] * esqn(dF);
  }
  double dc[3] = {com[0] - d->com_ref[0], com[1] - d->com_ref[1], com[2] - d->com_ref[2]};
  value += 0.5 * d->W_com * esqn(dc);
  return value;
}
/* MinimizeCentroidalVariables::FillJacobianBlock src/MinimizeCentroidalVariables.cpp:151-192,
 * assembled into IPOPT's dense grad_f (absent entries are 0) */
static void cost_fill(const ctx_t* c, varset_t vs, blk_t* b) {
  const cpl_problem_desc* d = c->d;
  blk_zero(b);
  const double* com = xcom(c->x);
  for (int k = 0; k < d->n_contacts; ++k) {
    int i = d->map_order[k];
    if (vs.kind == VK_F && vs.contact == i) {
      const double* F = xF(c->x, i);
      double w = d->W_F[i];
      *blk_ref(b, 0, 0) = w * (F[0] - d->F_ref[i][0]);
      *blk_ref(b, 0, 1) = w * (F[1] - d->F_ref[i][1]);
      *blk_ref(b, 0, 2) = w * (F[2] - d->F_ref[i][2]);
    }
    if (vs.kind == VK_P && vs.contact == i) {
      const double* p = xp(c->x, i);
      double w = d->W_p[i];
      *blk_ref(b, 0, 0) = w * (p[0] - d->p_ref[i][0]);
      *blk_ref(b, 0, 1) = w * (p[1] - d->p_ref[i][1]);
      *blk_ref(b, 0, 2) = w * (p[2] - d->p_ref[i][2]);
    }
  }
  if (vs.kind == VK_COM) {
    *blk_ref(b, 0, 0) = d->W_com * (com[0] - d->com_ref[0]);
    *blk_ref(b, 0, 1) = d->W_com * (com[1] - d->com_ref[1]);
    *blk_ref(b, 0, 2) = d->W_com * (com[2] - d->com_ref[2]);
  }
}

/* ---------------------------------------------------------------------------------------- */
/* Problem-level entry points                                                                */
/* ---------------------------------------------------------------------------------------- */
static int has_env_kind(int k) { return k == CPL_ENV_GROUND || k == CPL_ENV_SUPERQUADRIC || k == CPL_ENV_MIXED; }

static int check_desc(const cpl_problem_desc* d) {
  if (!d || d->n_contacts < 1 || d->n_contacts > CPL_MAX_CONTACTS) return CPL_ERR_INVALID_ARGUMENT;
  if (d->env_kind < CPL_ENV_NONE || d->env_kind > CPL_ENV_MIXED) return CPL_ERR_INVALID_ARGUMENT;
  return CPL_OK;
}

int cplo_dims(const cpl_problem_desc* d, int32_t* n, int32_t* m, int32_t* nnz);

/* Workspace: dense value image + stored-entry mask of the assembled Jacobian */
typedef struct {
  int n, m, nnz;
  double* dense;  /* m*n */
  int32_t* pos;   /* nnz: row-major index r*n+c of each stored entry, CSR order */
} work_t;

/* One instance through IFOPT's walk: every constraint set x every variable set. */
static void assemble_instance(const ctx_t* c, work_t* w, double* g, double* jac, unsigned char* mask) {
  cset_t sets[1 + 3 * CPL_MAX_CONTACTS];
  int ns = constraint_sets(c->d, c->has_env, sets);
  int nvar = 1 + 3 * c->d->n_contacts;
  int row = 0;
  blk_t b;
  double v[6];
  for (int s = 0; s < ns; ++s) {
    if (g) {
      cset_values(c, sets[s], v);
      for (int r = 0; r < sets[s].rows; ++r) g[row + r] = v[r];
    }
    if (jac || mask) {
      for (int vi = 0; vi < nvar; ++vi) {
        cset_fill(c, sets[s], varset_of(vi), &b);
        for (int k = 0; k < b.n; ++k) {
          int idx = (row + b.r[k]) * w->n + 3 * vi + b.c[k];
          w->dense[idx] = b.v[k];
          if (mask) mask[idx] = 1;
        }
      }
    }
    row += sets[s].rows;
  }
  if (jac)
    for (int k = 0; k < w->nnz; ++k) jac[k] = w->dense[w->pos[k]];
}

static void make_ctx(ctx_t* c, const cpl_problem_desc* d, const double* x, double mass, int kind) {
  c->d = d;
  c->x = x;
  c->mass = mass;
  c->has_env = has_env_kind(d->env_kind);
  c->env.kind = kind;
  c->env.z = d->ground_z;
  for (int i = 0; i < 3; ++i) { c->env.C[i] = d->sq_C[i]; c->env.R[i] = d->sq_R[i]; c->env.P[i] = d->sq_P[i]; }
}

/* Structure: assembled from the stored entries of one walk (value-independent on this path). */
static int build_structure(const cpl_problem_desc* d, work_t* w) {
  int32_t n, m, nnz;
  w->dense = NULL;
  w->pos = NULL;
  int st = cplo_dims(d, &n, &m, &nnz);
  if (st) return st;
  w->n = n; w->m = m; w->nnz = nnz;
  w->dense = (double*)calloc((size_t)m * n, sizeof(double));
  w->pos = (int32_t*)malloc(sizeof(int32_t) * (size_t)nnz);
  unsigned char* mask = (unsigned char*)calloc((size_t)m * n, 1);
  double* x0 = (double*)calloc((size_t)n, sizeof(double));
  for (int i = 0; i < n; ++i) x0[i] = 0.25 + 0.01 * i; /* any point: the structure is value-independent */
  ctx_t c;
  make_ctx(&c, d, x0, d->mass, d->env_kind == CPL_ENV_MIXED ? CPL_ENV_GROUND : d->env_kind);
  assemble_instance(&c, w, NULL, NULL, mask);
  int k = 0;
  for (int idx = 0; idx < m * n; ++idx)
    if (mask[idx]) {
      if (k < nnz) w->pos[k] = idx;
      ++k;
    }
  free(mask);
  free(x0);
  return k == nnz ? CPL_OK : CPL_ERR_RUNTIME;
}
static void free_work(work_t* w) { free(w->dense); free(w->pos); }

/* get_nlp_info: n = 3+9N; m = 6+6N (env) / 6+2N; nnz counted from the blocks' stored entries */
int cplo_dims(const cpl_problem_desc* d, int32_t* n, int32_t* m, int32_t* nnz) {
  int st = check_desc(d);
  if (st) return st;
  int N = d->n_contacts, he = has_env_kind(d->env_kind);
  cset_t sets[1 + 3 * CPL_MAX_CONTACTS];
  int ns = constraint_sets(d, he, sets);
  int rows = 0;
  for (int s = 0; s < ns; ++s) rows += sets[s].rows;
  /* count stored entries by walking every block once at a generic point */
  int nv = 3 + 9 * N;
  double* x0 = (double*)calloc((size_t)nv, sizeof(double));
  for (int i = 0; i < nv; ++i) x0[i] = 0.25 + 0.01 * i;
  ctx_t c;
  make_ctx(&c, d, x0, d->mass, d->env_kind == CPL_ENV_MIXED ? CPL_ENV_GROUND : d->env_kind);
  int count = 0;
  blk_t b;
  for (int s = 0; s < ns; ++s)
    for (int vi = 0; vi < 1 + 3 * N; ++vi) {
      cset_fill(&c, sets[s], varset_of(vi), &b);
      count += b.n;
    }
  free(x0);
  if (n) *n = nv;
  if (m) *m = rows;
  if (nnz) *nnz = count;
  return CPL_OK;
}

int cplo_structure(const cpl_problem_desc* d, int32_t* iRow, int32_t* jCol) {
  work_t w;
  int st = build_structure(d, &w);
  if (st == CPL_OK)
    for (int k = 0; k < w.nnz; ++k) {
      if (iRow) iRow[k] = w.pos[k] / w.n;
      if (jCol) jCol[k] = w.pos[k] % w.n;
    }
  free_work(&w);
  return st;
}

/* get_bounds_info: Variable3D::GetBounds src/Variable3D.cpp:54-65; constraint bounds
 * CentroidalStatics.cpp:64-73 [0,0]; EnvironmentConstraint.cpp:31-40 [0,0];
 * EnvironmentNormal.cpp:36-50 [0,0]; FrictionCone.cpp:48-58 BoundSmallerZero = [-1e20, 0] */
int cplo_bounds(const cpl_problem_desc* d, double* xl, double* xu, double* gl, double* gu) {
  int st = check_desc(d);
  if (st) return st;
  int N = d->n_contacts;
  if (xl || xu)
    for (int j = 0; j < 3; ++j) {
      if (xl) xl[j] = d->com_lb[j];
      if (xu) xu[j] = d->com_ub[j];
    }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < 3; ++j) {
      if (xl) { xl[3 + 9 * i + j] = d->F_lb[i][j]; xl[6 + 9 * i + j] = d->p_lb[i][j]; xl[9 + 9 * i + j] = d->n_lb[i][j]; }
      if (xu) { xu[3 + 9 * i + j] = d->F_ub[i][j]; xu[6 + 9 * i + j] = d->p_ub[i][j]; xu[9 + 9 * i + j] = d->n_ub[i][j]; }
    }
  cset_t sets[1 + 3 * CPL_MAX_CONTACTS];
  int ns = constraint_sets(d, has_env_kind(d->env_kind), sets);
  int row = 0;
  for (int s = 0; s < ns; ++s) {
    for (int r = 0; r < sets[s].rows; ++r) {
      double lo = 0.0, hi = 0.0;
      if (sets[s].kind == CS_CONE) lo = -CPL_INF;
      if (gl) gl[row + r] = lo;
      if (gu) gu[row + r] = hi;
    }
    row += sets[s].rows;
  }
  return CPL_OK;
}

static void eval_one(const cpl_problem_desc* d, work_t* w, const double* x, double mass, int kind, double* g,
                     double* jac, double* f, double* grad) {
  ctx_t c;
  make_ctx(&c, d, x, mass, kind);
  assemble_instance(&c, w, g, jac, NULL);
  if (f) *f = cost_value(&c);
  if (grad) {
    int nvar = 1 + 3 * d->n_contacts;
    for (int j = 0; j < w->n; ++j) grad[j] = 0.0;
    blk_t b;
    for (int vi = 0; vi < nvar; ++vi) {
      cost_fill(&c, varset_of(vi), &b);
      for (int k = 0; k < b.n; ++k) grad[3 * vi + b.c[k]] = b.v[k];
    }
  }
}

static int instance_kind(const cpl_problem_desc* d, const uint8_t* tags, int64_t b) {
  if (d->env_kind == CPL_ENV_MIXED) return tags ? (tags[b] == CPL_ENV_SUPERQUADRIC ? CPL_ENV_SUPERQUADRIC : CPL_ENV_GROUND) : CPL_ENV_GROUND;
  return d->env_kind;
}

/* Batched evaluation over instances (OpenMP over instances when nthreads > 1). */
int cplo_eval_batch(const cpl_problem_desc* d, int64_t B, const double* x, const double* mass,
                    const uint8_t* tags, double* g, double* jac, double* f, double* grad, int nthreads) {
  int st = check_desc(d);
  if (st) return st;
  if (B < 0 || !x) return CPL_ERR_INVALID_ARGUMENT;
  if (d->env_kind == CPL_ENV_MIXED && !tags) return CPL_ERR_INVALID_ARGUMENT;
  work_t w0;
  st = build_structure(d, &w0);
  if (st) { free_work(&w0); return st; }
  int n = w0.n, m = w0.m, nnz = w0.nnz;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    work_t w = w0;
    w.dense = (double*)calloc((size_t)m * n, sizeof(double));
#pragma omp for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
      eval_one(d, &w, x + b * n, mass ? mass[b] : d->mass, instance_kind(d, tags, b), g ? g + b * m : NULL,
               jac ? jac + b * nnz : NULL, f ? f + b : NULL, grad ? grad + b * n : NULL);
    }
    free(w.dense);
  }
  free_work(&w0);
  return CPL_OK;
}

/* One-instance evaluation with a kept workspace (the solve restatement's callbacks,
 * cpl_solve_host.c): the structure is built once per solve, not per call. */
void* cplo_ws_new(const cpl_problem_desc* d) {
  if (check_desc(d)) return NULL;
  work_t* w = (work_t*)calloc(1, sizeof(work_t));
  if (!w) return NULL;
  if (build_structure(d, w)) { free_work(w); free(w); return NULL; }
  return w;
}
void cplo_ws_eval(const cpl_problem_desc* d, void* ws, const double* x, double mass, double* g, double* jac,
                  double* f, double* grad) {
  eval_one(d, (work_t*)ws, x, mass, instance_kind(d, NULL, 0), g, jac, f, grad);
}
void cplo_ws_free(void* ws) {
  if (!ws) return;
  free_work((work_t*)ws);
  free(ws);
}

/* Wall-clock timing of cplo_eval_batch for the bench's cpu_baseline leg. */
double cplo_time_eval_batch(const cpl_problem_desc* d, int64_t B, const double* x, const double* mass,
                            const uint8_t* tags, double* g, double* jac, double* f, double* grad, int nthreads,
                            int reps) {
#ifdef _OPENMP
  double t0 = omp_get_wtime();
  for (int r = 0; r < reps; ++r)
    if (cplo_eval_batch(d, B, x, mass, tags, g, jac, f, grad, nthreads)) return -1.0;
  return (omp_get_wtime() - t0) / (reps > 0 ? reps : 1);
#else
  (void)d; (void)B; (void)x; (void)mass; (void)tags; (void)g; (void)jac; (void)f; (void)grad; (void)nthreads; (void)reps;
  return -1.0;
#endif
}

int cplo_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
