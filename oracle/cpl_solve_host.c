/* cpl_solve_host.c — TEST / BASELINE INFRASTRUCTURE, not the product path.
 *
 * A compiled, single-core restatement of the solve loop (centroidalplanner_amd/batch_ipm.py's host
 * path, B = 1, IFOPT's limited-memory Hessian) over the oracle's callbacks (cpl_oracle.c): the CPU
 * baseline of bench.py's single-solve and configs[4] solve legs.  The reference solves each instance
 * with IPOPT through IFOPT's IpoptSolver (src/CentroidalPlanner.cpp:22-34); IPOPT (and MUMPS) is not
 * in this image, so this is a restatement of the same method — IPOPT's primal-dual interior-point
 * iteration with its filter line search (second-order corrections, tiny steps, alpha_min, the soft
 * restoration step), monotone barrier update, limited-memory BFGS (6 pairs, scalar1) and
 * MinC_1Nrm restoration phase — with dense factorisations written out here: a Householder QR of
 * A^T for the null-space Newton step with the inertia test on the reduced Hessian's Cholesky, and the
 * restoration phase's p / n-eliminated system by Cholesky.  Every constant and branch follows
 * batch_ipm.py (which cites IPOPT's option defaults); the iterates agree with it to rounding, not
 * bitwise (different summation orders in the dense kernels).
 *
 * Only tests/ and bench.py's cpu_baseline legs call it (ctypes).
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/cpl_mi355x.h"

void* cplo_ws_new(const cpl_problem_desc* d);
void cplo_ws_eval(const cpl_problem_desc* d, void* ws, const double* x, double mass, double* g, double* jac,
                  double* f, double* grad);
void cplo_ws_free(void* ws);
int cplo_dims(const cpl_problem_desc* d, int32_t* n, int32_t* m, int32_t* nnz);
int cplo_structure(const cpl_problem_desc* d, int32_t* iRow, int32_t* jCol);
int cplo_bounds(const cpl_problem_desc* d, double* xl, double* xu, double* gl, double* gu);

#define EPS DBL_EPSILON
#define LM_HIST 6
#define LM_MAX_SKIP 2
#define BIG 1e19
#define GAMMA_TH 1e-5
#define GAMMA_PHI 1e-8
#define DELTA_SW 1.0
#define S_TH 1.1
#define S_PHI 2.3
#define ETA_PHI 1e-8
#define ALPHA_MIN_FRAC 0.05
#define KAPPA_SOC 0.99
#define OBJ_MAX_INC 5.0
#define KAPPA_SIGMA 1e10
#define BARRIER_TOL_FACTOR 10.0
#define COMPL_INF_TOL 1e-4
#define MU_ROUNDS 6
#define TINY_STEP_TOL (10.0 * DBL_EPSILON)
#define TINY_STEP_Y_TOL 1e-2
#define RHO_R 1000.0
#define KAPPA_RESTO 0.9
#define BOUND_MULT_RESET 1000.0
#define SOFT_RESTO_FACTOR 0.9999
#define ALMOST_FEASIBLE 1e-2   /* BacktrackingLineSearch: no restoration phase at theta <= 1e-2 tol */
#define MAX_SOFT_RESTO 10
#define FMAX 64
#define PIVOT_REL DBL_EPSILON
#define NWMAX 128
#define MMAX 128
#define NMAX 300

enum { ST_OPTIMAL = 0, ST_ACCEPTABLE = 1, ST_MAX_ITER = 2, ST_INFEASIBLE = 3, ST_RESTO_FAILED = 4 };

typedef struct {
  const cpl_problem_desc* d;
  void* ws;
  double mass;
  int n, m, nnz, nf, nI, nw, nbounds;
  int free_idx[NMAX], ineq[MMAX], row_slack[MMAX], iRow[4096], jCol[4096];
  double xl[NMAX], xu[NMAX], gl[MMAX], gu[MMAX], wl0[NWMAX], wu0[NWMAX];
  unsigned char hasL[NWMAX], hasU[NWMAX], is_fixed[NMAX];
  double Xbase[NMAX];
  double jac[4096];
  long evals;
  int exact;
  /* IPOPT's gradient-based NLP scaling (batch_ipm.py nlp_scaling): objective factor df, constraint
   * row factors dc; scaled = 0: all 1, the callbacks' values unchanged */
  int scaled;
  double df, dc[MMAX];
} Prob;

typedef struct {
  double f, grad[NMAX], g[MMAX];
  double J[MMAX * NMAX]; /* dense m x n, 0/0 entries as 0 */
} Eval;

static double dmin(double a, double b) { return a < b ? a : b; }
static double dmax(double a, double b) { return a > b ? a : b; }

static void unpack(const Prob* P, const double* w, double* X) {
  memcpy(X, P->Xbase, sizeof(double) * (size_t)P->n);
  for (int k = 0; k < P->nf; ++k) X[P->free_idx[k]] = w[k];
}

static void evaluate(Prob* P, const double* X, Eval* o) {
  ++P->evals;
  cplo_ws_eval(P->d, P->ws, X, P->mass, o->g, P->jac, &o->f, o->grad);
  memset(o->J, 0, sizeof(double) * (size_t)P->m * P->n);
  for (int k = 0; k < P->nnz; ++k) {
    const double v = P->jac[k];
    o->J[P->iRow[k] * P->n + P->jCol[k]] = v == v ? v : 0.0;  /* a cone at F_t = 0: 0/0 */
  }
  if (P->scaled) {  /* the scaled problem: df f, df grad f, dc g, dc J (one product per value) */
    o->f = o->f * P->df;
    for (int j = 0; j < P->n; ++j) o->grad[j] = o->grad[j] * P->df;
    for (int r = 0; r < P->m; ++r) {
      o->g[r] = o->g[r] * P->dc[r];
      for (int j = 0; j < P->n; ++j) o->J[r * P->n + j] = o->J[r * P->n + j] * P->dc[r];
    }
  }
}
static void evaluate_fg(Prob* P, const double* X, double* f, double* g) {
  ++P->evals;
  cplo_ws_eval(P->d, P->ws, X, P->mass, g, NULL, f, NULL);
  if (P->scaled) {
    *f = *f * P->df;
    for (int r = 0; r < P->m; ++r) g[r] = g[r] * P->dc[r];
  }
}
/* the multipliers of the unscaled callbacks: (dc y) / df (the scaled Lagrangian df f + (dc y)^T g is
 * df (f + ((dc y) / df)^T g)) */
static void y_raw(const Prob* P, const double* y, double* yr) {
  for (int r = 0; r < P->m; ++r) yr[r] = P->scaled ? (P->dc[r] * y[r]) / P->df : y[r];
}
/* IPOPT GradientScaling::DetermineScalingParametersImpl at the starting point X (nlp_scaling_max_gradient
 * 100, nlp_scaling_min_value 1e-8; gradients over the free variables, NaN entries as 0): df when
 * max |grad f| > 100; per constraint block (equality rows, inequality rows) whose largest row gradient
 * exceeds 100, dc_i = max(1e-8, 100 * (1 / max(100, row max))) on every row of the block */
static void nlp_scaling(Prob* P, const double* X) {
  double grad[NMAX], g[MMAX], f, rmax[MMAX];
  ++P->evals;
  cplo_ws_eval(P->d, P->ws, X, P->mass, g, P->jac, &f, grad);
  double gmax = 0.0;
  for (int k = 0; k < P->nf; ++k) {
    const double v = grad[P->free_idx[k]];
    gmax = dmax(gmax, v == v ? fabs(v) : 0.0);
  }
  P->df = gmax > 100.0 ? dmax(100.0 / gmax, 1e-8) : 1.0;
  for (int r = 0; r < P->m; ++r) { rmax[r] = 0.0; P->dc[r] = 1.0; }
  for (int k = 0; k < P->nnz; ++k) {
    const double v = P->jac[k];
    if (P->is_fixed[P->jCol[k]] || v != v) continue;
    rmax[P->iRow[k]] = dmax(rmax[P->iRow[k]], fabs(v));
  }
  for (int blk = 0; blk < 2; ++blk) {  /* 0: equality rows, 1: inequality rows */
    double bmax = 0.0;
    for (int r = 0; r < P->m; ++r)
      if ((P->row_slack[r] >= 0) == blk) bmax = dmax(bmax, rmax[r]);
    if (!(bmax > 100.0)) continue;
    for (int r = 0; r < P->m; ++r)
      if ((P->row_slack[r] >= 0) == blk) P->dc[r] = dmax(100.0 * (1.0 / dmax(rmax[r], 100.0)), 1e-8);
  }
  P->scaled = P->df != 1.0;
  for (int r = 0; r < P->m; ++r) P->scaled |= P->dc[r] != 1.0;
}

static void cons(const Prob* P, const double* g, const double* w, double* c) {
  for (int r = 0; r < P->m; ++r) {
    const int s = P->row_slack[r];
    c[r] = s >= 0 ? g[r] - w[P->nf + s] : g[r] - P->gl[r];
  }
}
static double sum_abs(const double* v, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += fabs(v[i]);
  return s;
}
static double max_abs(const double* v, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s = dmax(s, fabs(v[i]));
  return s;
}
/* A = dc/dw = [J_free | -P] (m x nw, row-major) */
static void jac_w(const Prob* P, const double* J, double* A) {
  const int nw = P->nw, nf = P->nf;
  for (int r = 0; r < P->m; ++r) {
    for (int k = 0; k < nf; ++k) A[r * nw + k] = J[r * P->n + P->free_idx[k]];
    for (int k = nf; k < nw; ++k) A[r * nw + k] = P->row_slack[r] == k - nf ? -1.0 : 0.0;
  }
}
static double barrier(const Prob* P, const double* w, double mu) {
  double s = 0.0;
  for (int k = 0; k < P->nw; ++k) {
    if (P->hasL[k]) s += log(w[k] - P->wl0[k]);
    if (P->hasU[k]) s += log(P->wu0[k] - w[k]);
  }
  return -mu * s;
}

/* Exact Hessian of f + y^T g over the free variables, nf x nf (zero_cost: of y^T g alone) — the C
 * form of pyoracle.lagrangian_hessian (Ground / no environment; the same operations in the same
 * order): cost diagonal (src/MinimizeCentroidalVariables.cpp:124-148), torque cross terms
 * (src/Constraints/CentroidalStatics.cpp:37-61), the cone rows' second derivatives
 * (src/Constraints/FrictionCone.cpp:30-45; the |t| terms count as 0 where |t| = 0). */
static void lagr_hessian(const Prob* P, const double* X, const double* Y, int zero_cost, double* Hf) {
  const cpl_problem_desc* d = P->d;
  const int N = d->n_contacts, n = P->n;
  static __thread double H[NMAX * NMAX];
  memset(H, 0, sizeof(double) * (size_t)n * n);
  const int crow = (d->env_kind == 1 || d->env_kind == 2 || d->env_kind == 3) ? 6 : 2;
  int pos[CPL_MAX_CONTACTS];
  for (int k = 0; k < N; ++k) pos[d->map_order[k]] = k;
  for (int a = 0; a < 3; ++a) H[a * n + a] = 0.0 + (zero_cost ? 0.0 : d->W_com);
  for (int i = 0; i < N; ++i)
    for (int a = 0; a < 3; ++a) {
      const int f = 3 + 9 * i + a, p = 6 + 9 * i + a, q = 9 + 9 * i + a;
      H[f * n + f] = 0.0 + (zero_cost ? 0.0 : d->W_F[i]);
      H[p * n + p] = 0.0 + (zero_cost ? 0.0 : d->W_p[i]);
      H[q * n + q] = 0.0 + 0.0;
    }
#define EPS_AC(a, c) ((a) == (c) ? 0.0 : (((a) + 1) % 3 == (c) ? 1.0 : -1.0) * Y[3 + (3 - (a) - (c))])
  for (int i = 0; i < N; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        const int Fb = 3 + 9 * i + b, pa = 6 + 9 * i + a, ca = a;
        const double e = EPS_AC(a, b);
        H[pa * n + Fb] = 0.0 + e;
        H[Fb * n + pa] = 0.0 + e;
        H[ca * n + Fb] = 0.0 - e;
        H[Fb * n + ca] = 0.0 - e;
      }
#undef EPS_AC
  const double mu = d->mu;
  for (int i = 0; i < N; ++i) {
    const double* q = X + 3 + 9 * i;
    const double F[3] = {q[0], q[1], q[2]}, nn[3] = {q[6], q[7], q[8]};
    const int r0 = 6 + crow * pos[i] + (crow - 2);
    const double y0 = Y[r0], y1 = Y[r0 + 1];
    const double sdot = (F[0] * nn[0] + F[1] * nn[1]) + F[2] * nn[2];
    double t[3], u[3];
    for (int j = 0; j < 3; ++j) t[j] = F[j] - sdot * nn[j];
    const double rr = sqrt((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
    const int ok = rr > 0.0 && rr < INFINITY && y1 != 0.0;
    for (int j = 0; j < 3; ++j) u[j] = t[j] / rr;
    for (int u6 = 0; u6 < 6; ++u6)
      for (int v6 = 0; v6 < 6; ++v6) {
        const int ku = u6 < 3 ? 1 : 3, au = u6 < 3 ? u6 : u6 - 3;
        const int kv = v6 < 3 ? 1 : 3, av = v6 < 3 ? v6 : v6 - 3;
        const int uu = 3 + 9 * i + (u6 < 3 ? u6 : 3 + u6), vv = 3 + 9 * i + (v6 < 3 ? v6 : 3 + v6);
        double h = H[uu * n + vv];
        const int fn = (ku == 1 && kv == 3) || (ku == 3 && kv == 1);
        const int aF = ku == 1 ? au : av, an = ku == 3 ? au : av;
        if (fn && aF == an) h = h - (y0 + mu * y1);
        double cu[3], cv[3];
        for (int j = 0; j < 3; ++j) {
          cu[j] = ku == 1 ? (j == au ? 1.0 : 0.0) - nn[j] * nn[au] : -(nn[j] * F[au] + (j == au ? sdot : 0.0));
          cv[j] = kv == 1 ? (j == av ? 1.0 : 0.0) - nn[j] * nn[av] : -(nn[j] * F[av] + (j == av ? sdot : 0.0));
        }
        const double jj = (cu[0] * cv[0] + cu[1] * cv[1]) + cu[2] * cv[2];
        const double pu = (u[0] * cu[0] + u[1] * cu[1]) + u[2] * cu[2];
        const double pv = (u[0] * cv[0] + u[1] * cv[1]) + u[2] * cv[2];
        double second = 0.0;
        if (fn) {
          const double un = (u[0] * nn[0] + u[1] * nn[1]) + u[2] * nn[2];
          second = -((aF == an ? un : 0.0) + nn[aF] * u[an]);
        } else if (ku == 3 && kv == 3) {
          second = -(F[au] * u[av] + F[av] * u[au]);
        }
        H[uu * n + vv] = ok ? h + y1 * ((jj - pu * pv) / rr + second) : h;
      }
  }
  for (int a = 0; a < P->nf; ++a)
    for (int b = 0; b < P->nf; ++b) Hf[a * P->nf + b] = H[P->free_idx[a] * n + P->free_idx[b]];
}

/* ---- dense linear algebra (row-major) ------------------------------------------------------- */
/* Cholesky K = L L^T in place (lower), returns 0, or 1 if a pivot is <= piv_tol (or not positive) */
static int cholesky(double* K, int n, double piv_tol) {
  for (int j = 0; j < n; ++j) {
    double s = K[j * n + j];
    for (int k = 0; k < j; ++k) s -= K[j * n + k] * K[j * n + k];
    if (!(s > 0.0) || s <= piv_tol) return 1;
    const double ljj = sqrt(s);
    K[j * n + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double t = K[i * n + j];
      for (int k = 0; k < j; ++k) t -= K[i * n + k] * K[j * n + k];
      K[i * n + j] = t / ljj;
    }
  }
  return 0;
}
static void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
    b[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
    b[i] = s / L[i * n + i];
  }
}
/* Cholesky of K + delta_w I with IPOPT's inertia-correction schedule (first 1e-4 or dwl / 3, growth
 * x100 / x8); pivots at or below PIVOT_REL max|K_ii| count as zero eigenvalues */
static double chol_inertia(const double* K, int n, double dwl, double* L) {
  double dmx = 0.0;
  for (int i = 0; i < n; ++i) dmx = dmax(dmx, fabs(K[i * n + i]));
  const double piv_tol = PIVOT_REL * dmx;
  double delta = 0.0;
  for (int it = 0; it < 65; ++it) {
    memcpy(L, K, sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) L[i * n + i] += delta;
    if (!cholesky(L, n, piv_tol)) return delta;
    const double first = dwl == 0.0 ? 1e-4 : dmax(dwl / 3.0, 1e-20);
    delta = delta == 0.0 ? first : delta * (dwl == 0.0 ? 100.0 : 8.0);
  }
  return delta;
}

/* The Newton step's factors (null-space method on a Householder QR of A^T): kept for the
 * second-order corrections' re-solves */
typedef struct {
  int nw, m, nz;
  double Q[NWMAX * NWMAX]; /* nw x nw, columns: Y (m) | Z (nz) */
  double R[MMAX * MMAX];   /* m x m upper */
  double L[NWMAX * NWMAX]; /* nz x nz Cholesky of Z^T (M + dW I) Z */
  double Mw[NWMAX * NWMAX];
  double A[MMAX * NWMAX];
  int rank_def;
  int aug, nw0;  /* (g_jac_reg) the regularised system of a rank-deficient A, in nw0 + m unknowns */
} Kkt;

/* IPOPT's regularisation of a rank-deficient Jacobian (PDPerturbationHandler: delta_c =
 * jacobian_regularization_value 1e-8 * mu^jacobian_regularization_exponent 0.25 on the (2,2) block):
 * [[W + dW I, A^T], [A, -delta_c I]] — solved by the same null-space method as the augmented system in
 * (dw, s): W~ = diag(W, I), A~ = [A, -sqrt(delta_c) I] (full row rank), whose KKT conditions are exactly
 * the regularised system's (s = sqrt(delta_c) dy).  Opt-in (cplo_set_jac_reg): the default keeps the
 * engine's treatment (delta_c added to R's near-zero pivots). */
static int g_jac_reg = 0;
void cplo_set_jac_reg(int on) { g_jac_reg = on != 0; }

/* Householder QR of At (nw x m): Q (nw x nw) and R (m x m) */
static void householder_qr(const double* At, int nw, int m, double* Q, double* R) {
  static __thread double Wk[NWMAX * MMAX];
  memcpy(Wk, At, sizeof(double) * (size_t)nw * m);
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < nw; ++j) Q[i * nw + j] = i == j ? 1.0 : 0.0;
  double v[NWMAX];
  for (int j = 0; j < m; ++j) {
    double nrm = 0.0;
    for (int i = j; i < nw; ++i) nrm += Wk[i * m + j] * Wk[i * m + j];
    nrm = sqrt(nrm);
    if (nrm == 0.0) continue;
    const double alpha = Wk[j * m + j] > 0.0 ? -nrm : nrm;
    for (int i = 0; i < nw; ++i) v[i] = i < j ? 0.0 : Wk[i * m + j];
    v[j] -= alpha;
    double vv = 0.0;
    for (int i = j; i < nw; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;
    const double beta = 2.0 / vv;
    for (int c = j; c < m; ++c) {  /* W <- (I - beta v v^T) W */
      double s = 0.0;
      for (int i = j; i < nw; ++i) s += v[i] * Wk[i * m + c];
      s *= beta;
      for (int i = j; i < nw; ++i) Wk[i * m + c] -= s * v[i];
    }
    for (int r = 0; r < nw; ++r) {  /* Q <- Q (I - beta v v^T) */
      double s = 0.0;
      for (int i = j; i < nw; ++i) s += Q[r * nw + i] * v[i];
      s *= beta;
      for (int i = j; i < nw; ++i) Q[r * nw + i] -= s * v[i];
    }
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) R[i * m + j] = j >= i ? Wk[i * m + j] : 0.0;
}

/* factorise: QR of A^T, delta_c on R's small diagonal, the reduced Hessian with the inertia test */
static double kkt_factor(Kkt* k, const double* M, const double* A, int nw, int m, double mu, double dwl) {
  static __thread double At[NWMAX * MMAX];
  static __thread double Ma[NWMAX * NWMAX];
  k->nw = nw; k->m = m; k->nz = nw - m; k->aug = 0; k->nw0 = nw;
  memcpy(k->A, A, sizeof(double) * (size_t)m * nw);
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < m; ++j) At[i * m + j] = A[j * nw + i];
  householder_qr(At, nw, m, k->Q, k->R);
  double rmax = 0.0;
  for (int i = 0; i < m; ++i) rmax = dmax(rmax, fabs(k->R[i * m + i]));
  const double dc = 1e-8 * pow(mu, 0.25) * (rmax > 0.0 ? rmax : 1.0);
  k->rank_def = 0;
  for (int i = 0; i < m; ++i) {
    double* rd = &k->R[i * m + i];
    if (!(fabs(*rd) >= 1e-10 * rmax) || rmax == 0.0) {
      k->rank_def = 1;
      if (!g_jac_reg) *rd += *rd < 0.0 ? -dc : dc;
    }
  }
  const double* Mr = M;
  if (k->rank_def && g_jac_reg && nw + m <= NWMAX) {  /* the regularised system as the augmented one */
    const int na = nw + m;
    const double sdc = sqrt(1e-8 * pow(mu, 0.25));
    for (int i = 0; i < na; ++i)
      for (int j = 0; j < m; ++j) At[i * m + j] = i < nw ? A[j * nw + i] : (i - nw == j ? -sdc : 0.0);
    householder_qr(At, na, m, k->Q, k->R);
    for (int r = 0; r < m; ++r)
      for (int j = 0; j < na; ++j) k->A[r * na + j] = j < nw ? A[r * nw + j] : (j - nw == r ? -sdc : 0.0);
    for (int i = 0; i < na; ++i)
      for (int j = 0; j < na; ++j) Ma[i * na + j] = (i < nw && j < nw) ? M[i * nw + j] : (i == j ? 1.0 : 0.0);
    k->aug = 1; k->rank_def = 0;
    nw = na; k->nw = na; k->nz = na - m;
    Mr = Ma;
  }
  const int nz = k->nz;
  double dmx = 0.0;
  for (int i = 0; i < nw; ++i) dmx = dmax(dmx, fabs(Mr[i * nw + i]));
  /* Hr = Z^T M Z, symmetrised */
  static __thread double MZ[NWMAX * NWMAX], Hr[NWMAX * NWMAX], Pz[NWMAX * NWMAX];
  for (int i = 0; i < nw; ++i)
    for (int c = 0; c < nz; ++c) {
      double s = 0.0;
      for (int t = 0; t < nw; ++t) s += Mr[i * nw + t] * k->Q[t * nw + m + c];
      MZ[i * nz + c] = s;
    }
  for (int a = 0; a < nz; ++a)
    for (int b = 0; b < nz; ++b) {
      double s = 0.0;
      for (int t = 0; t < nw; ++t) s += k->Q[t * nw + m + a] * MZ[t * nz + b];
      Hr[a * nz + b] = s;
    }
  for (int a = 0; a < nz; ++a)
    for (int b = a + 1; b < nz; ++b) {
      const double s = 0.5 * (Hr[a * nz + b] + Hr[b * nz + a]);
      Hr[a * nz + b] = Hr[b * nz + a] = s;
    }
  if (k->aug)  /* dW acts on W only: Z~^T diag(I, 0) Z~ */
    for (int a = 0; a < nz; ++a)
      for (int b = 0; b < nz; ++b) {
        double s = 0.0;
        for (int t = 0; t < k->nw0; ++t) s += k->Q[t * nw + m + a] * k->Q[t * nw + m + b];
        Pz[a * nz + b] = s;
      }
  double delta = 0.0;
  if (nz) {
    const double piv_tol = PIVOT_REL * dmx;
    for (int it = 0; it < 65; ++it) {
      memcpy(k->L, Hr, sizeof(double) * (size_t)nz * nz);
      if (k->aug)
        for (int a = 0; a < nz; ++a)
          for (int b = 0; b < nz; ++b) k->L[a * nz + b] += delta * Pz[a * nz + b];
      else
        for (int i = 0; i < nz; ++i) k->L[i * nz + i] += delta;
      if (!cholesky(k->L, nz, piv_tol)) break;
      const double first = dwl == 0.0 ? 1e-4 : dmax(dwl / 3.0, 1e-20);
      delta = delta == 0.0 ? first : delta * (dwl == 0.0 ? 100.0 : 8.0);
    }
  }
  memcpy(k->Mw, Mr, sizeof(double) * (size_t)nw * nw);
  for (int i = 0; i < (k->aug ? k->nw0 : nw); ++i) k->Mw[i * nw + i] += delta;
  return delta;
}

static void kkt_solve_once(const Kkt* k, const double* q1, const double* q2, double* dw, double* dy) {
  const int nw = k->nw, m = k->m, nz = k->nz;
  double py[MMAX], t[NWMAX], pz[NWMAX];
  for (int i = 0; i < m; ++i) {  /* R^T py = q2 */
    double s = q2[i];
    for (int j = 0; j < i; ++j) s -= k->R[j * m + i] * py[j];
    py[i] = s / k->R[i * m + i];
  }
  for (int i = 0; i < nw; ++i) {
    double s = 0.0;
    for (int j = 0; j < m; ++j) s += k->Q[i * nw + j] * py[j];
    dw[i] = s;
  }
  if (nz) {
    for (int i = 0; i < nw; ++i) {
      double s = 0.0;
      for (int j = 0; j < nw; ++j) s += k->Mw[i * nw + j] * dw[j];
      t[i] = q1[i] - s;
    }
    for (int a = 0; a < nz; ++a) {
      double s = 0.0;
      for (int i = 0; i < nw; ++i) s += k->Q[i * nw + m + a] * t[i];
      pz[a] = s;
    }
    chol_solve(k->L, nz, pz);
    for (int i = 0; i < nw; ++i) {
      double s = 0.0;
      for (int a = 0; a < nz; ++a) s += k->Q[i * nw + m + a] * pz[a];
      dw[i] += s;
    }
  }
  for (int i = 0; i < nw; ++i) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += k->Mw[i * nw + j] * dw[j];
    t[i] = q1[i] - s;
  }
  double u[MMAX];
  for (int j = 0; j < m; ++j) {
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += k->Q[i * nw + j] * t[i];
    u[j] = s;
  }
  for (int i = m - 1; i >= 0; --i) {  /* R dy = Y^T (q1 - Mw dw) */
    double s = u[i];
    for (int j = i + 1; j < m; ++j) s -= k->R[i * m + j] * dy[j];
    dy[i] = s / k->R[i * m + i];
  }
}
/* one refinement step when A has full rank */
static void kkt_solve_full(const Kkt* k, const double* q1, const double* q2, double* dw, double* dy);
static void kkt_solve(const Kkt* k, const double* q1, const double* q2, double* dw, double* dy) {
  if (k->aug) {  /* the augmented system: q1~ = [q1; 0], dw = the first nw0 unknowns */
    double qa[NWMAX], da[NWMAX];
    for (int i = 0; i < k->nw; ++i) qa[i] = i < k->nw0 ? q1[i] : 0.0;
    kkt_solve_full(k, qa, q2, da, dy);
    memcpy(dw, da, sizeof(double) * (size_t)k->nw0);
    return;
  }
  kkt_solve_full(k, q1, q2, dw, dy);
}
static void kkt_solve_full(const Kkt* k, const double* q1, const double* q2, double* dw, double* dy) {
  const int nw = k->nw, m = k->m;
  kkt_solve_once(k, q1, q2, dw, dy);
  if (k->rank_def) return;
  double e1[NWMAX] = {0}, e2[MMAX] = {0}, c1[NWMAX], c2[MMAX];
  for (int i = 0; i < nw; ++i) {
    double s = q1[i];
    for (int j = 0; j < nw; ++j) s -= k->Mw[i * nw + j] * dw[j];
    for (int r = 0; r < m; ++r) s -= k->A[r * nw + i] * dy[r];
    e1[i] = s;
  }
  for (int r = 0; r < m; ++r) {
    double s = q2[r];
    for (int j = 0; j < nw; ++j) s -= k->A[r * nw + j] * dw[j];
    e2[r] = s;
  }
  kkt_solve_once(k, e1, e2, c1, c2);
  for (int i = 0; i < nw; ++i) dw[i] += c1[i];
  for (int r = 0; r < m; ++r) dy[r] += c2[r];
}

/* the restoration phase's quasi-definite system: K = W + A^T Dinv A by Cholesky with the inertia
 * correction; dw = K^-1 (r1 + A^T Dinv r2), dy = Dinv (A dw - r2) */
static double kkt_qd(const double* W, const double* A, const double* Dinv, const double* r1, const double* r2,
                     int nw, int m, double dwl, double* dw, double* dy) {
  static __thread double K[NWMAX * NWMAX], L[NWMAX * NWMAX];
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < nw; ++j) {
      double s = 0.0;
      for (int r = 0; r < m; ++r) s += A[r * nw + i] * Dinv[r] * A[r * nw + j];
      K[i * nw + j] = W[i * nw + j] + s;
    }
  for (int i = 0; i < nw; ++i)
    for (int j = i + 1; j < nw; ++j) {
      const double s = 0.5 * (K[i * nw + j] + K[j * nw + i]);
      K[i * nw + j] = K[j * nw + i] = s;
    }
  const double delta = chol_inertia(K, nw, dwl, L);
  for (int i = 0; i < nw; ++i) {
    double s = r1[i];
    for (int r = 0; r < m; ++r) s += A[r * nw + i] * Dinv[r] * r2[r];
    dw[i] = s;
  }
  chol_solve(L, nw, dw);
  for (int r = 0; r < m; ++r) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += A[r * nw + j] * dw[j];
    dy[r] = Dinv[r] * (s - r2[r]);
  }
  return delta;
}

/* ---- IPOPT's filter line-search acceptance ------------------------------------------------- */
typedef struct {
  double t[FMAX], p[FMAX];
  long cnt;
} Filter;
static void filter_reset(Filter* F) {
  for (int k = 0; k < FMAX; ++k) F->t[k] = F->p[k] = INFINITY;
  F->cnt = 0;
}
static void filter_add(Filter* F, double th, double ph) {
  const int slot = (int)(F->cnt % FMAX);
  F->t[slot] = (1.0 - GAMMA_TH) * th;
  F->p[slot] = ph - GAMMA_PHI * th;
  F->cnt += 1;
}
/* (ok, h_type) — batch_ipm.py acceptable(); switch_ok = theta_k <= theta_min */
static int acceptable(double th, double ph, double tk, double pk, double gd, double al, int switch_ok,
                      double theta_max, const Filter* F, int from_resto, int* h_type) {
  const int fin = isfinite(ph) && isfinite(th);
  int in_filter = 1;
  for (int k = 0; k < FMAX; ++k)
    if (!((th <= F->t[k]) || (ph <= F->p[k]))) in_filter = 0;
  const int is_ftype = gd < 0.0 && al * pow(gd < 0.0 ? -gd : 0.0, S_PHI) > DELTA_SW * pow(tk, S_TH);
  const int ftype = is_ftype && switch_ok;
  const double ro_p = 10.0 * EPS * fabs(pk), ro_t = 10.0 * EPS * fabs(tk);
  int armijo = (ph - pk) - ETA_PHI * al * gd <= ro_p;
  int suff = (th - (1.0 - GAMMA_TH) * tk <= ro_t) || ((ph - pk) - (-GAMMA_PHI * tk) <= ro_p);
  if (!from_resto) {
    const double base = fabs(pk) > 10.0 ? log10(fabs(pk)) : 1.0;
    const double inc = ph - pk;
    if (inc > 0 && log10(inc) > OBJ_MAX_INC + base) armijo = suff = 0;
  }
  if (h_type) *h_type = !(is_ftype && armijo);
  return fin && th <= theta_max && in_filter && (ftype ? armijo : suff);
}
static double max_step(const double* v, const double* dv, const unsigned char* has, const double* lo, int n,
                       double tau) {
  double r = INFINITY;
  for (int i = 0; i < n; ++i)
    if (has[i] && dv[i] < 0.0) r = dmin(r, -tau * (v[i] - (lo ? lo[i] : 0.0)) / dv[i]);
  return dmin(r, 1.0);
}
static double max_step_all(const double* v, const double* dv, int n, double tau) {
  double r = INFINITY;
  for (int i = 0; i < n; ++i)
    if (dv[i] < 0.0) r = dmin(r, -tau * v[i] / dv[i]);
  return dmin(r, 1.0);
}
static double alpha_min_of(double theta_k, double gd, double theta_min) {
  if (!(gd < 0.0)) return ALPHA_MIN_FRAC * GAMMA_TH;
  double a = dmin(GAMMA_TH, GAMMA_PHI * theta_k / -gd);
  if (theta_k <= theta_min) a = dmin(a, DELTA_SW * pow(theta_k, S_TH) / pow(-gd, S_PHI));
  return ALPHA_MIN_FRAC * a;
}

/* ---- the solver state --------------------------------------------------------------------- */
typedef struct {
  double w[NWMAX], y[MMAX], zL[NWMAX], zU[NWMAX], mu;
  int active, status, iters, acc;
  Filter F;
  double dwl, d_inf;
  Eval cur;
  int tiny_last, tiny_flag, in_soft, soft_cnt;
  double Hq[NWMAX * NWMAX];
  double lm_s[LM_HIST][NWMAX], lm_y[LM_HIST][NWMAX];
  int lm_cnt, lm_skip;
  int resto;
  double wR[NWMAX], p[MMAX], nn[MMAX], zp[MMAX], zn[MMAX], zLR[NWMAX], zUR[NWMAX], muR;
  Filter FR;
  double th_o0, ph_o0, dwlR, thmaxR, thminR;
  int n_resto, resto_tight;
  double theta_max, theta_min;
  double best_w[NWMAX], best_f;
  double acc_w[NWMAX], acc_y[MMAX], acc_zL[NWMAX], acc_zU[NWMAX];  /* IPOPT's backup acceptable point */
  int has_acc;
  /* IPOPT's watchdog (cplo_set_watchdog): active, shortened-step count, trial iterations; the watchdog
   * iterate and its step, its line search's references (theta, barrier objective, grad phi^T dw),
   * its fraction-to-the-boundary step (alpha_primal_test) and optimality error (its values: g_wd_cur) */
  int in_wd, wd_cnt, wd_trial;
  double wd_w[NWMAX], wd_y[MMAX], wd_zL[NWMAX], wd_zU[NWMAX], wd_dw[NWMAX], wd_dy[MMAX], wd_dzL[NWMAX], wd_dzU[NWMAX];
  double wd_th, wd_ph, wd_gd, wd_alpha;
} State;

typedef struct {
  double A[MMAX * NWMAX], gw[NWMAX], c[MMAX], d_inf, c_inf, base, cl[NWMAX], cu[NWMAX], sc, err0;
} Errors;

static void errors(const Prob* P, const Eval* o, const double* w, const double* y, const double* zl,
                   const double* zu, Errors* E) {
  const int nw = P->nw, m = P->m, nf = P->nf;
  jac_w(P, o->J, E->A);
  for (int k = 0; k < nw; ++k) E->gw[k] = k < nf ? o->grad[P->free_idx[k]] : 0.0;
  cons(P, o->g, w, E->c);
  double dinf = 0.0, zs = 0.0, ys = 0.0;
  for (int k = 0; k < nw; ++k) {
    double s = E->gw[k];
    for (int r = 0; r < m; ++r) s += E->A[r * nw + k] * y[r];
    s = s - zl[k] + zu[k];
    dinf = dmax(dinf, fabs(s));
    E->cl[k] = P->hasL[k] ? (w[k] - P->wl0[k]) * zl[k] : 0.0;
    E->cu[k] = P->hasU[k] ? (P->wu0[k] - w[k]) * zu[k] : 0.0;
    zs += fabs(zl[k]) + fabs(zu[k]);
  }
  ys = sum_abs(y, m);
  const double s_max = 100.0;
  const double sd = dmax((ys + zs) / (double)(m + P->nbounds > 1 ? m + P->nbounds : 1), s_max) / s_max;
  E->sc = dmax(zs / (double)(P->nbounds > 1 ? P->nbounds : 1), s_max) / s_max;
  E->d_inf = dinf;
  E->c_inf = m ? max_abs(E->c, m) : 0.0;
  E->base = dmax(dinf / sd, E->c_inf);
  double cm = 0.0;
  for (int k = 0; k < nw; ++k) cm = dmax(cm, dmax(E->cl[k], E->cu[k]));
  E->err0 = dmax(E->base, cm / E->sc);
}
static double err_mu(const Prob* P, const Errors* E, double mu) {
  double cm = 0.0;
  for (int k = 0; k < P->nw; ++k) {
    if (P->hasL[k]) cm = dmax(cm, fabs(E->cl[k] - mu));
    else cm = dmax(cm, fabs(E->cl[k]));
    if (P->hasU[k]) cm = dmax(cm, fabs(E->cu[k] - mu));
    else cm = dmax(cm, fabs(E->cu[k]));
  }
  return dmax(E->base, cm / E->sc);
}
static double pd_error(const Prob* P, const Eval* o, const double* w, const double* y, const double* zl,
                       const double* zu, double mu) {
  const int nw = P->nw, m = P->m, nf = P->nf;
  static __thread double A[MMAX * NWMAX];
  double c[MMAX];
  jac_w(P, o->J, A);
  cons(P, o->g, w, c);
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0;
  for (int k = 0; k < nw; ++k) {
    double s = k < nf ? o->grad[P->free_idx[k]] : 0.0;
    for (int r = 0; r < m; ++r) s += A[r * nw + k] * y[r];
    s = s - zl[k] + zu[k];
    s1 += fabs(s);
    s3 += P->hasL[k] ? fabs((w[k] - P->wl0[k]) * zl[k] - mu) : 0.0;
    s4 += P->hasU[k] ? fabs((P->wu0[k] - w[k]) * zu[k] - mu) : 0.0;
  }
  s2 = sum_abs(c, m);
  return s1 + s2 + s3 + s4;
}

static void lbfgs_reset(const Prob* P, State* S) {
  const int nf = P->nf;
  S->lm_skip = 0;
  S->lm_cnt = 0;
  for (int i = 0; i < nf; ++i)
    for (int j = 0; j < nf; ++j) S->Hq[i * nf + j] = i == j ? 1.0 : 0.0;
}
/* IPOPT's LimMemQuasiNewtonUpdater with IFOPT's defaults; yk from both Lagrangian gradients at y_new
 * (with_grad = 0: J^T y alone, the restoration phase's constraint curvature) */
static void lbfgs_update(const Prob* P, State* S, const double* sk, const Eval* nw_, const Eval* cur,
                         const double* y_new, int with_grad) {
  if (P->exact) return;
  const int nf = P->nf, m = P->m, n = P->n;
  double yk[NWMAX];
  for (int k = 0; k < nf; ++k) {
    const int j = P->free_idx[k];
    double a = with_grad ? nw_->grad[j] : 0.0, b = with_grad ? cur->grad[j] : 0.0;
    for (int r = 0; r < m; ++r) {
      a += nw_->J[r * n + j] * y_new[r];
      b += cur->J[r * n + j] * y_new[r];
    }
    yk[k] = a - b;
  }
  double sy = 0.0, ss = 0.0, yy = 0.0;
  for (int k = 0; k < nf; ++k) { sy += sk[k] * yk[k]; ss += sk[k] * sk[k]; yy += yk[k] * yk[k]; }
  const int take = sy > sqrt(EPS) * sqrt(ss) * sqrt(yy);
  if (!take) {
    const int skipped = S->lm_skip + 1;
    if (skipped > LM_MAX_SKIP) lbfgs_reset(P, S);
    else S->lm_skip = skipped;
    return;
  }
  S->lm_skip = 0;
  if (S->lm_cnt == LM_HIST) {  /* drop the oldest pair */
    for (int j = 0; j < LM_HIST - 1; ++j) {
      memcpy(S->lm_s[j], S->lm_s[j + 1], sizeof(double) * (size_t)nf);
      memcpy(S->lm_y[j], S->lm_y[j + 1], sizeof(double) * (size_t)nf);
    }
  }
  const int last = S->lm_cnt < LM_HIST ? S->lm_cnt : LM_HIST - 1;
  memcpy(S->lm_s[last], sk, sizeof(double) * (size_t)nf);
  memcpy(S->lm_y[last], yk, sizeof(double) * (size_t)nf);
  S->lm_cnt = last + 1;
  double sigma = sy / (ss > 0.0 ? ss : 1.0);
  sigma = dmin(dmax(sigma, 1e-8), 1e8);
  double* H = S->Hq;
  for (int i = 0; i < nf; ++i)
    for (int j = 0; j < nf; ++j) H[i * nf + j] = i == j ? sigma : 0.0;
  double Hs[NWMAX];
  for (int p = 0; p < S->lm_cnt; ++p) {
    const double* sj = S->lm_s[p];
    const double* yj = S->lm_y[p];
    double sHs = 0.0, sjy = 0.0;
    for (int i = 0; i < nf; ++i) {
      double t = 0.0;
      for (int j = 0; j < nf; ++j) t += H[i * nf + j] * sj[j];
      Hs[i] = t;
    }
    for (int i = 0; i < nf; ++i) { sHs += sj[i] * Hs[i]; sjy += sj[i] * yj[i]; }
    if (!(sHs > 0.0)) continue;
    for (int i = 0; i < nf; ++i)
      for (int j = 0; j < nf; ++j) H[i * nf + j] = (H[i * nf + j] - Hs[i] * Hs[j] / sHs) + yj[i] * yj[j] / sjy;
  }
}

static void push(const Prob* P, double* v) {  /* bound_push = bound_frac = 1e-2 */
  const double k = 1e-2;
  for (int i = 0; i < P->nw; ++i) {
    const double rng = (P->hasL[i] && P->hasU[i]) ? P->wu0[i] - P->wl0[i] : INFINITY;
    const double pl = dmin(k * dmax(fabs(P->wl0[i]), 1.0), k * rng);
    const double pu = dmin(k * dmax(fabs(P->wu0[i]), 1.0), k * rng);
    if (P->hasL[i]) v[i] = dmax(v[i], P->wl0[i] + pl);
    if (P->hasU[i]) v[i] = dmin(v[i], P->wu0[i] - pu);
  }
}

typedef struct {
  double tol, acceptable_tol, mu_min, fallback_viol_tol;
  int acceptable_iter, max_ls, max_soc;
} Opts;

/* the violation of the ORIGINAL constraints: g holds the scaled values dc g on a scaled solve */
static double orig_violation(const Prob* P, const double* g) {
  double v = 0.0;
  for (int r = 0; r < P->m; ++r) {
    const double gv = P->scaled ? g[r] / P->dc[r] : g[r];
    if (gv != gv) return INFINITY;
    v = dmax(v, dmax(dmax(P->gl[r] - gv, gv - P->gu[r]), 0.0));
  }
  return v;
}

static void check(State* S, const Errors* E, const Opts* o) {
  const double e0 = E->err0;
  const int done = e0 <= o->tol;
  S->acc = e0 <= o->acceptable_tol ? S->acc + 1 : 0;
  const int accn = !done && S->acc >= o->acceptable_iter;
  if (done) S->status = ST_OPTIMAL;
  else if (accn) S->status = ST_ACCEPTABLE;
  if (done || accn) S->active = 0;
  S->d_inf = E->d_inf;
}

static void enter_resto(const Prob* P, State* S, const double* c, const double* A, double f0) {
  const int nw = P->nw, m = P->m, nf = P->nf;
  const double c_inf = m ? max_abs(c, m) : 0.0;
  const double muR = dmax(S->mu, c_inf);
  for (int r = 0; r < m; ++r) {
    const double a = (muR - RHO_R * c[r]) / (2.0 * RHO_R);
    S->nn[r] = a + sqrt(a * a + muR * c[r] / (2.0 * RHO_R));
    S->p[r] = c[r] + S->nn[r];
    S->zp[r] = muR / S->p[r];
    S->zn[r] = muR / S->nn[r];
  }
  for (int k = 0; k < nw; ++k) {
    S->zLR[k] = P->hasL[k] ? dmin(S->zL[k], RHO_R) : 0.0;
    S->zUR[k] = P->hasU[k] ? dmin(S->zU[k], RHO_R) : 0.0;
    S->wR[k] = S->w[k];
  }
  /* least-squares multipliers: the p / n-eliminated system with W = I, Sigma_p = Sigma_n = 1 */
  static __thread double Wi[NWMAX * NWMAX];
  double Dinv[MMAX], r1[NWMAX], r2[MMAX], dw[NWMAX], yR[MMAX];
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < nw; ++j) Wi[i * nw + j] = i == j ? 1.0 : 0.0;
  for (int r = 0; r < m; ++r) { Dinv[r] = 0.5; r2[r] = S->zp[r] - S->zn[r]; }
  for (int k = 0; k < nw; ++k) r1[k] = S->zLR[k] - S->zUR[k];
  kkt_qd(Wi, A, Dinv, r1, r2, nw, m, 0.0, dw, yR);
  const double ymx = max_abs(yR, m);
  for (int r = 0; r < m; ++r) S->y[r] = ymx <= 1e3 ? yR[r] : 0.0;
  double thR0 = 0.0;
  for (int r = 0; r < m; ++r) thR0 += fabs(c[r] - S->p[r] + S->nn[r]);
  S->resto = 1;
  S->n_resto += 1;
  S->muR = muR;
  filter_reset(&S->FR);
  S->thmaxR = 1e4 * dmax(thR0, 1.0);
  S->thminR = 1e-4 * dmax(thR0, 1.0);
  S->th_o0 = sum_abs(c, m);
  S->ph_o0 = f0 + barrier(P, S->w, S->mu);
  S->dwlR = 0.0;
  (void)nf;
  lbfgs_reset(P, S);
}

static void leave_resto(const Prob* P, State* S, const double* w_new) {
  const int nw = P->nw, m = P->m;
  const double mu = S->mu, tau = dmax(1.0 - mu, 0.99);
  double dzL[NWMAX], dzU[NWMAX];
  double ad = INFINITY;
  for (int k = 0; k < nw; ++k) {
    dzL[k] = dzU[k] = 0.0;
    if (P->hasL[k]) {
      const double s0 = S->wR[k] - P->wl0[k], s1 = w_new[k] - P->wl0[k];
      dzL[k] = (S->zL[k] * (s0 - s1) + mu) / s0 - S->zL[k];
      if (dzL[k] < 0.0) ad = dmin(ad, -tau * S->zL[k] / dzL[k]);
    }
    if (P->hasU[k]) {
      const double s0 = P->wu0[k] - S->wR[k], s1 = P->wu0[k] - w_new[k];
      dzU[k] = (S->zU[k] * (s0 - s1) + mu) / s0 - S->zU[k];
      if (dzU[k] < 0.0) ad = dmin(ad, -tau * S->zU[k] / dzU[k]);
    }
  }
  ad = dmin(ad, 1.0);
  double zmax = -INFINITY;
  for (int k = 0; k < nw; ++k) {
    if (P->hasL[k]) S->zL[k] += ad * dzL[k];
    if (P->hasU[k]) S->zU[k] += ad * dzU[k];
    zmax = dmax(zmax, dmax(S->zL[k], S->zU[k]));
  }
  if (zmax > BOUND_MULT_RESET)
    for (int k = 0; k < nw; ++k) {
      if (P->hasL[k]) S->zL[k] = 1.0;
      if (P->hasU[k]) S->zU[k] = 1.0;
    }
  for (int r = 0; r < m; ++r) S->y[r] = 0.0;
  S->resto = 0;
  S->acc = 0;
  lbfgs_reset(P, S);
}

/* One regular iteration (batch_ipm.py regular_step) */
/* IPOPT's watchdog (BacktrackingLineSearch: watchdog_shortened_iter_trigger 10, watchdog_trial_iter_max 3),
 * opt-in here (cplo_set_watchdog; the device engine and batch_ipm.py have none): after 10 consecutive
 * iterations whose step the line search shortened, the iterate and its step are kept and the next
 * iterations take the full step of their own direction, judged against the kept iterate's references
 * (theta, barrier objective, grad phi^T dw, its alpha_max as the switching condition's alpha); a full
 * step acceptable to them ends the watchdog; otherwise the step is taken anyway, up to 3 times, after
 * which the kept iterate is restored and searched along its own step from alpha_max / 2 (no
 * second-order correction).  A barrier-parameter change ends the watchdog (the line search's Reset).
 * IPOPT is absent offline: restated from its published method, parity unpinned. */
static int WD_TRIGGER = 10, WD_TRIAL_MAX = 3;  /* (cplo_set_watchdog_params: a lower trigger in the tests) */
static int g_watchdog = 0;
static int g_trace = -1;  /* CPLO_TRACE set: one line per regular iteration on stderr */
void cplo_set_watchdog(int on) { g_watchdog = on != 0; }
void cplo_set_watchdog_params(int trigger, int trial_max) { WD_TRIGGER = trigger; WD_TRIAL_MAX = trial_max; }
static __thread Eval g_wd_cur;
/* this thread's watchdog events since the last read: starts, successes, restorations of the kept iterate */
static __thread long g_wd_events[3];
static __thread long g_resto_fail_events[2];  /* (cplo_resto_fail_events) */
void cplo_watchdog_events(long* out) {
  for (int k = 0; k < 3; ++k) { out[k] = g_wd_events[k]; g_wd_events[k] = 0; }
}

static void regular_step(Prob* P, State* S, const Errors* E, const Opts* o) {
  const int nw = P->nw, m = P->m, nf = P->nf;
  static __thread Kkt K;
  static __thread double M[NWMAX * NWMAX];
  static __thread Eval trial, tsoc, ev_new;
  double mu = S->mu;
  if (E->err0 <= o->acceptable_tol) {  /* StoreAcceptablePoint (CurrentIsAcceptable) */
    memcpy(S->acc_w, S->w, sizeof(double) * (size_t)nw);
    memcpy(S->acc_zL, S->zL, sizeof(double) * (size_t)nw);
    memcpy(S->acc_zU, S->zU, sizeof(double) * (size_t)nw);
    memcpy(S->acc_y, S->y, sizeof(double) * (size_t)m);
    S->has_acc = 1;
  }
  /* monotone barrier update (mu_allow_fast_monotone_decrease), the filter reset where mu changed */
  const int force = S->tiny_flag;
  for (int r = 0; r < MU_ROUNDS; ++r) {
    if (((err_mu(P, E, mu) <= BARRIER_TOL_FACTOR * mu) || (r == 0 && force)) && mu > o->mu_min) {
      mu = dmax(dmin(0.2 * mu, pow(mu, 1.5)), o->mu_min);
      filter_reset(&S->F);
      S->in_soft = 0;  /* BacktrackingLineSearch::Reset (MonotoneMuUpdate): the soft restoration phase ends */
      S->in_wd = 0;  /* (the line search's Reset: the watchdog ends, its count restarts) */
      S->wd_cnt = 0;
    }
  }
  const double tau = dmax(1.0 - mu, 0.99);
  const double* w = S->w;
  double dl[NWMAX], du[NWMAX], Sig[NWMAX], gphi[NWMAX], r1[NWMAX], r2[MMAX];
  for (int k = 0; k < nw; ++k) {
    dl[k] = P->hasL[k] ? w[k] - P->wl0[k] : 1.0;
    du[k] = P->hasU[k] ? P->wu0[k] - w[k] : 1.0;
    Sig[k] = (P->hasL[k] ? S->zL[k] / dl[k] : 0.0) + (P->hasU[k] ? S->zU[k] / du[k] : 0.0);
    gphi[k] = E->gw[k] - (P->hasL[k] ? mu / dl[k] : 0.0) + (P->hasU[k] ? mu / du[k] : 0.0);
  }
  for (int k = 0; k < nw; ++k) {
    double s = 0.0;
    for (int r = 0; r < m; ++r) s += E->A[r * nw + k] * S->y[r];
    r1[k] = -(gphi[k] + s);
  }
  for (int r = 0; r < m; ++r) r2[r] = -E->c[r];
  if (P->exact) {  /* the analytic Lagrangian Hessian at (w, y) in place of the model */
    double Xc[NMAX];
    unpack(P, w, Xc);
    double yr[MMAX];
    y_raw(P, S->y, yr);
    lagr_hessian(P, Xc, yr, 0, S->Hq);
    if (P->scaled)
      for (int q = 0; q < P->nf * P->nf; ++q) S->Hq[q] = S->Hq[q] * P->df;
  }
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < nw; ++j) M[i * nw + j] = (i == j ? Sig[i] : 0.0) + ((i < nf && j < nf) ? S->Hq[i * nf + j] : 0.0);
  const double theta_k = sum_abs(E->c, m);
  const double phi_k = S->cur.f + barrier(P, w, mu);
  double dw[NWMAX], dy[MMAX];
  const double delta_w = kkt_factor(&K, M, E->A, nw, m, mu, S->dwl);
  kkt_solve(&K, r1, r2, dw, dy);
  if (g_trace && getenv("CPLO_DUMP") && S->iters == atoi(getenv("CPLO_DUMP"))) {  /* (diagnostics) */
    FILE* fd = fopen("/tmp/cplo_dump.bin", "wb");
    if (fd) {
      fwrite(M, sizeof(double), (size_t)nw * nw, fd); fwrite(E->A, sizeof(double), (size_t)m * nw, fd);
      fwrite(r1, sizeof(double), (size_t)nw, fd); fwrite(r2, sizeof(double), (size_t)m, fd);
      fwrite(dw, sizeof(double), (size_t)nw, fd); fwrite(dy, sizeof(double), (size_t)m, fd);
      fwrite(S->w, sizeof(double), (size_t)nw, fd); fwrite(S->y, sizeof(double), (size_t)m, fd);
      fclose(fd);
    }
  }
  double dzL[NWMAX], dzU[NWMAX];
  for (int k = 0; k < nw; ++k) {
    dzL[k] = P->hasL[k] ? mu / dl[k] - S->zL[k] - S->zL[k] / dl[k] * dw[k] : 0.0;
    dzU[k] = P->hasU[k] ? mu / du[k] - S->zU[k] + S->zU[k] / du[k] * dw[k] : 0.0;
  }
  double mdw[NWMAX], mw[NWMAX], mwu[NWMAX];
  for (int k = 0; k < nw; ++k) { mdw[k] = -dw[k]; mw[k] = -w[k]; mwu[k] = -P->wu0[k]; }
  const double a_max = dmin(max_step(w, dw, P->hasL, P->wl0, nw, tau), max_step(mw, mdw, P->hasU, mwu, nw, tau));
  const double a_z = dmin(max_step(S->zL, dzL, P->hasL, NULL, nw, tau), max_step(S->zU, dzU, P->hasU, NULL, nw, tau));
  double gd = 0.0;
  for (int k = 0; k < nw; ++k) gd += gphi[k] * dw[k];
  const int switch_ok = theta_k <= S->theta_min;
  double rel = 0.0;
  for (int k = 0; k < nw; ++k) rel = dmax(rel, fabs(dw[k]) / (1.0 + fabs(w[k])));
  const int tiny = rel < TINY_STEP_TOL && max_abs(dy, m) < TINY_STEP_Y_TOL && E->c_inf < 1e-4;
  S->tiny_flag = tiny && S->tiny_last;
  S->tiny_last = tiny && !S->tiny_last;
  double a_min = alpha_min_of(theta_k, gd, S->theta_min);
  const int soft_now = S->in_soft && !tiny;
  S->soft_cnt += soft_now;
  int searching = !tiny && !soft_now, found = 0, aug = 0;
  double st_w[NWMAX], st_alpha = 0.0;
  memcpy(st_w, w, sizeof(double) * (size_t)nw);
  double wt[NWMAX], Xt[NMAX];
  double alpha = a_max;
  /* the line search's references: this iterate's, or the watchdog iterate's */
  double th_ref = theta_k, ph_ref = phi_k, gd_ref = gd;
  int sw_ref = switch_ok, ls0 = 0, n_steps = 0, max_soc = o->max_soc;
  double a_max_r = a_max, a_z_r = a_z;
  const int was_wd = g_watchdog && S->in_wd && searching;
  if (was_wd) {  /* one trial: the full step, judged against the watchdog iterate */
    th_ref = S->wd_th; ph_ref = S->wd_ph; gd_ref = S->wd_gd;
    sw_ref = S->wd_th <= S->theta_min;
    for (int k = 0; k < nw; ++k) wt[k] = w[k] + a_max * dw[k];
    unpack(P, wt, Xt);
    evaluate_fg(P, Xt, &trial.f, trial.g);
    double ct[MMAX];
    cons(P, trial.g, wt, ct);
    int h = 0;
    const int ok = acceptable(sum_abs(ct, m), trial.f + barrier(P, wt, mu), th_ref, ph_ref, gd_ref, S->wd_alpha, sw_ref,
                              S->theta_max, &S->F, 0, &h);
    searching = 0;
    if (ok || ++S->wd_trial <= WD_TRIAL_MAX) {  /* acceptable: the watchdog succeeded; else taken anyway */
      memcpy(st_w, wt, sizeof(double) * (size_t)nw);
      st_alpha = a_max; aug = h; found = 1;
      if (ok) { S->in_wd = 0; ++g_wd_events[1]; }
    } else {
      ++g_wd_events[2];  /* StopWatchDog: back to the watchdog iterate, a search along its step without the full one */
      S->in_wd = 0;
      S->wd_cnt = 0;
      memcpy(S->w, S->wd_w, sizeof(double) * (size_t)nw);
      memcpy(S->y, S->wd_y, sizeof(double) * (size_t)m);
      memcpy(S->zL, S->wd_zL, sizeof(double) * (size_t)nw);
      memcpy(S->zU, S->wd_zU, sizeof(double) * (size_t)nw);
      memcpy(dw, S->wd_dw, sizeof(double) * (size_t)nw);
      memcpy(dy, S->wd_dy, sizeof(double) * (size_t)m);
      memcpy(dzL, S->wd_dzL, sizeof(double) * (size_t)nw);
      memcpy(dzU, S->wd_dzU, sizeof(double) * (size_t)nw);
      S->cur = g_wd_cur;
      static __thread Errors Ew;
      errors(P, &S->cur, S->w, S->y, S->zL, S->zU, &Ew);
      E = &Ew;
      memcpy(st_w, w, sizeof(double) * (size_t)nw);
      for (int k = 0; k < nw; ++k) { mdw[k] = -dw[k]; mw[k] = -w[k]; }
      a_max_r = dmin(max_step(w, dw, P->hasL, P->wl0, nw, tau), max_step(mw, mdw, P->hasU, mwu, nw, tau));
      a_z_r = dmin(max_step(S->zL, dzL, P->hasL, NULL, nw, tau), max_step(S->zU, dzU, P->hasU, NULL, nw, tau));
      a_min = alpha_min_of(th_ref, gd_ref, S->theta_min);
      alpha = 0.5 * a_max_r;
      searching = alpha > a_min;
      ls0 = 1; n_steps = 1; max_soc = 0;
    }
  }
  for (int ls = ls0; ls < (o->max_ls > 1 ? o->max_ls : 1) && searching; ++ls) {
    for (int k = 0; k < nw; ++k) wt[k] = w[k] + alpha * dw[k];
    unpack(P, wt, Xt);
    evaluate_fg(P, Xt, &trial.f, trial.g);
    double ct[MMAX];
    cons(P, trial.g, wt, ct);
    double th = sum_abs(ct, m);
    double ph = trial.f + barrier(P, wt, mu);
    int h = 0;
    if (acceptable(th, ph, th_ref, ph_ref, gd_ref, alpha, sw_ref, S->theta_max, &S->F, 0, &h)) {
      memcpy(st_w, wt, sizeof(double) * (size_t)nw);
      st_alpha = alpha; aug = h; found = 1; searching = 0;
    }
    if (g_trace > 1)
      fprintf(stderr, "      [C] trial %d alpha=%.17g th=%.17g ph=%.17g found=%d th_k=%.17g ph_k=%.17g gd=%.17g a_min=%.17g\n", ls,
              alpha, th, ph, found, th_ref, ph_ref, gd_ref, a_min);
    if (ls == 0 && max_soc > 0 && searching && th >= theta_k) {  /* second-order corrections */
      double c_soc[MMAX], a_soc = alpha, th_old = th, dws[NWMAX], dys[MMAX], ws[NWMAX], Xs[NMAX];
      memcpy(c_soc, E->c, sizeof(double) * (size_t)m);
      int soc = 1;
      for (int q = 0; q < o->max_soc && soc; ++q) {
        double r2s[MMAX];
        for (int r = 0; r < m; ++r) { c_soc[r] = a_soc * c_soc[r] + ct[r]; r2s[r] = -c_soc[r]; }
        kkt_solve(&K, r1, r2s, dws, dys);
        for (int k = 0; k < nw; ++k) { mdw[k] = -dws[k]; }
        a_soc = dmin(max_step(w, dws, P->hasL, P->wl0, nw, tau), max_step(mw, mdw, P->hasU, mwu, nw, tau));
        for (int k = 0; k < nw; ++k) ws[k] = w[k] + a_soc * dws[k];
        unpack(P, ws, Xs);
        evaluate_fg(P, Xs, &tsoc.f, tsoc.g);
        double cs[MMAX];
        cons(P, tsoc.g, ws, cs);
        const double ths = sum_abs(cs, m);
        const double phs = tsoc.f + barrier(P, ws, mu);
        const int oks = acceptable(ths, phs, theta_k, phi_k, gd, alpha, switch_ok, S->theta_max, &S->F, 0, &h);
        if (g_trace > 1) fprintf(stderr, "      [C] soc %d a_soc=%.17g th=%.17g ph=%.17g ok=%d\n", q, a_soc, ths, phs, oks);
        if (oks) {
          memcpy(st_w, ws, sizeof(double) * (size_t)nw);
          st_alpha = alpha; aug = h; found = 1; searching = 0;
        }
        soc = !oks && ths <= KAPPA_SOC * th_old;
        th_old = ths;
        memcpy(ct, cs, sizeof(double) * (size_t)m);
      }
    }
    alpha = searching ? 0.5 * alpha : alpha;
    n_steps += searching;
    searching = searching && alpha > a_min;
  }
  if (g_watchdog && found) {  /* the shortened-step count; the watchdog starts at this iterate and step */
    S->wd_cnt = n_steps == 0 ? 0 : S->wd_cnt + 1;
    if (!S->in_wd && !soft_now && S->wd_cnt >= WD_TRIGGER) {
      ++g_wd_events[0];
      S->in_wd = 1;
      S->wd_trial = 0;
      memcpy(S->wd_w, w, sizeof(double) * (size_t)nw);
      memcpy(S->wd_y, S->y, sizeof(double) * (size_t)m);
      memcpy(S->wd_zL, S->zL, sizeof(double) * (size_t)nw);
      memcpy(S->wd_zU, S->zU, sizeof(double) * (size_t)nw);
      memcpy(S->wd_dw, dw, sizeof(double) * (size_t)nw);
      memcpy(S->wd_dy, dy, sizeof(double) * (size_t)m);
      memcpy(S->wd_dzL, dzL, sizeof(double) * (size_t)nw);
      memcpy(S->wd_dzU, dzU, sizeof(double) * (size_t)nw);
      g_wd_cur = S->cur;
      S->wd_th = th_ref; S->wd_ph = ph_ref; S->wd_gd = gd_ref; S->wd_alpha = a_max_r;
    }
  }
  if (tiny) {
    for (int k = 0; k < nw; ++k) st_w[k] = w[k] + a_max * dw[k];
    st_alpha = a_max;
  }
  /* soft restoration step */
  const int bt_failed = !tiny && !soft_now && !found;
  const int soft_try = (soft_now && S->soft_cnt <= MAX_SOFT_RESTO) || bt_failed;
  const double a_soft = dmin(a_max_r, a_z_r);
  int soft_ok = 0;
  if (soft_try) {
    double wsft[NWMAX], Xsft[NMAX], ys[MMAX], zLs[NWMAX], zUs[NWMAX], cs[MMAX];
    static __thread Eval os;
    for (int k = 0; k < nw; ++k) wsft[k] = w[k] + a_soft * dw[k];
    unpack(P, wsft, Xsft);
    evaluate(P, Xsft, &os);
    cons(P, os.g, wsft, cs);
    const double th_s = sum_abs(cs, m), ph_s = os.f + barrier(P, wsft, mu);
    const int orig_ok = acceptable(th_s, ph_s, th_ref, ph_ref, gd_ref, 0.0, sw_ref, S->theta_max, &S->F, 0, NULL);
    for (int r = 0; r < m; ++r) ys[r] = S->y[r] + a_soft * dy[r];
    for (int k = 0; k < nw; ++k) {
      zLs[k] = P->hasL[k] ? S->zL[k] + a_soft * dzL[k] : S->zL[k];
      zUs[k] = P->hasU[k] ? S->zU[k] + a_soft * dzU[k] : S->zU[k];
    }
    const int fin_s = isfinite(th_s) && isfinite(ph_s);
    const int better = pd_error(P, &os, wsft, ys, zLs, zUs, mu) <= SOFT_RESTO_FACTOR * pd_error(P, &S->cur, w, S->y, S->zL, S->zU, mu);
    soft_ok = fin_s && (orig_ok || better);
    if (soft_ok) {
      memcpy(st_w, wsft, sizeof(double) * (size_t)nw);
      st_alpha = a_soft; aug = 0; found = 1;
      const int left = orig_ok;
      S->in_soft = left ? 0 : 1;
      if (left || !soft_now) S->soft_cnt = 0;
    }
  }
  int failed = !tiny && !found;
  if (failed && E->err0 <= o->acceptable_tol) {  /* no restoration phase at an acceptable point */
    S->status = ST_ACCEPTABLE;
    S->active = 0;
    S->mu = mu;
    return;
  }
  if (failed && th_ref <= ALMOST_FEASIBLE * o->tol) {  /* (th_ref: the current iterate's theta, the kept one after a watchdog restore) */
    /* nor at an almost feasible point (BacktrackingLineSearch: theta <= 1e-2 tol): the backup acceptable
     * point is restored and the solve stops there as acceptable (RestoreAcceptablePoint), or without
     * one it ends as a restoration failure ("Restoration phase called, but point is almost feasible") */
    S->active = 0;
    S->mu = mu;
    S->status = S->has_acc ? ST_ACCEPTABLE : ST_RESTO_FAILED;
    g_resto_fail_events[0] += 1;
    if (S->has_acc) {
      g_resto_fail_events[1] += 1;
      memcpy(S->w, S->acc_w, sizeof(double) * (size_t)nw);
      memcpy(S->zL, S->acc_zL, sizeof(double) * (size_t)nw);
      memcpy(S->zU, S->acc_zU, sizeof(double) * (size_t)nw);
      memcpy(S->y, S->acc_y, sizeof(double) * (size_t)m);
    }
    return;
  }
  if (failed) { S->in_soft = 0; S->soft_cnt = 0; }
  if (g_trace)  /* (diagnostics: batch_ipm.py's verbose line, scripts/solve_divergence.py) */
    fprintf(stderr, "   [C] mu=%.2e err0=%.2e a_max=%.2e alpha=%.2e dw=%.2e dy=%.2e dW=%.1e f=%.6e d_inf=%.2e c_inf=%.2e resto_next=%d tiny=%d rank_def=%d\n",
            mu, E->err0, a_max, st_alpha, max_abs(dw, nw), max_abs(dy, m), delta_w, S->cur.f, E->d_inf, E->c_inf, failed, S->tiny_last, K.rank_def);
  const int moved = !failed;
  const double al = st_alpha;
  const double az = soft_ok ? a_soft : a_z_r;
  if (moved) {
    double Xn[NMAX];
    unpack(P, st_w, Xn);
    evaluate(P, Xn, &ev_new);
    if (aug) filter_add(&S->F, th_ref, ph_ref);
    double y_new[MMAX];
    for (int r = 0; r < m; ++r) y_new[r] = S->y[r] + al * dy[r];
    for (int k = 0; k < nw; ++k) {
      const double dln = P->hasL[k] ? st_w[k] - P->wl0[k] : 1.0;
      const double dun = P->hasU[k] ? P->wu0[k] - st_w[k] : 1.0;
      if (P->hasL[k]) {
        const double z = S->zL[k] + az * dzL[k];
        S->zL[k] = dmin(dmax(z, mu / (KAPPA_SIGMA * dln)), KAPPA_SIGMA * mu / dln);
      }
      if (P->hasU[k]) {
        const double z = S->zU[k] + az * dzU[k];
        S->zU[k] = dmin(dmax(z, mu / (KAPPA_SIGMA * dun)), KAPPA_SIGMA * mu / dun);
      }
    }
    double sk[NWMAX];
    for (int k = 0; k < nf; ++k) sk[k] = st_w[k] - w[k];
    lbfgs_update(P, S, sk, &ev_new, &S->cur, y_new, 1);
    memcpy(S->w, st_w, sizeof(double) * (size_t)nw);
    memcpy(S->y, y_new, sizeof(double) * (size_t)m);
    S->cur = ev_new;
  } else {
    filter_add(&S->F, th_ref, ph_ref);  /* PrepareRestoPhaseStart */
    S->in_wd = 0;  /* (the restoration phase ends the watchdog) */
    S->wd_cnt = 0;
    enter_resto(P, S, E->c, E->A, S->cur.f);
  }
  S->mu = mu;
  S->iters += 1;
  S->dwl = delta_w;
}

/* One restoration-phase iteration (batch_ipm.py resto_step) */
static void resto_step(Prob* P, State* S, const Opts* o) {
  const int nw = P->nw, m = P->m, nf = P->nf;
  static __thread double A[MMAX * NWMAX], W[NWMAX * NWMAX];
  static __thread Eval trial, ev_new;
  double c[MMAX], DR2[NWMAX];
  const double* w = S->w;
  jac_w(P, S->cur.J, A);
  cons(P, S->cur.g, w, c);
  for (int k = 0; k < nw; ++k) DR2[k] = k < nf ? 1.0 / pow(dmax(fabs(S->wR[k]), 1.0), 2) : 0.0;
  double muR = S->muR;
  double cR[MMAX], cl[NWMAX], cu[NWMAX], gfw[NWMAX];
  for (int r = 0; r < m; ++r) cR[r] = c[r] - S->p[r] + S->nn[r];
  double eta = sqrt(muR);
  double dinf = 0.0, zsum = 0.0;
  for (int k = 0; k < nw; ++k) {
    gfw[k] = k < nf ? eta * DR2[k] * (w[k] - S->wR[k]) : 0.0;
    double s = gfw[k];
    for (int r = 0; r < m; ++r) s += A[r * nw + k] * S->y[r];
    s = s - S->zLR[k] + S->zUR[k];
    dinf = dmax(dinf, fabs(s));
    cl[k] = P->hasL[k] ? (w[k] - P->wl0[k]) * S->zLR[k] : 0.0;
    cu[k] = P->hasU[k] ? (P->wu0[k] - w[k]) * S->zUR[k] : 0.0;
    zsum += fabs(S->zLR[k]) + fabs(S->zUR[k]);
  }
  double cmax = 0.0;
  for (int r = 0; r < m; ++r) {
    dinf = dmax(dinf, dmax(fabs(RHO_R - S->y[r] - S->zp[r]), fabs(RHO_R + S->y[r] - S->zn[r])));
    zsum += fabs(S->zp[r]) + fabs(S->zn[r]);
    cmax = dmax(cmax, dmax(S->p[r] * S->zp[r], S->nn[r] * S->zn[r]));
  }
  for (int k = 0; k < nw; ++k) cmax = dmax(cmax, dmax(cl[k], cu[k]));
  const int nbR = P->nbounds + 2 * m;
  const double sd = dmax((sum_abs(S->y, m) + zsum) / (double)(m + nbR > 1 ? m + nbR : 1), 100.0) / 100.0;
  const double sc = dmax(zsum / (double)(nbR > 1 ? nbR : 1), 100.0) / 100.0;
  const double base = dmax(dinf / sd, m ? max_abs(cR, m) : 0.0);
  const double errR0 = dmax(base, cmax / sc);
  if (errR0 <= (S->resto_tight ? 1e-2 * o->tol : o->tol)) {  /* RestoConvergenceCheck */
    const int feas = (m ? max_abs(c, m) : 0.0) <= 1e2 * o->tol;
    if (!feas || S->resto_tight) {
      S->status = feas ? ST_RESTO_FAILED : ST_INFEASIBLE;
      S->active = 0;
      if (feas) g_resto_fail_events[0] += 1;
      if (feas && S->has_acc) {  /* RestoreAcceptablePoint: stop there as acceptable */
        g_resto_fail_events[1] += 1;
        memcpy(S->w, S->acc_w, sizeof(double) * (size_t)nw);
        memcpy(S->zL, S->acc_zL, sizeof(double) * (size_t)nw);
        memcpy(S->zU, S->acc_zU, sizeof(double) * (size_t)nw);
        memcpy(S->y, S->acc_y, sizeof(double) * (size_t)m);
        S->status = ST_ACCEPTABLE;
      }
      return;
    }
    S->resto_tight = 1;
  }
  Filter* FR = &S->FR;
  for (int rr = 0; rr < MU_ROUNDS; ++rr) {
    double cm = 0.0;
    for (int k = 0; k < nw; ++k) {
      cm = dmax(cm, P->hasL[k] ? fabs(cl[k] - muR) : fabs(cl[k]));
      cm = dmax(cm, P->hasU[k] ? fabs(cu[k] - muR) : fabs(cu[k]));
    }
    for (int r = 0; r < m; ++r) cm = dmax(cm, dmax(fabs(S->p[r] * S->zp[r] - muR), fabs(S->nn[r] * S->zn[r] - muR)));
    if (dmax(base, cm / sc) <= BARRIER_TOL_FACTOR * muR && muR > o->mu_min) {
      muR = dmax(dmin(0.2 * muR, pow(muR, 1.5)), o->mu_min);
      filter_reset(FR);
    }
  }
  const double tauR = dmax(1.0 - muR, 0.99);
  eta = sqrt(muR);
  for (int k = 0; k < nw; ++k) gfw[k] = k < nf ? eta * DR2[k] * (w[k] - S->wR[k]) : 0.0;
  double dl[NWMAX], du[NWMAX], Sig[NWMAX], gphi[NWMAX], r1[NWMAX], r2[MMAX], rp[MMAX], rn[MMAX], Dinv[MMAX];
  for (int k = 0; k < nw; ++k) {
    dl[k] = P->hasL[k] ? w[k] - P->wl0[k] : 1.0;
    du[k] = P->hasU[k] ? P->wu0[k] - w[k] : 1.0;
    Sig[k] = (P->hasL[k] ? S->zLR[k] / dl[k] : 0.0) + (P->hasU[k] ? S->zUR[k] / du[k] : 0.0);
    gphi[k] = gfw[k] - (P->hasL[k] ? muR / dl[k] : 0.0) + (P->hasU[k] ? muR / du[k] : 0.0);
    double s = 0.0;
    for (int r = 0; r < m; ++r) s += A[r * nw + k] * S->y[r];
    r1[k] = -(gphi[k] + s);
  }
  for (int r = 0; r < m; ++r) {
    const double Sp = S->zp[r] / S->p[r], Sn = S->zn[r] / S->nn[r];
    rp[r] = -((RHO_R - muR / S->p[r]) - S->y[r]);
    rn[r] = -((RHO_R - muR / S->nn[r]) + S->y[r]);
    Dinv[r] = 1.0 / (1.0 / Sp + 1.0 / Sn);
    r2[r] = -cR[r] + rp[r] / Sp - rn[r] / Sn;
  }
  if (P->exact) {  /* the constraints' curvature y^T g (the proximity term's is added below) */
    double Xc[NMAX];
    unpack(P, w, Xc);
    double yr[MMAX];
    y_raw(P, S->y, yr);
    lagr_hessian(P, Xc, yr, 1, S->Hq);
    if (P->scaled)
      for (int q = 0; q < P->nf * P->nf; ++q) S->Hq[q] = S->Hq[q] * P->df;
  }
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < nw; ++j)
      W[i * nw + j] = (i == j ? Sig[i] + (i < nf ? eta * DR2[i] : 0.0) : 0.0) + ((i < nf && j < nf) ? S->Hq[i * nf + j] : 0.0);
  double dw[NWMAX], dy[MMAX], dp[MMAX], dn[MMAX];
  S->dwlR = kkt_qd(W, A, Dinv, r1, r2, nw, m, S->dwlR, dw, dy);
  double dzL[NWMAX], dzU[NWMAX], dzp[MMAX], dzn[MMAX];
  for (int r = 0; r < m; ++r) {
    const double Sp = S->zp[r] / S->p[r], Sn = S->zn[r] / S->nn[r];
    dp[r] = (rp[r] + dy[r]) / Sp;
    dn[r] = (rn[r] - dy[r]) / Sn;
    dzp[r] = muR / S->p[r] - S->zp[r] - S->zp[r] / S->p[r] * dp[r];
    dzn[r] = muR / S->nn[r] - S->zn[r] - S->zn[r] / S->nn[r] * dn[r];
  }
  for (int k = 0; k < nw; ++k) {
    dzL[k] = P->hasL[k] ? muR / dl[k] - S->zLR[k] - S->zLR[k] / dl[k] * dw[k] : 0.0;
    dzU[k] = P->hasU[k] ? muR / du[k] - S->zUR[k] + S->zUR[k] / du[k] * dw[k] : 0.0;
  }
  double mdw[NWMAX], mw[NWMAX], mwu[NWMAX];
  for (int k = 0; k < nw; ++k) { mdw[k] = -dw[k]; mw[k] = -w[k]; mwu[k] = -P->wu0[k]; }
  const double a_max = dmin(dmin(max_step(w, dw, P->hasL, P->wl0, nw, tauR), max_step(mw, mdw, P->hasU, mwu, nw, tauR)),
                            dmin(max_step_all(S->p, dp, m, tauR), max_step_all(S->nn, dn, m, tauR)));
  const double a_z = dmin(dmin(max_step(S->zLR, dzL, P->hasL, NULL, nw, tauR), max_step(S->zUR, dzU, P->hasU, NULL, nw, tauR)),
                          dmin(max_step_all(S->zp, dzp, m, tauR), max_step_all(S->zn, dzn, m, tauR)));
  double gd = 0.0;
  for (int k = 0; k < nw; ++k) gd += gphi[k] * dw[k];
  for (int r = 0; r < m; ++r) gd += (RHO_R - muR / S->p[r]) * dp[r] + (RHO_R - muR / S->nn[r]) * dn[r];
  const double thetaR = sum_abs(cR, m);
  double prox = 0.0, lpn = 0.0;
  for (int k = 0; k < nf; ++k) prox += DR2[k] * (w[k] - S->wR[k]) * (w[k] - S->wR[k]);
  for (int r = 0; r < m; ++r) lpn += log(S->p[r]) + log(S->nn[r]);
  const double phR_k = RHO_R * (sum_abs(S->p, m) + sum_abs(S->nn, m)) + 0.5 * eta * prox + barrier(P, w, muR) - muR * lpn;
  const int switch_ok = thetaR <= S->thminR;
  const double a_min = alpha_min_of(thetaR, gd, S->thminR);
  int searching = 1, found = 0, aug = 0;
  double st_w[NWMAX], st_p[MMAX], st_n[MMAX], al = 0.0;
  double alpha = a_max;
  for (int ls = 0; ls < (o->max_ls > 1 ? o->max_ls : 1) && searching; ++ls) {
    double wt[NWMAX], Xt[NMAX], pt[MMAX], nt[MMAX], ct[MMAX];
    for (int k = 0; k < nw; ++k) wt[k] = w[k] + alpha * dw[k];
    for (int r = 0; r < m; ++r) { pt[r] = S->p[r] + alpha * dp[r]; nt[r] = S->nn[r] + alpha * dn[r]; }
    unpack(P, wt, Xt);
    evaluate_fg(P, Xt, &trial.f, trial.g);
    cons(P, trial.g, wt, ct);
    double th = 0.0, pr = 0.0, lp = 0.0;
    for (int r = 0; r < m; ++r) { th += fabs(ct[r] - pt[r] + nt[r]); lp += log(pt[r]) + log(nt[r]); }
    for (int k = 0; k < nf; ++k) pr += DR2[k] * (wt[k] - S->wR[k]) * (wt[k] - S->wR[k]);
    const double ph = RHO_R * (sum_abs(pt, m) + sum_abs(nt, m)) + 0.5 * eta * pr + barrier(P, wt, muR) - muR * lp;
    int h = 0;
    if (acceptable(th, ph, thetaR, phR_k, gd, alpha, switch_ok, S->thmaxR, FR, 0, &h)) {
      memcpy(st_w, wt, sizeof(double) * (size_t)nw);
      memcpy(st_p, pt, sizeof(double) * (size_t)m);
      memcpy(st_n, nt, sizeof(double) * (size_t)m);
      al = alpha; aug = h; found = 1; searching = 0;
    }
    alpha = searching ? 0.5 * alpha : alpha;
    searching = searching && alpha > a_min;
  }
  S->muR = muR;
  S->iters += 1;
  if (!found) {  /* RestoRestorationPhase: p, n reset at the current point */
    for (int r = 0; r < m; ++r) {
      const double a = (muR - RHO_R * c[r]) / (2.0 * RHO_R);
      S->nn[r] = a + sqrt(a * a + muR * c[r] / (2.0 * RHO_R));
      S->p[r] = c[r] + S->nn[r];
    }
    return;
  }
  double Xn[NMAX];
  unpack(P, st_w, Xn);
  evaluate(P, Xn, &ev_new);
  if (aug) filter_add(FR, thetaR, phR_k);
  double y_new[MMAX];
  for (int r = 0; r < m; ++r) y_new[r] = S->y[r] + al * dy[r];
  for (int k = 0; k < nw; ++k) {
    const double dln = P->hasL[k] ? st_w[k] - P->wl0[k] : 1.0;
    const double dun = P->hasU[k] ? P->wu0[k] - st_w[k] : 1.0;
    if (P->hasL[k]) S->zLR[k] = dmin(dmax(S->zLR[k] + a_z * dzL[k], muR / (KAPPA_SIGMA * dln)), KAPPA_SIGMA * muR / dln);
    if (P->hasU[k]) S->zUR[k] = dmin(dmax(S->zUR[k] + a_z * dzU[k], muR / (KAPPA_SIGMA * dun)), KAPPA_SIGMA * muR / dun);
  }
  for (int r = 0; r < m; ++r) {
    S->zp[r] = dmin(dmax(S->zp[r] + a_z * dzp[r], muR / (KAPPA_SIGMA * st_p[r])), KAPPA_SIGMA * muR / st_p[r]);
    S->zn[r] = dmin(dmax(S->zn[r] + a_z * dzn[r], muR / (KAPPA_SIGMA * st_n[r])), KAPPA_SIGMA * muR / st_n[r]);
  }
  double sk[NWMAX];
  for (int k = 0; k < nf; ++k) sk[k] = st_w[k] - w[k];
  lbfgs_update(P, S, sk, &ev_new, &S->cur, y_new, 0);
  memcpy(S->p, st_p, sizeof(double) * (size_t)m);
  memcpy(S->nn, st_n, sizeof(double) * (size_t)m);
  memcpy(S->w, st_w, sizeof(double) * (size_t)nw);
  memcpy(S->y, y_new, sizeof(double) * (size_t)m);
  S->cur = ev_new;
  /* back to the regular iteration? (TestOrigProgress) */
  double c_o[MMAX];
  cons(P, ev_new.g, st_w, c_o);
  const double th_o = sum_abs(c_o, m);
  const double ph_o = ev_new.f + barrier(P, st_w, S->mu);
  int in_filter = 1;
  for (int k = 0; k < FMAX; ++k)
    if (!((th_o <= S->F.t[k]) || (ph_o <= S->F.p[k]))) in_filter = 0;
  const double t0 = S->th_o0, p0 = S->ph_o0;
  const int vs_start = (th_o - (1.0 - GAMMA_TH) * t0 <= 10.0 * EPS * fabs(t0)) ||
                       ((ph_o - p0) - (-GAMMA_PHI * t0) <= 10.0 * EPS * fabs(p0));
  if (isfinite(th_o) && isfinite(ph_o) && th_o <= KAPPA_RESTO * t0 && in_filter && vs_start) leave_resto(P, S, st_w);
}

/* The best-feasible-iterate fallback (not IPOPT; cpl_solve_options.fallback_viol_tol): off (0) by
 * default like the engine's; cplo_set_fallback_viol_tol opts in (process-wide). */
static double g_fallback_viol_tol = 0.0;
void cplo_set_fallback_viol_tol(double v) { g_fallback_viol_tol = v; }
/* IPOPT's acceptable_tol (default 1e-6, process-wide) and the count of failed restoration phases on this
 * thread (feasible end points; those with a backup acceptable point second): the search for the
 * RestoreAcceptablePoint branch (scripts/resto_acc_search.py). */
static double g_acceptable_tol = 1e-6;
void cplo_set_acceptable_tol(double v) { g_acceptable_tol = v; }
void cplo_resto_fail_events(long* out) {
  out[0] = g_resto_fail_events[0]; out[1] = g_resto_fail_events[1];
  g_resto_fail_events[0] = g_resto_fail_events[1] = 0;
}
/* nlp_scaling_method: 1 gradient-based (IPOPT's default, the reference's), 0 none (process-wide) */
static int g_nlp_scaling = 1;
void cplo_set_nlp_scaling(int on) { g_nlp_scaling = on != 0; }

/* Solve one instance from x0 (IFOPT's IpoptSolver defaults: limited-memory Hessian; exact_hessian:
 * the analytic Lagrangian Hessian, batch_ipm.py's hessian="exact", Ground / no environment).  Returns 0;
 * x_out [n] (projected onto the original bounds), status (0 optimal, 1 acceptable, 2 max_iter,
 * 3 local infeasibility, 4 restoration failure), iterations, objective at x_out, restorations. */
int cplo_solve(const cpl_problem_desc* d, const double* x0, double mass, int max_iter, double tol, int exact_hessian,
               double* x_out,
               int32_t* status, int32_t* iterations, double* objective, int32_t* restorations, int64_t* evaluations) {
  /* per thread (cplo_time_solve_mt solves instances on OpenMP threads): large, so not on the stack */
  static __thread Prob P;
  static __thread State S;
  static __thread Errors E;
  int32_t n, m, nnz;
  if (cplo_dims(d, &n, &m, &nnz) || n > NMAX || m > MMAX || nnz > 4096) return CPL_ERR_UNSUPPORTED;
  if (g_trace < 0) g_trace = getenv("CPLO_TRACE") ? atoi(getenv("CPLO_TRACE")) : 0;
  memset(&P, 0, sizeof(P));
  if (exact_hessian && d->env_kind != CPL_ENV_NONE && d->env_kind != CPL_ENV_GROUND) return CPL_ERR_UNSUPPORTED;
  P.d = d; P.n = n; P.m = m; P.nnz = nnz; P.mass = mass; P.exact = exact_hessian != 0;
  cplo_structure(d, P.iRow, P.jCol);
  cplo_bounds(d, P.xl, P.xu, P.gl, P.gu);
  P.nf = 0;
  for (int j = 0; j < n; ++j) {
    P.is_fixed[j] = fabs(P.xu[j] - P.xl[j]) <= 1e-14 * dmax(1.0, fabs(P.xl[j]));
    if (!P.is_fixed[j]) P.free_idx[P.nf++] = j;
  }
  P.nI = 0;
  for (int r = 0; r < m; ++r) {
    P.row_slack[r] = -1;
    if (P.gl[r] != P.gu[r]) { P.row_slack[r] = P.nI; P.ineq[P.nI++] = r; }
  }
  P.nw = P.nf + P.nI;
  if (P.nw > NWMAX) return CPL_ERR_UNSUPPORTED;
  P.nbounds = 0;
  for (int k = 0; k < P.nw; ++k) {
    double lo = k < P.nf ? P.xl[P.free_idx[k]] : P.gl[P.ineq[k - P.nf]];
    double up = k < P.nf ? P.xu[P.free_idx[k]] : P.gu[P.ineq[k - P.nf]];
    if (k >= P.nf) {
      if (!(lo > -BIG)) lo = -INFINITY;
      if (!(up < BIG)) up = INFINITY;
    }
    lo = lo - 1e-8 * dmax(fabs(lo), 1.0);
    up = up + 1e-8 * dmax(fabs(up), 1.0);
    P.hasL[k] = isfinite(lo);
    P.hasU[k] = isfinite(up);
    P.wl0[k] = P.hasL[k] ? lo : 0.0;
    P.wu0[k] = P.hasU[k] ? up : 0.0;
    P.nbounds += P.hasL[k] + P.hasU[k];
  }
  P.ws = cplo_ws_new(d);
  if (!P.ws) return CPL_ERR_RUNTIME;
  for (int j = 0; j < n; ++j) P.Xbase[j] = P.is_fixed[j] ? P.xl[j] : x0[j];
  P.scaled = 0;
  if (g_nlp_scaling) nlp_scaling(&P, P.Xbase);
  Opts o = {tol, g_acceptable_tol, dmin(tol, COMPL_INF_TOL) / (BARRIER_TOL_FACTOR + 1.0), g_fallback_viol_tol, 15, 40, 4};
  /* starting point: x pushed into its bounds, slacks = g_I(x) pushed into theirs */
  const int nw = P.nw, nf = P.nf;
  double w0[NWMAX], Xs[NMAX];
  memset(&S, 0, sizeof(S));
  for (int k = 0; k < nw; ++k) w0[k] = k < nf ? P.Xbase[P.free_idx[k]] : 0.0;
  push(&P, w0);
  unpack(&P, w0, Xs);
  evaluate(&P, Xs, &S.cur);
  for (int k = 0; k < nw; ++k) w0[k] = k < nf ? Xs[P.free_idx[k]] : S.cur.g[P.ineq[k - nf]];
  push(&P, w0);
  memcpy(S.w, w0, sizeof(double) * (size_t)nw);
  for (int k = 0; k < nw; ++k) { S.zL[k] = P.hasL[k] ? 1.0 : 0.0; S.zU[k] = P.hasU[k] ? 1.0 : 0.0; }
  double c0[MMAX];
  cons(&P, S.cur.g, S.w, c0);
  const double theta0 = sum_abs(c0, m);
  S.theta_max = 1e4 * dmax(theta0, 1.0);
  S.theta_min = 1e-4 * dmax(theta0, 1.0);
  {  /* least-squares constraint multipliers (constr_mult_init_max = 1e3) */
    static __thread double A0[MMAX * NWMAX], AAt[MMAX * MMAX];
    double rhs[MMAX];
    jac_w(&P, S.cur.J, A0);
    for (int a = 0; a < m; ++a) {
      for (int b = 0; b < m; ++b) {
        double s = 0.0;
        for (int k = 0; k < nw; ++k) s += A0[a * nw + k] * A0[b * nw + k];
        AAt[a * m + b] = s + (a == b ? 1e-12 : 0.0);
      }
      double s = 0.0;
      for (int k = 0; k < nw; ++k) s += A0[a * nw + k] * ((k < nf ? S.cur.grad[P.free_idx[k]] : 0.0) - S.zL[k] + S.zU[k]);
      rhs[a] = s;
    }
    const int bad = cholesky(AAt, m, 0.0);
    if (!bad) chol_solve(AAt, m, rhs);
    const double ymx = bad ? INFINITY : max_abs(rhs, m);
    for (int r = 0; r < m; ++r) S.y[r] = (!bad && ymx <= 1e3) ? -rhs[r] : 0.0;
  }
  S.mu = 0.1;
  S.active = 1;
  S.status = ST_MAX_ITER;
  filter_reset(&S.F);
  lbfgs_reset(&P, &S);
  S.best_f = INFINITY;
  int it = 0;
  while (it < max_iter && S.active) {
    errors(&P, &S.cur, S.w, S.y, S.zL, S.zU, &E);
    if (!S.resto) check(&S, &E, &o);
    if (S.active) {
      if (S.resto) resto_step(&P, &S, &o);
      else regular_step(&P, &S, &E, &o);
    }
    if (o.fallback_viol_tol > 0.0 && S.active && orig_violation(&P, S.cur.g) <= o.fallback_viol_tol && S.cur.f < S.best_f) {
      memcpy(S.best_w, S.w, sizeof(double) * (size_t)nw);
      S.best_f = S.cur.f;
    }
    ++it;
  }
  if (S.active && !S.resto) {  /* the final convergence test at the last iterate */
    errors(&P, &S.cur, S.w, S.y, S.zL, S.zU, &E);
    check(&S, &E, &o);
  }
  if (o.fallback_viol_tol > 0.0 && S.status > ST_ACCEPTABLE && orig_violation(&P, S.cur.g) > o.fallback_viol_tol &&
      isfinite(S.best_f))
    memcpy(S.w, S.best_w, sizeof(double) * (size_t)nw);
  double X[NMAX], gfin[MMAX], f = 0.0;
  unpack(&P, S.w, X);
  for (int j = 0; j < n; ++j) X[j] = dmin(dmax(X[j], P.xl[j]), P.xu[j]);  /* honor_original_bounds */
  P.scaled = 0;  /* the objective / constraints reported at x_out: the unscaled callbacks */
  evaluate_fg(&P, X, &f, gfin);
  if (x_out) memcpy(x_out, X, sizeof(double) * (size_t)n);
  if (status) *status = S.status;
  if (iterations) *iterations = S.iters;
  if (objective) *objective = f;
  if (restorations) *restorations = S.n_resto;
  if (evaluations) *evaluations = P.evals;
  cplo_ws_free(P.ws);
  return CPL_OK;
}

/* Wall-clock seconds of cplo_solve over `count` instances (x0 [count][n], masses) on this thread */
double cplo_time_solve(const cpl_problem_desc* d, int64_t count, const double* x0, const double* mass, int max_iter,
                       double tol, int exact_hessian, int32_t* status, int32_t* iterations) {
  int32_t n, m, nnz;
  if (cplo_dims(d, &n, &m, &nnz)) return -1.0;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  double xo[NMAX];
  for (int64_t b = 0; b < count; ++b)
    if (cplo_solve(d, x0 + b * n, mass ? mass[b] : d->mass, max_iter, tol, exact_hessian, xo, status ? status + b : NULL,
                   iterations ? iterations + b : NULL, NULL, NULL, NULL))
      return -1.0;
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* The same over `threads` OpenMP threads (<= 0: omp_get_max_threads()), instances split statically:
 * the all-core CPU baseline of the solve legs; wall-clock seconds, -1 on failure */
double cplo_time_solve_mt(const cpl_problem_desc* d, int64_t count, const double* x0, const double* mass, int max_iter,
                          double tol, int exact_hessian, int threads, int32_t* status, int32_t* iterations) {
  int32_t n, m, nnz;
  if (cplo_dims(d, &n, &m, &nnz)) return -1.0;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#else
  threads = 1;
#endif
  struct timespec t0, t1;
  int failed = 0;
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads) reduction(| : failed)
  for (int64_t b = 0; b < count; ++b) {
    double xo[NMAX];
    if (cplo_solve(d, x0 + b * n, mass ? mass[b] : d->mass, max_iter, tol, exact_hessian, xo, status ? status + b : NULL,
                   iterations ? iterations + b : NULL, NULL, NULL, NULL))
      failed |= 1;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (failed) return -1.0;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
