// cpl_solver.hip — the native batched solve engine (C-ABI cpl_solver_*, include/cpl_mi355x.h).
//
// Many concurrent CentroidalPlanner solves in lock-step on one GPU: IPOPT's primal-dual
// interior-point method (Waechter & Biegler 2006) as restated in centroidalplanner_amd/batch_ipm.py
// — whose host path (CPU tensors, the oracle's callbacks) is the checker of this engine — with every
// per-instance quantity a row of a device buffer:
//   * callbacks: cpl_eval_batch(_ex) (values-only Jacobian records), the analytic Lagrangian Hessian
//     (cpl_lagrangian_hessian) or central differences (cpl_ipm_fd_points + cpl_eval_lagrangian_grad
//     + cpl_ipm_fd_hessian_raw), or IPOPT's limited-memory BFGS model (6 pairs, scalar1; IFOPT's
//     IpoptSolver default, the reference's configuration, src/CentroidalPlanner.cpp:22-29);
//   * per-instance iteration work: cpl_ipm_optimality / newton_setup / post_step / trial_point /
//     judge_take / accept / max_step / dense_a / masked_rows, the Newton step cpl_kkt_solve;
//   * the glue between them (the line-search state, second-order corrections, the feasibility step
//     standing in for the restoration phase, L-BFGS) in the small kernels below — no framework ops.
// One iteration (fixed trip counts, masked updates, no host synchronisation) is captured once as a
// HIP graph and replayed; the host reads an "any instance active" byte one iteration behind.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <algorithm>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "cpl_layout.hpp"
#include "cpl_status.hpp"

namespace cpl {
// cpl_ipm.hip: cpl_ipm_newton_setup over the engine's compact limited-memory model
int32_t ipm_newton_setup_lm(int64_t batch, int32_t nw, int32_t m, int32_t nf, const double* d_w, const double* d_zL,
                            const double* d_zU, const double* d_gw, const double* d_A, const double* d_y,
                            const double* d_c, const double* d_f, const double* d_mu, const uint8_t* d_hasL,
                            const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0, const double* d_Hc,
                            int32_t lm_pairs, double* d_M, double* d_r1, double* d_r2, double* d_gphi,
                            double* d_mr_diag, double* d_theta, double* d_phi, const uint8_t* d_active, void* stream);
namespace {

constexpr int FMAX = 64;          // filter entries kept per instance (a ring), as batch_ipm.FMAX
constexpr double BIG = 1.0e19;    // |bound| >= 1e19 is infinite (IPOPT nlp_lower/upper_bound_inf)
constexpr int WPB = 4;            // instances per 256-thread workgroup (one wave each)

#define CK(expr)                      \
  do {                                \
    const int32_t st_ = (expr);       \
    if (st_ != CPL_OK) return st_;    \
  } while (0)

inline unsigned blocks_for(int64_t batch) { return (unsigned)((batch + WPB - 1) / WPB); }
inline unsigned blocks_elems(int64_t total) { return (unsigned)((total + 255) / 256); }

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

// IPOPT bound_push = bound_frac = 1e-2 (absolute and relative to the range), batch_ipm.push
__device__ __forceinline__ double push_into(double v, bool hl, bool hu, double lo, double up) {
  const double k = 1e-2;
  const double rng = (hl && hu) ? up - lo : INFINITY;
  const double pl = fmin(k * fmax(fabs(lo), 1.0), k * rng);
  const double pu = fmin(k * fmax(fabs(up), 1.0), k * rng);
  if (hl) v = fmax(v, lo + pl);
  if (hu) v = fmin(v, up - pu);
  return v;
}

// constraint residual of row r: g - g_l (equality), g - s (inequality, slack s)
__device__ __forceinline__ double cons_row(const double* g, const double* w, int nf, int r, const int32_t* row_slack,
                                           const double* gl) {
  const int s = row_slack[r];
  return s >= 0 ? g[r] - w[nf + s] : g[r] - gl[r];
}

// Xbase = x0 with the fixed variables at their (equal) bounds
__global__ void k_xbase(int64_t total, int n, const double* __restrict__ x0, const uint8_t* __restrict__ is_fixed,
                        const double* __restrict__ xl, double* __restrict__ Xbase) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int j = (int)(e % n);
  Xbase[e] = is_fixed[j] ? xl[j] : x0[e];
}

// the starting point's x: the free variables pushed into their bounds (batch_ipm: Xs)
__global__ void k_start_x(int64_t total, int n, const int32_t* __restrict__ freepos, const double* __restrict__ Xbase,
                          const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU,
                          const double* __restrict__ wl0, const double* __restrict__ wu0, double* __restrict__ X) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int j = (int)(e % n);
  const int k = freepos[j];
  X[e] = k >= 0 ? push_into(Xbase[e], hasL[k], hasU[k], wl0[k], wu0[k]) : Xbase[e];
}

// the starting state of every instance (one wave each): w0 = push([x_free, g_I]), bound multipliers
// 1, theta_0 and the filter's theta_max / theta_min, mu, flags; gw0 and the least-squares system's
// right-hand side r1 = -(gw0 - zL0 + zU0) (the multiplier estimate is one KKT solve with M = I)
__global__ __launch_bounds__(256) void k_init_state(
    int64_t B, int n, int m, int nf, int nw, const int32_t* __restrict__ free_idx, const int32_t* __restrict__ ineq_row,
    const int32_t* __restrict__ row_slack, const double* __restrict__ gl, const uint8_t* __restrict__ hasL,
    const uint8_t* __restrict__ hasU, const double* __restrict__ wl0, const double* __restrict__ wu0, double mu_init,
    const double* __restrict__ X, const double* __restrict__ g, const double* __restrict__ grad,
    double* __restrict__ w, double* __restrict__ zL, double* __restrict__ zU, double* __restrict__ theta_max,
    double* __restrict__ theta_min, double* __restrict__ mu, uint8_t* __restrict__ active,
    int64_t* __restrict__ status, int64_t* __restrict__ iters, int64_t* __restrict__ acc, double* __restrict__ filt_t,
    double* __restrict__ filt_p, int64_t* __restrict__ fcount, double* __restrict__ dwl, double* __restrict__ d_inf,
    uint8_t* __restrict__ lm_cnt, uint8_t* __restrict__ lm_skip, double* __restrict__ r1, double* __restrict__ r2, double* __restrict__ M) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  double* wb = w + b * nw;
  for (int k = lane; k < nw; k += 64) {
    const double v = k < nf ? X[b * n + free_idx[k]] : g[b * m + ineq_row[k - nf]];
    const bool hl = hasL[k], hu = hasU[k];
    wb[k] = push_into(v, hl, hu, wl0[k], wu0[k]);
    const double zl = hl ? 1.0 : 0.0, zu = hu ? 1.0 : 0.0;
    zL[b * nw + k] = zl;
    zU[b * nw + k] = zu;
    const double gw = k < nf ? grad[b * n + free_idx[k]] : 0.0;
    r1[b * nw + k] = -((gw - zl) + zu);
    for (int j = 0; j < nw; ++j) M[(b * nw + k) * nw + j] = j == k ? 1.0 : 0.0;
  }
  double th = 0.0;
  for (int r = lane; r < m; r += 64) {  // (the slack recomputed: this lane did not write it)
    const int sl = row_slack[r];
    const double gv = g[b * m + r];
    const double c = sl >= 0 ? gv - push_into(gv, hasL[nf + sl], hasU[nf + sl], wl0[nf + sl], wu0[nf + sl]) : gv - gl[r];
    th += fabs(c);
    r2[b * m + r] = 0.0;
  }
  th = wave_sum(th);
  for (int k = lane; k < FMAX; k += 64) {
    filt_t[b * FMAX + k] = INFINITY;
    filt_p[b * FMAX + k] = INFINITY;
  }
  if (lane == 0) {
    theta_max[b] = 1e4 * fmax(th, 1.0);
    theta_min[b] = 1e-4 * fmax(th, 1.0);
    mu[b] = mu_init;
    active[b] = 1;
    status[b] = CPL_SOLVE_MAX_ITER;
    iters[b] = 0;
    acc[b] = 0;
    fcount[b] = 0;
    dwl[b] = 0.0;
    d_inf[b] = 0.0;
    lm_cnt[b] = 0;
    lm_skip[b] = 0;
  }
}

// least-squares multipliers: kept when |y|max <= 1e3 (IPOPT constr_mult_init_max) and the solve succeeded
__global__ __launch_bounds__(256) void k_y0(int64_t B, int m, const double* __restrict__ dy, const int32_t* __restrict__ info,
                                            double* __restrict__ y) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  double mx = 0.0;
  for (int r = lane; r < m; r += 64) mx = fmax(mx, fabs(dy[b * m + r]));
  mx = wave_max(mx);
  const bool keep = mx <= 1e3 && info[b] == 0;
  for (int r = lane; r < m; r += 64) y[b * m + r] = keep ? dy[b * m + r] : 0.0;
}

// gradient over w (gw = [grad f over the free variables, 0]) and the constraint residual c
__global__ __launch_bounds__(256) void k_prep(int64_t B, int n, int m, int nf, int nw, const int32_t* __restrict__ free_idx,
                                              const int32_t* __restrict__ row_slack, const double* __restrict__ gl,
                                              const double* __restrict__ grad, const double* __restrict__ g,
                                              const double* __restrict__ w, double* __restrict__ gradw,
                                              double* __restrict__ c) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) gradw[b * nw + k] = k < nf ? grad[b * n + free_idx[k]] : 0.0;
  if (c)
    for (int r = lane; r < m; r += 64) c[b * m + r] = cons_row(g + b * m, w + b * nw, nf, r, row_slack, gl);
}

// after the optimality kernel: tau = max(0.99, 1 - mu), the iteration's active snapshot, and the
// evaluation point X = unpack(w) for the Hessian
__global__ void k_unpack_tau(int64_t total, int n, int nw, const int32_t* __restrict__ freepos,
                             const double* __restrict__ Xbase, const double* __restrict__ w,
                             const double* __restrict__ mu, const uint8_t* __restrict__ active,
                             double* __restrict__ X, double* __restrict__ tau, uint8_t* __restrict__ act) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int64_t b = e / n;
  const int j = (int)(e - b * n);
  const int k = freepos[j];
  X[e] = k >= 0 ? w[b * nw + k] : Xbase[e];
  if (j == 0) {
    tau[b] = fmax(1.0 - mu[b], 0.99);
    act[b] = active[b];
  }
}

// X = unpack(w) (optionally clamped into [xl, xu]: IPOPT honor_original_bounds)
__global__ void k_unpack(int64_t total, int n, int nw, const int32_t* __restrict__ freepos,
                         const double* __restrict__ Xbase, const double* __restrict__ w, const double* __restrict__ xl,
                         const double* __restrict__ xu, double* __restrict__ X) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int64_t b = e / n;
  const int j = (int)(e - b * n);
  const int k = freepos[j];
  double v = k >= 0 ? w[b * nw + k] : Xbase[e];
  if (xl) v = fmin(fmax(v, xl[j]), xu[j]);
  X[e] = v;
}

// line-search state at the current iterate, the first trial step = the fraction-to-the-boundary one
__global__ __launch_bounds__(256) void k_ls_init(int64_t B, int m, int nw, const uint8_t* __restrict__ act,
                                                 const double* __restrict__ f, const double* __restrict__ g,
                                                 const double* __restrict__ w, const double* __restrict__ a_max,
                                                 uint8_t* __restrict__ searching, double* __restrict__ st_f,
                                                 double* __restrict__ st_g, double* __restrict__ st_w,
                                                 double* __restrict__ st_alpha, uint8_t* __restrict__ st_aug,
                                                 double* __restrict__ alpha, uint8_t* __restrict__ failed,
                                                 uint8_t* __restrict__ rest, uint8_t* __restrict__ any) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  for (int r = lane; r < m; r += 64) st_g[b * m + r] = g[b * m + r];
  for (int k = lane; k < nw; k += 64) st_w[b * nw + k] = w[b * nw + k];
  if (lane == 0) {
    if (b == 0 && any) any[0] = 0;  // the any-searching flag of the split iteration
    failed[b] = 0;  // (set again by k_feas_prep / k_rest when the rest of the line search runs)
    rest[b] = 0;
    searching[b] = act[b];
    st_f[b] = f[b];
    st_alpha[b] = 0.0;
    st_aug[b] = 0;
    alpha[b] = a_max[b];
  }
}


// c_soc = a_soc c_soc + c(trial point); the correction's right-hand side r2 = -c_soc
__global__ __launch_bounds__(256) void k_soc_rhs(int64_t B, int m, int nf, int nw, const int32_t* __restrict__ row_slack,
                                                 const double* __restrict__ gl, const double* __restrict__ g_t,
                                                 const double* __restrict__ w_t, const double* __restrict__ a_soc,
                                                 double* __restrict__ c_soc, double* __restrict__ r2) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const double a = a_soc[b];
  for (int r = lane; r < m; r += 64) {
    const double ct = cons_row(g_t + b * m, w_t + b * nw, nf, r, row_slack, gl);
    const double v = a * c_soc[b * m + r] + ct;
    c_soc[b * m + r] = v;
    r2[b * m + r] = -v;
  }
}

// second-order correction bookkeeping (batch_ipm step(): soc, c_soc, a_soc, th_old) and the first
// correction's right-hand side in one launch: c_soc = a_soc c + c(trial point), r2 = -c_soc
__global__ __launch_bounds__(256) void k_soc_begin_rhs(int64_t B, int m, int nf, int nw, const uint8_t* __restrict__ searching,
                                                       const double* __restrict__ th, const double* __restrict__ theta_k,
                                                       const double* __restrict__ c, const double* __restrict__ alpha,
                                                       const int32_t* __restrict__ row_slack, const double* __restrict__ gl,
                                                       const double* __restrict__ g_t, const double* __restrict__ w_t,
                                                       uint8_t* __restrict__ soc, double* __restrict__ c_soc,
                                                       double* __restrict__ a_soc, double* __restrict__ th_old,
                                                       double* __restrict__ r2) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const double a = alpha[b];
  for (int r = lane; r < m; r += 64) {
    const double ct = cons_row(g_t + b * m, w_t + b * nw, nf, r, row_slack, gl);
    const double v = a * c[b * m + r] + ct;
    c_soc[b * m + r] = v;
    r2[b * m + r] = -v;
  }
  if (lane == 0) {
    soc[b] = searching[b] && th[b] >= theta_k[b];
    a_soc[b] = a;
    th_old[b] = theta_k[b];
  }
}

// the last k_soc_after and the trial's halving in one launch; with `any`, instances still searching
// also raise the any-searching flag (zeroed by k_ls_init)
__global__ void k_soc_after_halve(int64_t B, uint8_t* __restrict__ soc, const uint8_t* __restrict__ ok,
                                  const double* __restrict__ th, double* __restrict__ th_old,
                                  const uint8_t* __restrict__ searching, double* __restrict__ alpha,
                                  uint8_t* __restrict__ any) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  soc[b] = soc[b] && !ok[b] && th[b] <= 0.99 * th_old[b];  // kappa_soc = 0.99
  th_old[b] = th[b];
  if (searching[b]) {
    alpha[b] = 0.5 * alpha[b];
    if (any) any[0] = 1;
  }
}

__global__ void k_soc_after(int64_t B, uint8_t* __restrict__ soc, const uint8_t* __restrict__ ok,
                            const double* __restrict__ th, double* __restrict__ th_old) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  soc[b] = soc[b] && !ok[b] && th[b] <= 0.99 * th_old[b];  // kappa_soc = 0.99
  th_old[b] = th[b];
}

// any instance still searching after the first trial (small-batch split iterations): one workgroup
__global__ __launch_bounds__(256) void k_any_searching(int64_t B, const uint8_t* __restrict__ searching,
                                                       uint8_t* __restrict__ flag) {
  __shared__ int s_any;
  if (threadIdx.x == 0) s_any = 0;
  __syncthreads();
  int a = 0;
  for (int64_t b = threadIdx.x; b < B; b += blockDim.x) a |= searching[b];
  if (a) s_any = 1;
  __syncthreads();
  if (threadIdx.x == 0) flag[0] = (uint8_t)s_any;
}

__global__ void k_halve(int64_t B, const uint8_t* __restrict__ searching, double* __restrict__ alpha) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (searching[b]) alpha[b] = 0.5 * alpha[b];
}

// the feasibility step's system: failed = still searching; Mr = diag(mr_diag) (its zero off-diagonal
// part set once); r2 = -c
__global__ __launch_bounds__(256) void k_feas_prep(int64_t B, int m, int nw, const uint8_t* __restrict__ searching,
                                                   const double* __restrict__ mr_diag, const double* __restrict__ c,
                                                   uint8_t* __restrict__ failed, double* __restrict__ Mr,
                                                   double* __restrict__ negc) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) Mr[(b * nw + k) * nw + k] = mr_diag[b * nw + k];
  for (int r = lane; r < m; r += 64) negc[b * m + r] = -c[b * m + r];
  if (lane == 0) failed[b] = searching[b];
}

__global__ void k_rest(int64_t B, const uint8_t* __restrict__ failed, const uint8_t* __restrict__ ok_r,
                       const double* __restrict__ alpha, uint8_t* __restrict__ rest, double* __restrict__ alpha2) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  rest[b] = failed[b] && ok_r[b];
  alpha2[b] = 2.0 * alpha[b];
}

// IPOPT's limited-memory quasi-Newton model (LimMemQuasiNewtonUpdater [IPOPT] with the defaults
// IFOPT's IpoptSolver leaves in place behind src/CentroidalPlanner.cpp:22-29: update type bfgs,
// limited_memory_max_history 6, initialization scalar1, init_val 1 (bounds 1e-8 / 1e8),
// max_skipping 2; every variable is nonlinear since IFOPT declares no linear ones), over x_free,
// one workgroup per active instance (batch_ipm step(), use_bfgs):
//   s = dw_free, y = grad_x L(w_new, y_new) - grad_x L(w, y_new)  (the Jacobian parts from A = [J_free | -P]);
//   the pair is skipped when s'y <= sqrt(eps) |s| |y|; more than max_skipping consecutive skips
//   reset the memory (model back to init_val I), and so does a failed line search (the step came
//   from the feasibility step standing in for IPOPT's restoration phase, whose return restarts the
//   quasi-Newton model; without it the degenerate TestBasic ground problem — force weight 0 —
//   stalls on a model whose scalar1 sigma collapsed along a flat direction);
//   otherwise the pair enters the memory (the oldest of 6 dropped), sigma = s'y / s's of the newest
//   pair clamped to [1e-8, 1e8], and the dense model is rebuilt from sigma I by the BFGS recursion
//   over the stored pairs, oldest first: B <- B - (Bs)(Bs)' / s'Bs + y y' / s'y  (mathematically the
//   compact representation IPOPT applies; B stays bitwise symmetric: every update is an outer product).
constexpr int LM_HIST = 6, LM_MAX_SKIP = 2;
// doubles per instance of the compact model: sigma, the number of pairs nv, U [LM_HIST][nf], W [LM_HIST][nf]
__host__ __device__ constexpr int64_t LMC(int nf) { return 2 + 2 * (int64_t)LM_HIST * nf; }
__global__ __launch_bounds__(256) void k_lbfgs(int64_t B, int m, int nf, int nw, int nnz_rec,
                                               const int32_t* __restrict__ amap, const uint8_t* __restrict__ act,
                                               const double* __restrict__ w_old, const double* __restrict__ w_new,
                                               const double* __restrict__ y, const double* __restrict__ dy,
                                               const double* __restrict__ alpha, const double* __restrict__ gw_old,
                                               const double* __restrict__ J_old, const double* __restrict__ gw_new,
                                               const double* __restrict__ J_new, double* __restrict__ lm_s,
                                               double* __restrict__ lm_y, uint8_t* __restrict__ lm_cnt,
                                               uint8_t* __restrict__ lm_skip, const uint8_t* __restrict__ failed,
                                               double* __restrict__ Hq) {
  const int64_t b = blockIdx.x;
  if (b >= B || !act[b]) return;
  __shared__ double Ps[LM_HIST][128], Py[LM_HIST][128], yn[256], red[8];
  const int tid = threadIdx.x;
  const double al = alpha[b];
  for (int r = tid; r < m; r += blockDim.x) yn[r] = y[b * m + r] + al * dy[b * m + r];
  // both counters read before any barrier: thread 0 rewrites them below
  const int cnt = lm_cnt[b], skipped = lm_skip[b] + 1;
  __syncthreads();
  // the new pair goes to slot `last`; a full memory shifts down by one (the oldest dropped)
  const int shift = cnt == LM_HIST ? 1 : 0, last = cnt - shift;
  double* gs = lm_s + b * (int64_t)LM_HIST * nf;
  double* gy = lm_y + b * (int64_t)LM_HIST * nf;
  {  // J_free^T y at both points, straight from the values-only Jacobian records (the entries of A =
     // [J_free | -P] as cpl_ipm_dense_a forms them: amap -1 = 0, -2 = constant 1, NaN = 0); the rows
     // split over `parts` thread groups, partials summed in fixed order
    __shared__ double pjn[4][128], pjo[4][128];
    const int kp = nf <= 64 ? 64 : 128, parts = (int)blockDim.x / kp;
    const int k = tid % kp, part = tid / kp;
    if (k < nf && part < parts) {
      const double* jnb = J_new + b * (int64_t)nnz_rec;
      const double* job = J_old + b * (int64_t)nnz_rec;
      double jn = 0.0, jo = 0.0;
      for (int r = part; r < m; r += parts) {
        const int q = amap[r * nf + k];
        if (q == -1) continue;  // structural zero: A's entry is 0
        double an = 1.0, ao = 1.0;
        if (q >= 0) {
          an = jnb[q];
          ao = job[q];
          an = an == an ? an : 0.0;
          ao = ao == ao ? ao : 0.0;
        }
        jn += an * yn[r];
        jo += ao * yn[r];
      }
      pjn[part][k] = jn;
      pjo[part][k] = jo;
    }
    __syncthreads();
    for (int k2 = tid; k2 < nf; k2 += blockDim.x) {
      double jn = pjn[0][k2], jo = pjo[0][k2];
      for (int q = 1; q < parts; ++q) {
        jn += pjn[q][k2];
        jo += pjo[q][k2];
      }
      Ps[last][k2] = w_new[b * nw + k2] - w_old[b * nw + k2];
      Py[last][k2] = (gw_new[b * nw + k2] + jn) - (gw_old[b * nw + k2] + jo);
      for (int j = 0; j < last; ++j) {
        Ps[j][k2] = gs[(j + shift) * nf + k2];
        Py[j][k2] = gy[(j + shift) * nf + k2];
      }
    }
  }
  __syncthreads();
  auto block_dot = [&](const double* a, const double* c) {
    double v = 0.0;
    for (int k = tid; k < nf; k += blockDim.x) v += a[k] * c[k];
    v = wave_sum(v);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    double t = 0.0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) t += red[q];
    return t;
  };
  const double sy = block_dot(Ps[last], Py[last]);
  const double ss = block_dot(Ps[last], Ps[last]);
  const double yy = block_dot(Py[last], Py[last]);
  double* hc = Hq + b * (int64_t)LMC(nf);  // the compact model: [sigma, nv, U, W]
  const bool skip = !(sy > sqrt(DBL_EPSILON) * sqrt(ss) * sqrt(yy));
  if (skip || failed[b]) {  // (uniform branch)
    if (!failed[b] && skipped <= LM_MAX_SKIP) {
      if (tid == 0) lm_skip[b] = (uint8_t)skipped;
      return;
    }
    if (tid == 0) {  // the model back to init_val I
      hc[0] = 1.0;
      hc[1] = 0.0;
      lm_skip[b] = 0;
      lm_cnt[b] = 0;
    }
    return;
  }
  const int nc = last + 1;
  for (int k = tid; k < nf; k += blockDim.x)
    for (int j = 0; j < nc; ++j) {
      gs[j * nf + k] = Ps[j][k];
      gy[j * nf + k] = Py[j][k];
    }
  if (tid == 0) {
    lm_skip[b] = 0;
    lm_cnt[b] = (uint8_t)nc;
  }
  const double sigma = fmin(fmax(sy / ss, 1e-8), 1e8);
  // The recursion unrolled onto vectors: a_j = B_j s_j = sigma s_j + sum_{i<j} [y_i (y_i's_j) / s_i'y_i
  // - a_i (a_i's_j) / s_i'a_i] (pair i taken when s_i'a_i > 0), on wave 0 with lanes over x_free
  // (two entries per lane, wave sums: no barriers); then every entry of
  // B = sigma I + sum_i [-(a_i a_i') / s_i'a_i + (y_i y_i') / s_i'y_i] once (as products of the scaled
  // vectors a_i / sqrt(s_i'a_i), y_i / sqrt(s_i'y_i)), straight to global
  // memory.  Same model as the dense rank-2 recursion (which re-read and re-wrote B six times).
  __shared__ double Pa[LM_HIST][128], s_sa[LM_HIST], s_sy[LM_HIST];
  if (tid < 64) {
    const int k0 = tid, k1 = tid + 64;
    const bool h0 = k0 < nf, h1 = k1 < nf;
    for (int j = 0; j < nc; ++j) {
      const double s0 = h0 ? Ps[j][k0] : 0.0, s1 = h1 ? Ps[j][k1] : 0.0;
      double v0 = sigma * s0, v1 = sigma * s1;
      for (int i = 0; i < j; ++i) {
        if (!(s_sa[i] > 0.0)) continue;  // (uniform)
        const double a0 = h0 ? Pa[i][k0] : 0.0, a1 = h1 ? Pa[i][k1] : 0.0;
        const double y0 = h0 ? Py[i][k0] : 0.0, y1 = h1 ? Py[i][k1] : 0.0;
        const double as = wave_sum(a0 * s0 + a1 * s1) / s_sa[i];
        const double ys = wave_sum(y0 * s0 + y1 * s1) / s_sy[i];
        v0 = (v0 - a0 * as) + y0 * ys;
        v1 = (v1 - a1 * as) + y1 * ys;
      }
      if (h0) Pa[j][k0] = v0;
      if (h1) Pa[j][k1] = v1;
      const double y0 = h0 ? Py[j][k0] : 0.0, y1 = h1 ? Py[j][k1] : 0.0;
      const double sa = wave_sum(s0 * v0 + s1 * v1);
      const double sjy = wave_sum(s0 * y0 + s1 * y1);
      if (tid == 0) {
        s_sa[j] = sa;
        s_sy[j] = sjy;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // lane 0's s_sa / s_sy visible to the next j
    }
    // scaled in place, u_i = a_i / sqrt(s_i'a_i) and v_i = y_i / sqrt(s_i'y_i) (both > 0 for a taken
    // pair), so that every model entry is a sum of products u_r u_c, v_r v_c: symmetric bit for bit
    for (int i = 0; i < nc; ++i) {
      if (!(s_sa[i] > 0.0)) continue;
      const double qa = sqrt(s_sa[i]), qy = sqrt(s_sy[i]);
      if (h0) { Pa[i][k0] /= qa; Py[i][k0] /= qy; }
      if (h1) { Pa[i][k1] /= qa; Py[i][k1] /= qy; }
    }
  }
  __syncthreads();
  // the taken pairs (s_i'a_i > 0: always, for a positive definite model) in order, as the compact
  // model the Newton setup expands entry by entry (ipm_newton_setup_lm)
  for (int e = tid; e < nc * nf; e += blockDim.x) {
    const int i = e / nf, k = e - i * nf;
    if (!(s_sa[i] > 0.0)) continue;
    int pos = 0;
    for (int q = 0; q < i; ++q) pos += s_sa[q] > 0.0;
    hc[2 + pos * nf + k] = Pa[i][k];
    hc[2 + LM_HIST * nf + pos * nf + k] = Py[i][k];
  }
  if (tid == 0) {
    int nv = 0;
    for (int q = 0; q < nc; ++q) nv += s_sa[q] > 0.0;
    hc[0] = sigma;
    hc[1] = (double)nv;
  }
}

// the number of instances still active into one int (read by the host one iteration behind):
// zeroed by k_count_zero at the iteration's start, one atomic per workgroup
// up to COUNT1_MAX instances: one workgroup counts them and writes the count (no zeroing launch)
constexpr int64_t COUNT1_MAX = 65536;
__global__ __launch_bounds__(1024) void k_count1(int64_t B, const uint8_t* __restrict__ active,
                                                 int32_t* __restrict__ count) {
  __shared__ int s_w[16];
  int c = 0;
  for (int64_t b = threadIdx.x; b < B; b += 1024) c += active[b] ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int q = 0; q < 16; ++q) t += s_w[q];
    count[0] = t;
  }
}
// the accepted point's f, grad, g and Jacobian records into the iterate's, active instances only:
// one launch over the concatenated row [f | grad (n) | g (m) | J (nnz_rec)]
__global__ __launch_bounds__(256) void k_accept_rows(int64_t B, int n, int m, int nnz, const uint8_t* __restrict__ act,
                                                     const double* __restrict__ f_n, const double* __restrict__ grad_n,
                                                     const double* __restrict__ g_n, const double* __restrict__ J_n,
                                                     double* __restrict__ f, double* __restrict__ grad,
                                                     double* __restrict__ g, double* __restrict__ J) {
  const int64_t L = 1 + n + m + nnz;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * L) return;
  const int64_t b = e / L;
  if (!act[b]) return;
  int q = (int)(e - b * L);
  if (q == 0) { f[b] = f_n[b]; return; }
  q -= 1;
  if (q < n) { grad[b * n + q] = grad_n[b * n + q]; return; }
  q -= n;
  if (q < m) { g[b * m + q] = g_n[b * m + q]; return; }
  q -= m;
  J[b * nnz + q] = J_n[b * nnz + q];
}
__global__ void k_count_zero(int32_t* __restrict__ count) {
  if (threadIdx.x == 0 && blockIdx.x == 0) count[0] = 0;
}
__global__ __launch_bounds__(256) void k_count(int64_t B, const uint8_t* __restrict__ active, int32_t* __restrict__ count) {
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int a = (b < B && active[b]) ? 1 : 0;
  const unsigned long long bal = __ballot(a);
  if ((threadIdx.x & 63) == 0 && bal) atomicAdd(&s_cnt, __popcll(bal));
  __syncthreads();
  if (threadIdx.x == 0 && s_cnt) atomicAdd(count, s_cnt);
}

// ---- active-set compaction (the lock-step batch shrinks to its active instances) ----------
// pos[j] = the row of the j-th active instance (j < count), one workgroup scanning the flags
__global__ __launch_bounds__(1024) void k_positions(int64_t B, const uint8_t* __restrict__ active,
                                                    int32_t* __restrict__ pos) {
  __shared__ int s_base;
  __shared__ int s_wave[16];
  if (threadIdx.x == 0) s_base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t c0 = 0; c0 < B; c0 += blockDim.x) {
    const int64_t b = c0 + threadIdx.x;
    const int a = (b < B && active[b]) ? 1 : 0;
    const unsigned long long bal = __ballot(a);
    if (lane == 0) s_wave[wave] = __popcll(bal);
    __syncthreads();
    int off = s_base;
    for (int w = 0; w < wave; ++w) off += s_wave[w];
    if (a) pos[off + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)b;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_wave[w];
      s_base += t;
    }
    __syncthreads();
  }
}

// dst[j] = src[pos[j]] for rows of `len` 8-byte words (j < k); rows j in [k, rows) untouched
__global__ void k_gather_rows(int64_t k, int64_t len, const int32_t* __restrict__ pos, const uint64_t* __restrict__ src,
                              uint64_t* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= k * len) return;
  const int64_t j = e / len;
  dst[e] = src[(int64_t)pos[j] * len + (e - j * len)];
}
__global__ void k_gather_bytes(int64_t k, const int32_t* __restrict__ pos, const uint8_t* __restrict__ src,
                               uint8_t* __restrict__ dst) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < k) dst[j] = src[pos[j]];
}

// the final state of every row that leaves the batch (finished, or at the end: all rows), written
// to the instance's own position orig[r] of the full-batch result arrays
__global__ __launch_bounds__(256) void k_scatter_final(int64_t rows, int n, int m, int nw, bool finished_only,
                                                       const int32_t* __restrict__ orig, const uint8_t* __restrict__ active,
                                                       const double* __restrict__ w, const double* __restrict__ y,
                                                       const double* __restrict__ Xbase, const double* __restrict__ d_inf,
                                                       const int64_t* __restrict__ status, const int64_t* __restrict__ iters,
                                                       double* __restrict__ fw, double* __restrict__ fy,
                                                       double* __restrict__ fX, double* __restrict__ fdinf,
                                                       int64_t* __restrict__ fstatus, int64_t* __restrict__ fiters) {
  const int64_t r = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int32_t o = orig[r];
  if (o < 0 || (finished_only && active[r])) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) fw[(int64_t)o * nw + k] = w[r * nw + k];
  for (int k = lane; k < m; k += 64) fy[(int64_t)o * m + k] = y[r * m + k];
  for (int k = lane; k < n; k += 64) fX[(int64_t)o * n + k] = Xbase[r * n + k];
  if (lane == 0) {
    fdinf[o] = d_inf[r];
    fstatus[o] = status[r];
    fiters[o] = iters[r];
  }
}

__global__ void k_gather_i32(int64_t k, const int32_t* __restrict__ pos, const int32_t* __restrict__ src,
                             int32_t* __restrict__ dst) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < k) dst[j] = src[pos[j]];
}
__global__ void k_pad(int64_t k, int64_t rows, uint8_t* __restrict__ active, int32_t* __restrict__ orig) {
  const int64_t j = k + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= rows) return;
  active[j] = 0;
  orig[j] = -1;
}

__global__ void k_iota(int64_t B, int32_t* __restrict__ orig) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) orig[b] = (int32_t)b;
}

// results: max violation of g against its bounds, int32 copies of status / iterations
__global__ __launch_bounds__(256) void k_final(int64_t B, int m, const double* __restrict__ g, const double* __restrict__ gl,
                                               const double* __restrict__ gu, const int64_t* __restrict__ status,
                                               const int64_t* __restrict__ iters, double* __restrict__ pinf,
                                               int32_t* __restrict__ st32, int32_t* __restrict__ it32) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  double v = 0.0;
  for (int r = lane; r < m; r += 64) {
    const double gv = g[b * m + r];
    v = fmax(v, fmax(fmax(gl[r] - gv, gv - gu[r]), 0.0));
    if (gv != gv) v = INFINITY;
  }
  v = wave_max(v);
  if (lane == 0) {
    if (pinf) pinf[b] = v;
    if (st32) st32[b] = (int32_t)status[b];
    if (it32) it32[b] = (int32_t)iters[b];
  }
}

// the compact limited-memory model of every instance at init_val I: sigma = 1, no pairs
__global__ void k_lm_init(int64_t B, int nf, double* __restrict__ Hq) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Hq[b * LMC(nf)] = 1.0;
  Hq[b * LMC(nf) + 1] = 0.0;
}

__global__ void k_repeat(int64_t B, int rep, const double* __restrict__ src, double* __restrict__ dst,
                         const uint8_t* __restrict__ tsrc, uint8_t* __restrict__ tdst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * rep) return;
  if (src) dst[e] = src[e / rep];
  if (tsrc) tdst[e] = tsrc[e / rep];
}

// ------------------------------------------------------------------------------------------
struct Arena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  template <typename T>
  T* take(size_t count) {
    const size_t bytes = ((count ? count : 1) * sizeof(T) + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base + used);
    used += bytes;
    return p;
  }
};

}  // namespace
}  // namespace cpl

struct cpl_solver {
  cpl_problem_desc desc;
  cpl_solve_options opt;
  int64_t B = 0;
  int64_t Bcur = 0;  // rows in play: B, shrunk by active-set compaction
  int n = 0, m = 0, nnz = 0, nnz_rec = 0, nf = 0, nI = 0, nw = 0, nbounds = 0;
  bool analytic_H = false, bfgs = false, fd = false, fd_fused = true;
  hipStream_t stream = nullptr;
  hipGraph_t graph = nullptr;  // the graph of the current (Bcur, mass / tag presence)
  hipGraphExec_t gexec = nullptr;
  std::map<int64_t, std::pair<hipGraph_t, hipGraphExec_t>> graphs;  // every captured size
  hipEvent_t ev[2] = {nullptr, nullptr};
  uint8_t* h_flag = nullptr;  // pinned, 2 bytes
  cpl::Arena arena;
  const double* mass = nullptr;       // per solve
  const uint8_t* tag = nullptr;
  int64_t evals_per_step = 0;
  // problem constants (device)
  int32_t *free32, *ineq_row, *row_slack, *freepos, *amap, *col_ptr, *csc_k, *csc_row;
  int64_t *free64, *fixed64;
  uint8_t *is_fixed, *hasL, *hasU;
  double *xl, *xu, *gl, *gu, *wl0, *wu0, *zeros_w, *zeros_B;
  // state
  double *Xbase, *w, *y, *zL, *zU, *mu, *filt_t, *filt_p, *dwl, *f, *grad, *g, *J, *d_inf, *Hq, *lm_s, *lm_y, *theta_max,
      *theta_min;
  int64_t *status, *iters, *acc, *fcount;
  uint8_t *active, *lm_cnt, *lm_skip, *d_any;
  // iteration temporaries
  double *A, *gradw, *gradw_new, *c, *err0, *base, *mu_o, *ft, *fp, *tau, *X, *H, *M, *Mr, *r1, *r2, *gphi,
      *mr_diag, *theta_k, *phi_k, *dw, *dy, *delta_w, *delta_c, *dzL, *dzU, *a_max, *a_z, *gd, *ws;
  int64_t* fc;
  int32_t* info;
  uint8_t *act, *switch_ok, *searching, *st_aug, *ok, *soc, *ok_s, *failed, *ok_r, *rest;
  double *st_f, *st_g, *st_w, *st_alpha, *alpha, *alpha2, *th, *wt, *Xt, *f_t, *g_t;
  double *c_soc, *a_soc, *th_old, *r2s, *dws, *dys, *ws_, *Xs, *f_s, *g_s, *th_s;
  double *negc, *dwr, *dyr, *dwr_d, *dcr, *ar, *wr, *Xr, *f_r, *g_r, *th_r;
  int32_t* infor;
  double *Xn, *f_n, *grad_n, *g_n, *J_n, *Xp, *hfd, *gL, *mass_fd, *jac_fd, *grad_fd;
  uint8_t* tag_fd;
  double *fin_f, *fin_g;
  int32_t *st32, *it32;
  // compaction: original instance of each row, compacted masses / tags, full-batch results
  int32_t *orig, *pos, *d_count, *h_count = nullptr;
  double *mass_c, *fw, *fy, *fX, *fdinf;
  uint8_t* tag_c;
  int64_t *fstatus, *fiters;
  uint64_t* scratch;
  int64_t scratch_words = 0;
  int32_t compactions = 0;
};

namespace cpl {
namespace {

int32_t hip_err(hipError_t e, const char* what) {
  return fail(CPL_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HK(expr, what)                                   \
  do {                                                   \
    hipError_t e_ = (expr);                              \
    if (e_ != hipSuccess) return hip_err(e_, what);      \
  } while (0)
#define LAUNCHED(what) HK(hipGetLastError(), what)

int32_t eval_fg(cpl_solver* S, const double* X, double* fo, double* go) {
  return cpl_eval_batch(&S->desc, S->Bcur, X, S->mass, S->tag, go, nullptr, fo, nullptr, S->stream);
}
int32_t eval_full(cpl_solver* S, const double* X, double* fo, double* grado, double* go, double* jo) {
  return cpl_eval_batch_ex(&S->desc, S->Bcur, X, S->mass, S->tag, go, jo, fo, grado, nullptr, CPL_EVAL_JAC_FOLDED,
                           S->stream);
}

// One lock-step iteration of every instance (graph-capturable: no host synchronisation), in three
// phases: A = the Newton step and the first line-search trial with its second-order correction
// (+ the any-searching flag when `flag`), B = the remaining trials and the feasibility step, C = the
// accepted point's evaluation and the state update.  Small batches run them as separate graphs and
// skip B when no instance is still searching after A (the usual case: B is ~25 masked launches).
int32_t step_phase(cpl_solver* S, int phase, bool flag);
int32_t step(cpl_solver* S) {
  CK(step_phase(S, 1, false));
  CK(step_phase(S, 2, false));
  return step_phase(S, 3, false);
}
int32_t step_phase(cpl_solver* S, int phase, bool flag) {
  const int64_t B = S->Bcur;
  const int n = S->n, m = S->m, nf = S->nf, nw = S->nw;
  hipStream_t st = S->stream;
  const cpl_solve_options& o = S->opt;
  auto judge = [&](const double* wt, const double* ft_, const double* gt_, const double* al, const uint8_t* extra,
                   double* th, uint8_t* ok, int mode) {
    return cpl_ipm_judge_take(B, nw, m, nf, FMAX, S->row_slack, S->gl, S->hasL, S->hasU, S->wl0, S->wu0, wt, ft_, gt_,
                              al, S->mu_o, S->theta_k, S->phi_k, S->gd, S->switch_ok, S->theta_max, S->ft, S->fp,
                              extra, S->searching, S->st_f, S->st_g, S->st_w, S->st_alpha, S->st_aug, th, ok, mode,
                              st);
  };
  const int nls = o.max_ls > 0 ? o.max_ls : 1;
  // one trial of the filter line search (ls == 0: with the second-order correction), then the halving
  auto trial = [&](int ls, bool any) -> int32_t {
    CK(cpl_ipm_trial_point(B, n, nf, nw, S->free64, S->fixed64, S->Xbase, S->w, S->dw, S->alpha, S->searching,
                           S->st_w, S->wt, S->Xt, st));
    CK(eval_fg(S, S->Xt, S->f_t, S->g_t));
    CK(judge(S->wt, S->f_t, S->g_t, S->alpha, nullptr, S->th, S->ok, 0));
    if (ls == 0 && o.max_soc > 0) {
      const double *cg = S->g_t, *cw = S->wt;
      for (int q = 0; q < o.max_soc; ++q) {
        if (q == 0) {
          hipLaunchKernelGGL(k_soc_begin_rhs, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nf, nw, S->searching, S->th,
                             S->theta_k, S->c, S->alpha, S->row_slack, S->gl, cg, cw, S->soc, S->c_soc, S->a_soc,
                             S->th_old, S->r2s);
          LAUNCHED("k_soc_begin_rhs");
        } else {
          hipLaunchKernelGGL(k_soc_rhs, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nf, nw, S->row_slack, S->gl, cg,
                             cw, S->a_soc, S->c_soc, S->r2s);
          LAUNCHED("k_soc_rhs");
        }
        CK(cpl_kkt_solve(1, B, nw, m, S->M, S->A, S->r1, S->r2s, nullptr, nullptr, S->soc, S->dws, S->dys, nullptr,
                         nullptr, nullptr, S->ws, st));
        CK(cpl_ipm_max_step(B, nw, S->w, S->dws, nullptr, nullptr, S->hasL, S->hasU, S->wl0, S->wu0, S->tau, S->a_soc,
                            st));
        CK(cpl_ipm_trial_point(B, n, nf, nw, S->free64, S->fixed64, S->Xbase, S->w, S->dws, S->a_soc, S->soc, S->st_w,
                               S->ws_, S->Xs, st));
        CK(eval_fg(S, S->Xs, S->f_s, S->g_s));
        CK(judge(S->ws_, S->f_s, S->g_s, S->alpha, S->soc, S->th_s, S->ok_s, 0));
        if (q + 1 == o.max_soc) {  // the last correction: its bookkeeping with the halving
          hipLaunchKernelGGL(k_soc_after_halve, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->soc, S->ok_s, S->th_s,
                             S->th_old, S->searching, S->alpha, any ? S->d_any : nullptr);
          LAUNCHED("k_soc_after_halve");
          return CPL_OK;
        }
        hipLaunchKernelGGL(k_soc_after, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->soc, S->ok_s, S->th_s,
                           S->th_old);
        LAUNCHED("k_soc_after");
        cg = S->g_s;
        cw = S->ws_;
      }
    }
    hipLaunchKernelGGL(k_halve, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->searching, S->alpha);
    LAUNCHED("k_halve");
    if (any) {
      hipLaunchKernelGGL(k_any_searching, dim3(1), dim3(256), 0, st, B, S->searching, S->d_any);
      LAUNCHED("k_any_searching");
    }
    return CPL_OK;
  };
  if (phase == 1) {
    // optimality error, convergence test, barrier update (filters reset where mu changed)
    if (B > COUNT1_MAX) {  // (k_count accumulates with atomics; small batches use k_count1 at the end)
      hipLaunchKernelGGL(k_count_zero, dim3(1), dim3(64), 0, st, S->d_count);
      LAUNCHED("k_count_zero");
    }
    CK(cpl_ipm_dense_a(B, m, nw, nf, S->nnz_rec, S->amap, S->row_slack, S->J, S->A, S->active, st));
    hipLaunchKernelGGL(k_prep, dim3(blocks_for(B)), dim3(256), 0, st, B, n, m, nf, nw, S->free32, S->row_slack, S->gl,
                       S->grad, S->g, S->w, S->gradw, S->c);
    LAUNCHED("k_prep");
    CK(cpl_ipm_optimality(B, nw, m, FMAX, S->nbounds, o.tol, o.acceptable_tol, o.acceptable_iter, S->A, S->gradw, S->c,
                          S->w, S->y, S->zL, S->zU, S->hasL, S->hasU, S->wl0, S->wu0, S->mu, S->filt_t, S->filt_p,
                          S->fcount, S->active, S->status, S->acc, S->d_inf, S->err0, S->base, S->mu_o, S->ft, S->fp,
                          S->fc, st));
    hipLaunchKernelGGL(k_unpack_tau, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, nw, S->freepos, S->Xbase,
                       S->w, S->mu_o, S->active, S->X, S->tau, S->act);
    LAUNCHED("k_unpack_tau");
    // Hessian of the Lagrangian over x_free
    const double* Hblk = nullptr;
    int h_sym = 0;
    if (S->bfgs) {
      // the compact model is expanded inside the Newton setup (ipm_newton_setup_lm below)
    } else if (S->analytic_H) {
      CK(cpl_lagrangian_hessian(&S->desc, B, S->X, S->y, S->act, S->free32, nf, S->H, st));
      Hblk = S->H;
    } else {  // central differences of grad f + J^T y (the 2 nf points of every instance in one launch)
      CK(cpl_ipm_fd_points(B, n, nf, o.fd_step, S->freepos, S->X, S->Xp, S->hfd, S->act, st));
      int32_t rc = CPL_ERR_UNSUPPORTED;
      if (S->fd_fused)
        rc = cpl_eval_lagrangian_grad(&S->desc, B * 2 * nf, S->Xp, S->mass ? S->mass_fd : nullptr,
                                      S->tag ? S->tag_fd : nullptr, S->col_ptr, S->csc_k, S->csc_row, S->y, 2 * nf,
                                      S->act, S->gL, st);
      if (rc == CPL_ERR_UNSUPPORTED) {  // Superquadric / mixed: eval + J^T y in two launches
        S->fd_fused = false;
        CK(cpl_eval_batch(&S->desc, B * 2 * nf, S->Xp, S->mass ? S->mass_fd : nullptr, S->tag ? S->tag_fd : nullptr,
                          nullptr, S->jac_fd, nullptr, S->grad_fd, st));
        CK(cpl_lagrangian_grad(B * 2 * nf, n, m, S->nnz, S->col_ptr, S->csc_k, S->csc_row, S->grad_fd, S->jac_fd, S->y,
                               2 * nf, S->gL, st));
      } else {
        CK(rc);
      }
      CK(cpl_ipm_fd_hessian_raw(B, n, nf, S->free64, S->gL, S->hfd, S->H, S->act, st));
      Hblk = S->H;
      h_sym = 1;
    }
    // Newton system, step, multiplier steps, fraction-to-the-boundary steps
    if (S->bfgs)
      CK(ipm_newton_setup_lm(B, nw, m, nf, S->w, S->zL, S->zU, S->gradw, S->A, S->y, S->c, S->f, S->mu_o, S->hasL,
                             S->hasU, S->wl0, S->wu0, S->Hq, LM_HIST, S->M, S->r1, S->r2, S->gphi, S->mr_diag,
                             S->theta_k, S->phi_k, nullptr, st));
    else
      CK(cpl_ipm_newton_setup(B, nw, m, nf, S->w, S->zL, S->zU, S->gradw, S->A, S->y, S->c, S->f, S->mu_o, S->hasL,
                              S->hasU, S->wl0, S->wu0, Hblk, h_sym, S->M, S->r1, S->r2, S->gphi, S->mr_diag, S->theta_k,
                              S->phi_k, S->act, st));
    CK(cpl_kkt_solve(0, B, nw, m, S->M, S->A, S->r1, S->r2, S->mu_o, S->dwl, S->act, S->dw, S->dy, S->delta_w,
                     S->delta_c, S->info, S->ws, st));
    CK(cpl_ipm_post_step(B, nw, S->w, S->dw, S->zL, S->zU, S->gphi, S->mu_o, S->tau, S->hasL, S->hasU, S->wl0, S->wu0,
                         S->theta_k, S->theta_min, S->act, S->delta_w, S->dwl, S->dzL, S->dzU, S->a_max, S->a_z, S->gd,
                         S->switch_ok, st));
    // filter line search with a second-order correction on the first trial
    hipLaunchKernelGGL(k_ls_init, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nw, S->act, S->f, S->g, S->w, S->a_max,
                       S->searching, S->st_f, S->st_g, S->st_w, S->st_alpha, S->st_aug, S->alpha, S->failed, S->rest,
                       flag ? S->d_any : nullptr);
    LAUNCHED("k_ls_init");
    CK(trial(0, flag));  // (with `flag`: the any-searching flag for the split iteration)
    return CPL_OK;
  }
  if (phase == 2) {
    for (int ls = 1; ls < nls; ++ls) CK(trial(ls, false));
    // no acceptable trial: the feasibility step (min 1/2 dw^T (Sigma + sqrt(mu) D_R^2) dw s.t. A dw = -c)
    // stands in for IPOPT's restoration phase, taken when it cuts the violation by 10 %; else the last trial
    hipLaunchKernelGGL(k_feas_prep, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nw, S->searching, S->mr_diag, S->c,
                       S->failed, S->Mr, S->negc);
    LAUNCHED("k_feas_prep");
    CK(cpl_kkt_solve(0, B, nw, m, S->Mr, S->A, S->zeros_w, S->negc, S->mu_o, S->zeros_B, S->failed, S->dwr, S->dyr,
                     S->dwr_d, S->dcr, S->infor, S->ws, st));
    CK(cpl_ipm_max_step(B, nw, S->w, S->dwr, nullptr, nullptr, S->hasL, S->hasU, S->wl0, S->wu0, S->tau, S->ar, st));
    CK(cpl_ipm_trial_point(B, n, nf, nw, S->free64, S->fixed64, S->Xbase, S->w, S->dwr, S->ar, S->failed, S->st_w, S->wr,
                           S->Xr, st));
    CK(eval_fg(S, S->Xr, S->f_r, S->g_r));
    CK(judge(S->wr, S->f_r, S->g_r, S->zeros_B, S->failed, S->th_r, S->ok_r, 1));
    hipLaunchKernelGGL(k_rest, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->failed, S->ok_r, S->alpha, S->rest,
                       S->alpha2);
    LAUNCHED("k_rest");
    CK(judge(S->wt, S->f_t, S->g_t, S->alpha2, nullptr, S->th, S->ok, 2));
    return CPL_OK;
  }
  // the accepted points with their derivatives: one full evaluation
  hipLaunchKernelGGL(k_unpack, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, nw, S->freepos, S->Xbase,
                     S->st_w, nullptr, nullptr, S->Xn);
  LAUNCHED("k_unpack");
  CK(eval_full(S, S->Xn, S->f_n, S->grad_n, S->g_n, S->J_n));
  if (S->bfgs) {
    hipLaunchKernelGGL(k_prep, dim3(blocks_for(B)), dim3(256), 0, st, B, n, m, nf, nw, S->free32, S->row_slack, S->gl,
                       S->grad_n, S->g_n, S->st_w, S->gradw_new, nullptr);
    LAUNCHED("k_prep (new)");
    hipLaunchKernelGGL(k_lbfgs, dim3((unsigned)B), dim3(256), 0, st, B, m, nf, nw, S->nnz_rec, S->amap, S->act, S->w, S->st_w, S->y, S->dy,
                       S->st_alpha, S->gradw, S->J, S->gradw_new, S->J_n, S->lm_s, S->lm_y, S->lm_cnt, S->lm_skip,
                       S->failed, S->Hq);
    LAUNCHED("k_lbfgs");
  }
  CK(cpl_ipm_accept(B, nw, m, FMAX, S->act, S->st_aug, S->failed, S->rest, S->st_alpha, S->a_z, S->theta_k, S->phi_k,
                    S->ft, S->fp, S->fc, S->st_w, S->dy, S->dzL, S->dzU, S->mu_o, S->hasL, S->hasU, S->wl0, S->wu0,
                    S->w, S->y, S->zL, S->zU, S->mu, S->iters, S->filt_t, S->filt_p, S->fcount, st));
  hipLaunchKernelGGL(k_accept_rows, dim3(blocks_elems(B * (1 + n + m + S->nnz_rec))), dim3(256), 0, st, B, n, m,
                     S->nnz_rec, S->act, S->f_n, S->grad_n, S->g_n, S->J_n, S->f, S->grad, S->g, S->J);
  LAUNCHED("k_accept_rows");
  if (B > COUNT1_MAX)
    hipLaunchKernelGGL(k_count, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->active, S->d_count);
  else
    hipLaunchKernelGGL(k_count1, dim3(1), dim3(1024), 0, st, B, S->active, S->d_count);
  LAUNCHED("k_count");
  return CPL_OK;
}

// the graph of one iteration at the current batch size (captured once per size, then replayed)
// phase 0: the whole iteration (S->graph / S->gexec); 1..3: the split iteration's phases (*ex)
int32_t graph_for(cpl_solver* S, int phase = 0, hipGraphExec_t* ex_out = nullptr) {
  const int64_t key = (S->Bcur * 4 + (S->mass ? 2 : 0) + (S->tag ? 1 : 0)) * 4 + phase;
  auto it = S->graphs.find(key);
  if (it == S->graphs.end()) {
    HK(hipStreamBeginCapture(S->stream, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
    const int32_t rc = phase == 0 ? step(S) : step_phase(S, phase, phase == 1);
    hipGraph_t gr = nullptr;
    const hipError_t e = hipStreamEndCapture(S->stream, &gr);
    if (rc != CPL_OK) {
      if (gr) (void)hipGraphDestroy(gr);
      return rc;
    }
    HK(e, "hipStreamEndCapture");
    hipGraphExec_t ex = nullptr;
    const hipError_t e2 = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    if (e2 != hipSuccess) {
      (void)hipGraphDestroy(gr);
      return hip_err(e2, "hipGraphInstantiate");
    }
    it = S->graphs.emplace(key, std::make_pair(gr, ex)).first;
  }
  if (phase == 0) {
    S->graph = it->second.first;
    S->gexec = it->second.second;
  } else {
    *ex_out = it->second.second;
  }
  return CPL_OK;
}

// Active-set compaction: the finished rows' results go to the full-batch arrays, the `count` active
// rows move to the front (every per-instance state buffer gathered), the batch shrinks to Bn rows
// (the rows past `count` padded inactive), so later iterations cost what their active instances do.
int32_t compact(cpl_solver* S, int64_t count, int64_t Bn) {
  hipStream_t st = S->stream;
  const int64_t Bc = S->Bcur;
  const int n = S->n, m = S->m, nw = S->nw;
  hipLaunchKernelGGL(k_scatter_final, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, n, m, nw, true, S->orig, S->active,
                     S->w, S->y, S->Xbase, S->d_inf, S->status, S->iters, S->fw, S->fy, S->fX, S->fdinf, S->fstatus,
                     S->fiters);
  LAUNCHED("k_scatter_final");
  hipLaunchKernelGGL(k_positions, dim3(1), dim3(1024), 0, st, Bc, S->active, S->pos);
  LAUNCHED("k_positions");
  auto move = [&](void* buf, int64_t words) -> int32_t {
    if (!buf || words <= 0) return CPL_OK;
    hipLaunchKernelGGL(k_gather_rows, dim3(blocks_elems(count * words)), dim3(256), 0, st, count, words, S->pos,
                       (const uint64_t*)buf, S->scratch);
    LAUNCHED("k_gather_rows");
    HK(hipMemcpyAsync(buf, S->scratch, 8 * (size_t)(count * words), hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    return CPL_OK;
  };
  const int nf = S->nf;
  CK(move(S->w, nw)); CK(move(S->y, m)); CK(move(S->zL, nw)); CK(move(S->zU, nw)); CK(move(S->mu, 1));
  CK(move(S->filt_t, FMAX)); CK(move(S->filt_p, FMAX)); CK(move(S->dwl, 1)); CK(move(S->f, 1));
  CK(move(S->grad, n)); CK(move(S->g, m)); CK(move(S->J, S->nnz_rec)); CK(move(S->d_inf, 1));
  CK(move(S->theta_max, 1)); CK(move(S->theta_min, 1)); CK(move(S->Xbase, n));
  CK(move(S->status, 1)); CK(move(S->iters, 1)); CK(move(S->acc, 1)); CK(move(S->fcount, 1));
  if (S->bfgs) {
    CK(move(S->Hq, LMC(nf)));
    CK(move(S->lm_s, (int64_t)LM_HIST * nf));
    CK(move(S->lm_y, (int64_t)LM_HIST * nf));
  }
  if (S->mass) CK(move(S->mass_c, 1));
  // 1-byte and 4-byte rows
  auto move_bytes = [&](uint8_t* buf) -> int32_t {
    hipLaunchKernelGGL(k_gather_bytes, dim3(blocks_elems(count)), dim3(256), 0, st, count, S->pos, buf,
                       (uint8_t*)S->scratch);
    LAUNCHED("k_gather_bytes");
    HK(hipMemcpyAsync(buf, S->scratch, (size_t)count, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    return CPL_OK;
  };
  CK(move_bytes(S->active));
  CK(move_bytes(S->lm_cnt));
  CK(move_bytes(S->lm_skip));
  if (S->tag) CK(move_bytes(S->tag_c));
  hipLaunchKernelGGL(k_gather_i32, dim3(blocks_elems(count)), dim3(256), 0, st, count, S->pos, S->orig,
                     (int32_t*)S->scratch);
  LAUNCHED("k_gather_i32");
  HK(hipMemcpyAsync(S->orig, S->scratch, 4 * (size_t)count, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
  hipLaunchKernelGGL(k_pad, dim3(blocks_elems(Bn)), dim3(256), 0, st, count, Bn, S->active, S->orig);
  LAUNCHED("k_pad");
  S->Bcur = Bn;
  if (S->fd && (S->mass || S->tag)) {
    hipLaunchKernelGGL(k_repeat, dim3(blocks_elems(Bn * 2 * nf)), dim3(256), 0, st, Bn, 2 * nf, S->mass,
                       S->mass_fd, S->tag, S->tag_fd);
    LAUNCHED("k_repeat");
  }
  ++S->compactions;
  return CPL_OK;
}

}  // namespace
}  // namespace cpl

using namespace cpl;

extern "C" {

void cpl_solve_options_default(cpl_solve_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->max_iter = 3000;
  o->hessian = CPL_HESSIAN_EXACT;
  o->max_ls = 4;
  o->max_soc = 1;
  o->acceptable_iter = 15;
  o->use_graph = 1;
  o->compact = 1;
  o->tol = 1e-8;
  o->acceptable_tol = 1e-6;
  o->mu_init = 0.1;
  o->fd_step = 1e-6;
}

int32_t cpl_solver_destroy(cpl_solver* S) {
  if (!S) return CPL_OK;
  for (auto& g : S->graphs) {
    (void)hipGraphExecDestroy(g.second.second);
    (void)hipGraphDestroy(g.second.first);
  }
  S->graphs.clear();
  for (auto& e : S->ev)
    if (e) (void)hipEventDestroy(e);
  if (S->h_flag) (void)hipHostFree(S->h_flag);
  if (S->h_count) (void)hipHostFree(S->h_count);
  if (S->arena.base) (void)hipFree(S->arena.base);
  if (S->stream) (void)hipStreamDestroy(S->stream);
  delete S;
  return CPL_OK;
}

int32_t cpl_solver_dims(const cpl_solver* S, int32_t* nf, int32_t* n_ineq, int32_t* graph_captured) {
  if (!S) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_dims: null solver");
  if (nf) *nf = S->nf;
  if (n_ineq) *n_ineq = S->nI;
  if (graph_captured) *graph_captured = S->gexec != nullptr;
  return CPL_OK;
}

int32_t cpl_solver_stats(const cpl_solver* S, int32_t* compactions, int64_t* final_rows) {
  if (!S) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_stats: null solver");
  if (compactions) *compactions = S->compactions;
  if (final_rows) *final_rows = S->Bcur;
  return CPL_OK;
}

int32_t cpl_solver_create(const cpl_problem_desc* d, int64_t batch, const cpl_solve_options* o, cpl_solver** out) {
  if (!out) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_create: null output");
  *out = nullptr;
  int32_t st = validate_desc(d);
  if (st) return st;
  if (batch < 1 || batch > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_create: bad batch");
  cpl_solve_options opt;
  cpl_solve_options_default(&opt);
  if (o) opt = *o;
  if (opt.hessian < CPL_HESSIAN_EXACT || opt.hessian > CPL_HESSIAN_FD || opt.max_iter < 0 || opt.max_soc < 0 ||
      opt.max_ls < 0 || !(opt.tol > 0.0))
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_create: bad options");
  int32_t n, m, nnz;
  CK(cpl_dims(d, &n, &m, &nnz));
  std::vector<int32_t> iRow(nnz), jCol(nnz);
  CK(cpl_structure(d, iRow.data(), jCol.data(), nullptr));
  std::vector<double> xl(n), xu(n), gl(m), gu(m);
  CK(cpl_bounds(d, xl.data(), xu.data(), gl.data(), gu.data()));
  // free / fixed variables (IPOPT fixed_variable_treatment = make_parameter), inequality rows
  std::vector<int32_t> free_idx, fixed_idx, freepos(n, -1), ineq, row_slack(m, -1);
  std::vector<uint8_t> is_fixed(n, 0);
  for (int j = 0; j < n; ++j) {
    if (std::fabs(xu[j] - xl[j]) <= 1e-14 * std::fmax(1.0, std::fabs(xl[j]))) {
      is_fixed[j] = 1;
      fixed_idx.push_back(j);
    } else {
      freepos[j] = (int32_t)free_idx.size();
      free_idx.push_back(j);
    }
  }
  for (int r = 0; r < m; ++r)
    if (gl[r] != gu[r]) {
      row_slack[r] = (int32_t)ineq.size();
      ineq.push_back(r);
    }
  const int nf = (int)free_idx.size(), nI = (int)ineq.size(), nw = nf + nI;
  if (nw > 128) return fail(CPL_ERR_UNSUPPORTED, "cpl_solver_create: more than 128 primal-slack unknowns");
  if (m > nw) return fail(CPL_ERR_UNSUPPORTED, "cpl_solver_create: more constraints than primal-slack unknowns");
  // w bounds: [x_free, s] against [x_l, g_l(I)] / [x_u, g_u(I)], relaxed by bound_relax_factor 1e-8
  std::vector<double> wl0(nw), wu0(nw);
  std::vector<uint8_t> hasL(nw), hasU(nw);
  int nbounds = 0;
  for (int k = 0; k < nw; ++k) {
    double lo = k < nf ? xl[free_idx[k]] : gl[ineq[k - nf]];
    double up = k < nf ? xu[free_idx[k]] : gu[ineq[k - nf]];
    if (k >= nf) {
      if (!(lo > -BIG)) lo = -INFINITY;
      if (!(up < BIG)) up = INFINITY;
    }
    lo = lo - 1e-8 * std::fmax(std::fabs(lo), 1.0);
    up = up + 1e-8 * std::fmax(std::fabs(up), 1.0);
    hasL[k] = std::isfinite(lo);
    hasU[k] = std::isfinite(up);
    wl0[k] = hasL[k] ? lo : 0.0;
    wu0[k] = hasU[k] ? up : 0.0;
    nbounds += hasL[k] + hasU[k];
  }
  // Jacobian records: the values-only layout (CPL_EVAL_JAC_FOLDED); amap = record position of
  // (row, free column), -1 structural zero / constant 0, -2 constant 1
  int32_t nnz_rec = 0, n_const = 0;
  CK(cpl_jac_fold_info(d, &nnz_rec, nullptr, &n_const, nullptr, nullptr));
  std::vector<int32_t> var_k(nnz_rec), const_k(n_const);
  std::vector<double> const_val(n_const);
  CK(cpl_jac_fold_info(d, &nnz_rec, var_k.data(), &n_const, const_k.data(), const_val.data()));
  std::vector<int32_t> rec(nnz, -1);
  for (int q = 0; q < nnz_rec; ++q) rec[var_k[q]] = q;
  for (int q = 0; q < n_const; ++q) rec[const_k[q]] = const_val[q] == 1.0 ? -2 : -1;
  std::vector<int32_t> amap((size_t)m * (nf ? nf : 1), -1);
  for (int k = 0; k < nnz; ++k)
    if (freepos[jCol[k]] >= 0) amap[(size_t)iRow[k] * nf + freepos[jCol[k]]] = rec[k];
  // CSC index of the full structure (central-difference Hessian: grad f + J^T y)
  std::vector<int32_t> col_ptr(n + 1, 0), csc_k(nnz), csc_row(nnz);
  for (int k = 0; k < nnz; ++k) ++col_ptr[jCol[k] + 1];
  for (int j = 0; j < n; ++j) col_ptr[j + 1] += col_ptr[j];
  {
    std::vector<int32_t> fill(col_ptr.begin(), col_ptr.end() - 1);
    for (int k = 0; k < nnz; ++k) {  // rows ascending within a column (CSR order)
      const int q = fill[jCol[k]]++;
      csc_k[q] = k;
      csc_row[q] = iRow[k];
    }
  }

  cpl_solver* S = new cpl_solver();
  S->desc = *d;
  S->opt = opt;
  S->B = batch;
  S->n = n; S->m = m; S->nnz = nnz; S->nnz_rec = nnz_rec; S->nf = nf; S->nI = nI; S->nw = nw; S->nbounds = nbounds;
  S->bfgs = opt.hessian == CPL_HESSIAN_LIMITED_MEMORY;
  S->analytic_H = opt.hessian == CPL_HESSIAN_EXACT && cpl_lagrangian_hessian(d, 0, nullptr, nullptr, nullptr, nullptr,
                                                                             nf > 0 ? nf : 1, nullptr, nullptr) == CPL_OK;
  S->fd = !S->bfgs && !S->analytic_H;
  auto bad = [&](hipError_t e, const char* what) {
    cpl_solver_destroy(S);
    return hip_err(e, what);
  };
  hipError_t e = hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking);
  if (e != hipSuccess) return bad(e, "hipStreamCreate");
  for (auto& ev : S->ev)
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
  if ((e = hipHostMalloc(&S->h_flag, 2)) != hipSuccess) return bad(e, "hipHostMalloc");
  if ((e = hipHostMalloc(&S->h_count, 2 * sizeof(int32_t))) != hipSuccess) return bad(e, "hipHostMalloc");
  // every device buffer carved from one allocation: a measuring pass, then the real one
  const size_t Bz = (size_t)batch, kws = (size_t)cpl_kkt_workspace_doubles(nw, m);
  const size_t nfd = S->fd ? Bz * 2 * nf : 0;
  {  // the widest per-instance row the compaction moves
    int64_t wmax = nnz_rec;
    for (int64_t v : {(int64_t)n, (int64_t)nw, (int64_t)m, (int64_t)FMAX, S->bfgs ? LMC(nf) : 0}) wmax = std::max(wmax, v);
    S->scratch_words = wmax;
  }
  auto carve = [&](Arena& a) {
  // constants
  S->free32 = a.take<int32_t>(nf); S->ineq_row = a.take<int32_t>(nI); S->row_slack = a.take<int32_t>(m);
  S->freepos = a.take<int32_t>(n); S->amap = a.take<int32_t>((size_t)m * (nf ? nf : 1));
  S->col_ptr = a.take<int32_t>(n + 1); S->csc_k = a.take<int32_t>(nnz); S->csc_row = a.take<int32_t>(nnz);
  S->free64 = a.take<int64_t>(nf); S->fixed64 = a.take<int64_t>(fixed_idx.size());
  S->is_fixed = a.take<uint8_t>(n); S->hasL = a.take<uint8_t>(nw); S->hasU = a.take<uint8_t>(nw);
  S->xl = a.take<double>(n); S->xu = a.take<double>(n); S->gl = a.take<double>(m); S->gu = a.take<double>(m);
  S->wl0 = a.take<double>(nw); S->wu0 = a.take<double>(nw);
  // state
  S->Xbase = a.take<double>(Bz * n); S->w = a.take<double>(Bz * nw); S->y = a.take<double>(Bz * m);
  S->zL = a.take<double>(Bz * nw); S->zU = a.take<double>(Bz * nw); S->mu = a.take<double>(Bz);
  S->filt_t = a.take<double>(Bz * FMAX); S->filt_p = a.take<double>(Bz * FMAX); S->dwl = a.take<double>(Bz);
  S->f = a.take<double>(Bz); S->grad = a.take<double>(Bz * n); S->g = a.take<double>(Bz * m);
  S->J = a.take<double>(Bz * nnz_rec); S->d_inf = a.take<double>(Bz); S->Hq = a.take<double>(S->bfgs ? Bz * LMC(nf) : 0);
  S->lm_s = a.take<double>(S->bfgs ? Bz * LM_HIST * nf : 0); S->lm_y = a.take<double>(S->bfgs ? Bz * LM_HIST * nf : 0);
  S->theta_max = a.take<double>(Bz); S->theta_min = a.take<double>(Bz);
  S->status = a.take<int64_t>(Bz); S->iters = a.take<int64_t>(Bz); S->acc = a.take<int64_t>(Bz);
  S->fcount = a.take<int64_t>(Bz); S->fc = a.take<int64_t>(Bz);
  S->active = a.take<uint8_t>(Bz); S->lm_cnt = a.take<uint8_t>(Bz); S->lm_skip = a.take<uint8_t>(Bz); S->d_any = a.take<uint8_t>(2);
  // temporaries
  S->A = a.take<double>(Bz * m * nw);
  S->gradw = a.take<double>(Bz * nw); S->gradw_new = a.take<double>(Bz * nw); S->c = a.take<double>(Bz * m);
  S->err0 = a.take<double>(Bz); S->base = a.take<double>(Bz); S->mu_o = a.take<double>(Bz);
  S->ft = a.take<double>(Bz * FMAX); S->fp = a.take<double>(Bz * FMAX); S->tau = a.take<double>(Bz);
  S->X = a.take<double>(Bz * n); S->H = a.take<double>(Bz * nf * nf); S->M = a.take<double>(Bz * nw * nw);
  S->Mr = a.take<double>(Bz * nw * nw); S->r1 = a.take<double>(Bz * nw); S->r2 = a.take<double>(Bz * m);
  S->gphi = a.take<double>(Bz * nw); S->mr_diag = a.take<double>(Bz * nw); S->theta_k = a.take<double>(Bz);
  S->phi_k = a.take<double>(Bz); S->dw = a.take<double>(Bz * nw); S->dy = a.take<double>(Bz * m);
  S->delta_w = a.take<double>(Bz); S->delta_c = a.take<double>(Bz); S->dzL = a.take<double>(Bz * nw);
  S->dzU = a.take<double>(Bz * nw); S->a_max = a.take<double>(Bz); S->a_z = a.take<double>(Bz);
  S->gd = a.take<double>(Bz); S->ws = a.take<double>(Bz * kws); S->info = a.take<int32_t>(Bz);
  S->act = a.take<uint8_t>(Bz); S->switch_ok = a.take<uint8_t>(Bz); S->searching = a.take<uint8_t>(Bz);
  S->st_aug = a.take<uint8_t>(Bz); S->ok = a.take<uint8_t>(Bz); S->soc = a.take<uint8_t>(Bz);
  S->ok_s = a.take<uint8_t>(Bz); S->failed = a.take<uint8_t>(Bz); S->ok_r = a.take<uint8_t>(Bz);
  S->rest = a.take<uint8_t>(Bz);
  S->st_f = a.take<double>(Bz); S->st_g = a.take<double>(Bz * m); S->st_w = a.take<double>(Bz * nw);
  S->st_alpha = a.take<double>(Bz); S->alpha = a.take<double>(Bz); S->alpha2 = a.take<double>(Bz);
  S->th = a.take<double>(Bz); S->wt = a.take<double>(Bz * nw); S->Xt = a.take<double>(Bz * n);
  S->f_t = a.take<double>(Bz); S->g_t = a.take<double>(Bz * m);
  S->c_soc = a.take<double>(Bz * m); S->a_soc = a.take<double>(Bz); S->th_old = a.take<double>(Bz);
  S->r2s = a.take<double>(Bz * m); S->dws = a.take<double>(Bz * nw); S->dys = a.take<double>(Bz * m);
  S->ws_ = a.take<double>(Bz * nw); S->Xs = a.take<double>(Bz * n); S->f_s = a.take<double>(Bz);
  S->g_s = a.take<double>(Bz * m); S->th_s = a.take<double>(Bz);
  S->negc = a.take<double>(Bz * m); S->dwr = a.take<double>(Bz * nw); S->dyr = a.take<double>(Bz * m);
  S->dwr_d = a.take<double>(Bz); S->dcr = a.take<double>(Bz); S->ar = a.take<double>(Bz);
  S->wr = a.take<double>(Bz * nw); S->Xr = a.take<double>(Bz * n); S->f_r = a.take<double>(Bz);
  S->g_r = a.take<double>(Bz * m); S->th_r = a.take<double>(Bz); S->infor = a.take<int32_t>(Bz);
  S->Xn = a.take<double>(Bz * n); S->f_n = a.take<double>(Bz); S->grad_n = a.take<double>(Bz * n);
  S->g_n = a.take<double>(Bz * m); S->J_n = a.take<double>(Bz * nnz_rec);
  S->zeros_w = a.take<double>(Bz * nw); S->zeros_B = a.take<double>(Bz);
  S->fin_f = a.take<double>(Bz); S->fin_g = a.take<double>(Bz * m);
  S->st32 = a.take<int32_t>(Bz); S->it32 = a.take<int32_t>(Bz);
  S->Xp = a.take<double>(nfd * n); S->gL = a.take<double>(nfd * n); S->hfd = a.take<double>(Bz * nf);
  S->mass_fd = a.take<double>(nfd); S->jac_fd = a.take<double>(nfd * nnz); S->grad_fd = a.take<double>(nfd * n);
  S->tag_fd = a.take<uint8_t>(nfd);
  S->orig = a.take<int32_t>(Bz); S->pos = a.take<int32_t>(Bz); S->d_count = a.take<int32_t>(2);
  S->mass_c = a.take<double>(Bz); S->tag_c = a.take<uint8_t>(Bz);
  S->fw = a.take<double>(Bz * nw); S->fy = a.take<double>(Bz * m); S->fX = a.take<double>(Bz * n);
  S->fdinf = a.take<double>(Bz); S->fstatus = a.take<int64_t>(Bz); S->fiters = a.take<int64_t>(Bz);
  S->scratch = a.take<uint64_t>(Bz * (size_t)S->scratch_words);
  };
  Arena probe;
  carve(probe);
  if ((e = hipMalloc(&S->arena.base, probe.used)) != hipSuccess) return bad(e, "hipMalloc solver arena");
  S->arena.cap = probe.used;
  carve(S->arena);
  // constants up, zero buffers
  std::vector<int64_t> f64(free_idx.begin(), free_idx.end()), x64(fixed_idx.begin(), fixed_idx.end());
  struct Up { void* dst; const void* src; size_t bytes; };
  const Up ups[] = {
      {S->free32, free_idx.data(), 4 * free_idx.size()}, {S->ineq_row, ineq.data(), 4 * ineq.size()},
      {S->row_slack, row_slack.data(), 4 * (size_t)m}, {S->freepos, freepos.data(), 4 * (size_t)n},
      {S->amap, amap.data(), 4 * amap.size()}, {S->col_ptr, col_ptr.data(), 4 * col_ptr.size()},
      {S->csc_k, csc_k.data(), 4 * (size_t)nnz}, {S->csc_row, csc_row.data(), 4 * (size_t)nnz},
      {S->free64, f64.data(), 8 * f64.size()}, {S->fixed64, x64.data(), 8 * x64.size()},
      {S->is_fixed, is_fixed.data(), (size_t)n}, {S->hasL, hasL.data(), (size_t)nw}, {S->hasU, hasU.data(), (size_t)nw},
      {S->xl, xl.data(), 8 * (size_t)n}, {S->xu, xu.data(), 8 * (size_t)n}, {S->gl, gl.data(), 8 * (size_t)m},
      {S->gu, gu.data(), 8 * (size_t)m}, {S->wl0, wl0.data(), 8 * (size_t)nw}, {S->wu0, wu0.data(), 8 * (size_t)nw}};
  for (const Up& u : ups)
    if (u.bytes && (e = hipMemcpy(u.dst, u.src, u.bytes, hipMemcpyHostToDevice)) != hipSuccess) return bad(e, "hipMemcpy");
  if ((e = hipMemset(S->zeros_w, 0, 8 * Bz * nw)) != hipSuccess || (e = hipMemset(S->zeros_B, 0, 8 * Bz)) != hipSuccess ||
      (e = hipMemset(S->Mr, 0, 8 * Bz * nw * nw)) != hipSuccess)
    return bad(e, "hipMemset");
  *out = S;
  return CPL_OK;
}

int32_t cpl_solver_solve(cpl_solver* S, const double* d_x0, const double* d_mass, const uint8_t* d_env_tag, double* d_x,
                         double* d_y, int32_t* d_status, int32_t* d_iters, double* d_obj, double* d_primal_inf,
                         double* d_dual_inf, int32_t* iterations_run, int64_t* evaluations, void* stream) {
  if (!S || !d_x0) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_solve: missing solver or x0");
  if (S->desc.env_kind == CPL_ENV_MIXED && !d_env_tag)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_solve: mixed batches need the env tags");
  const int64_t B = S->B;
  const int n = S->n, m = S->m, nf = S->nf, nw = S->nw;
  hipStream_t st = S->stream;
  // order after the caller's stream (its inputs), then run on the solver's own stream
  HK(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize (caller stream)");
  S->Bcur = B;
  S->compactions = 0;
  // the iteration reads the solver's own copies of the masses / tags (compaction reorders them), so
  // a captured graph never holds a caller's pointer
  S->mass = d_mass ? S->mass_c : nullptr;
  S->tag = d_env_tag ? S->tag_c : nullptr;
  if (d_mass) HK(hipMemcpyAsync(S->mass_c, d_mass, 8 * (size_t)B, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync mass");
  if (d_env_tag) HK(hipMemcpyAsync(S->tag_c, d_env_tag, (size_t)B, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync tag");
  hipLaunchKernelGGL(k_iota, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->orig);
  LAUNCHED("k_iota");
  int64_t evals = 0;
  if (S->fd && (d_mass || d_env_tag)) {
    hipLaunchKernelGGL(k_repeat, dim3(blocks_elems(B * 2 * nf)), dim3(256), 0, st, B, 2 * nf, S->mass, S->mass_fd,
                       S->tag, S->tag_fd);
    LAUNCHED("k_repeat");
  }
  // starting point: x pushed into its bounds, slacks = g_I(x) pushed into theirs, least-squares y
  hipLaunchKernelGGL(k_xbase, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, d_x0, S->is_fixed, S->xl, S->Xbase);
  LAUNCHED("k_xbase");
  hipLaunchKernelGGL(k_start_x, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, S->freepos, S->Xbase, S->hasL,
                     S->hasU, S->wl0, S->wu0, S->X);
  LAUNCHED("k_start_x");
  CK(eval_full(S, S->X, S->f, S->grad, S->g, S->J));
  ++evals;
  hipLaunchKernelGGL(k_init_state, dim3(blocks_for(B)), dim3(256), 0, st, B, n, m, nf, nw, S->free32, S->ineq_row,
                     S->row_slack, S->gl, S->hasL, S->hasU, S->wl0, S->wu0, S->opt.mu_init, S->X, S->g, S->grad, S->w,
                     S->zL, S->zU, S->theta_max, S->theta_min, S->mu, S->active, S->status, S->iters, S->acc,
                     S->filt_t, S->filt_p, S->fcount, S->dwl, S->d_inf, S->lm_cnt, S->lm_skip, S->r1, S->r2, S->M);
  LAUNCHED("k_init_state");
  CK(cpl_ipm_dense_a(B, m, nw, nf, S->nnz_rec, S->amap, S->row_slack, S->J, S->A, nullptr, st));
  CK(cpl_kkt_solve(0, B, nw, m, S->M, S->A, S->r1, S->r2, S->mu, S->zeros_B, nullptr, S->dw, S->dy, S->delta_w,
                   S->delta_c, S->info, S->ws, st));
  hipLaunchKernelGGL(k_y0, dim3(blocks_for(B)), dim3(256), 0, st, B, m, S->dy, S->info, S->y);
  LAUNCHED("k_y0");
  if (S->bfgs) {  // model initialised to init_val I (IPOPT's limited_memory_init_val = 1)
    hipLaunchKernelGGL(k_lm_init, dim3(blocks_elems(B)), dim3(256), 0, st, B, nf, S->Hq);
    LAUNCHED("k_lm_init");
  }
  const int64_t per_step_full = (S->fd ? 1 : 0) + (S->opt.max_ls > 0 ? S->opt.max_ls : 1) + S->opt.max_soc + 2;
  int it = 0;
  const int max_iter = S->opt.max_iter;
  const bool compacting = S->opt.compact != 0 && S->opt.use_graph;
  const int64_t min_rows = 256;
  if (max_iter > 0) {
    // first iteration executed (warms per-stream state, the eval kernels' launch geometry)
    CK(step(S));
    ++it;
    evals += per_step_full;
    if (S->opt.use_graph) CK(graph_for(S));
    HK(hipMemcpyAsync(S->h_count, S->d_count, 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync count");
    HK(hipStreamSynchronize(st), "hipStreamSynchronize");
    int last = S->h_count[0] ? max_iter : it;
    int start = it;
    // batches of at most SPLIT_MAX rows: the iteration as three graphs, the line search's later
    // trials and feasibility step (phase B) launched only when an instance is still searching after
    // the first trial (read back before the launch: one stream synchronisation per iteration, against
    // ~25 masked launches skipped in most iterations)
    constexpr int64_t SPLIT_MAX = 256;
    auto split_loop = [&]() -> int32_t {
      const int64_t evA = (S->fd ? 1 : 0) + 1 + S->opt.max_soc;
      const int64_t evB = (S->opt.max_ls > 0 ? S->opt.max_ls : 1) - 1 + 1;
      hipGraphExec_t ga = nullptr, gb = nullptr, gc = nullptr;
      CK(graph_for(S, 1, &ga));
      CK(graph_for(S, 2, &gb));
      CK(graph_for(S, 3, &gc));
      bool have_count = false;  // h_count[0] holds the count after the previous iteration
      while (it < last) {
        HK(hipGraphLaunch(ga, st), "hipGraphLaunch");
        HK(hipMemcpyAsync(S->h_flag, S->d_any, 1, hipMemcpyDeviceToHost, st), "hipMemcpyAsync flag");
        HK(hipStreamSynchronize(st), "hipStreamSynchronize");
        ++it;
        evals += evA + 1;
        if (have_count && S->h_count[0] == 0) break;  // converged in the previous iteration (this one was idle)
        if (S->h_flag[0]) {
          HK(hipGraphLaunch(gb, st), "hipGraphLaunch");
          evals += evB;
        }
        HK(hipGraphLaunch(gc, st), "hipGraphLaunch");
        HK(hipMemcpyAsync(S->h_count, S->d_count, 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync count");
        have_count = true;
      }
      return CPL_OK;
    };
    if (S->opt.use_graph && S->Bcur <= SPLIT_MAX) {
      CK(split_loop());
      last = it;
    }
    while (it < last) {
      if (S->opt.use_graph) HK(hipGraphLaunch(S->gexec, st), "hipGraphLaunch");
      else CK(step(S));
      ++it;
      evals += per_step_full;
      const int k = it & 1;
      HK(hipMemcpyAsync(S->h_count + k, S->d_count, 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync count");
      HK(hipEventRecord(S->ev[k], st), "hipEventRecord");
      if (it - start >= 2) {  // the previous iteration's count (normally landed already)
        HK(hipEventSynchronize(S->ev[k ^ 1]), "hipEventSynchronize");
        const int64_t cnt = S->h_count[k ^ 1];
        if (cnt == 0) break;
        if (compacting && S->Bcur > min_rows && 2 * cnt <= S->Bcur) {
          // shrink to the smallest halving of the current size that holds the active instances
          HK(hipStreamSynchronize(st), "hipStreamSynchronize");
          const int64_t now = S->h_count[k];
          if (now == 0) break;
          int64_t Bn = S->Bcur;
          while (Bn / 2 >= now && Bn / 2 >= min_rows) Bn = (Bn + 1) / 2;
          if (Bn < S->Bcur) {
            CK(compact(S, now, Bn));
            if (Bn <= SPLIT_MAX) {  // the rest of the solve as split iterations
              CK(split_loop());
              break;
            }
            CK(graph_for(S));
            start = it;  // the flag pipeline restarts at the new size
          }
        }
      }
    }
  }
  // final convergence test at the last iterate (the barrier update outputs go to scratch)
  const int64_t Bc = S->Bcur;
  CK(cpl_ipm_dense_a(Bc, m, nw, nf, S->nnz_rec, S->amap, S->row_slack, S->J, S->A, S->active, st));
  hipLaunchKernelGGL(k_prep, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, n, m, nf, nw, S->free32, S->row_slack, S->gl,
                     S->grad, S->g, S->w, S->gradw, S->c);
  LAUNCHED("k_prep");
  CK(cpl_ipm_optimality(Bc, nw, m, FMAX, S->nbounds, S->opt.tol, S->opt.acceptable_tol, S->opt.acceptable_iter, S->A,
                        S->gradw, S->c, S->w, S->y, S->zL, S->zU, S->hasL, S->hasU, S->wl0, S->wu0, S->mu, S->filt_t,
                        S->filt_p, S->fcount, S->active, S->status, S->acc, S->d_inf, S->err0, S->base, S->mu_o, S->ft,
                        S->fp, S->fc, st));
  // every row still in the batch to its instance's place in the full-batch results
  hipLaunchKernelGGL(k_scatter_final, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, n, m, nw, false, S->orig, S->active,
                     S->w, S->y, S->Xbase, S->d_inf, S->status, S->iters, S->fw, S->fy, S->fX, S->fdinf, S->fstatus,
                     S->fiters);
  LAUNCHED("k_scatter_final");
  // IPOPT honor_original_bounds: the final point projected into the original bounds, re-evaluated
  double* Xf = d_x ? d_x : S->Xn;
  hipLaunchKernelGGL(k_unpack, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, nw, S->freepos, S->fX, S->fw,
                     S->xl, S->xu, Xf);
  LAUNCHED("k_unpack (final)");
  CK(cpl_eval_batch(&S->desc, B, Xf, d_mass, d_env_tag, S->fin_g, nullptr, d_obj ? d_obj : S->fin_f, nullptr, st));
  ++evals;
  hipLaunchKernelGGL(k_final, dim3(blocks_for(B)), dim3(256), 0, st, B, m, S->fin_g, S->gl, S->gu, S->fstatus,
                     S->fiters, d_primal_inf, d_status, d_iters);
  LAUNCHED("k_final");
  if (d_y) HK(hipMemcpyAsync(d_y, S->fy, 8 * (size_t)B * m, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync y");
  if (d_dual_inf) HK(hipMemcpyAsync(d_dual_inf, S->fdinf, 8 * (size_t)B, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
  HK(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (iterations_run) *iterations_run = it;
  if (evaluations) *evaluations = evals;
  return CPL_OK;
}

}  // extern "C"
