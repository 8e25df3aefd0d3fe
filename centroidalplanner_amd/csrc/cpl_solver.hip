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

#include "cpl_accept.hpp"
#include "cpl_kkt_qd.hpp"
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
// cpl_kernels.hip: the backtracking line search after the first trial, one wave per instance
int32_t ls_backtrack(const cpl_problem_desc* d, const LsBacktrackArgs& a, hipStream_t stream);
// cpl_kernels.hip: the NLP-scaled evaluation (pipelined kernel; CPL_ERR_UNSUPPORTED: not that path)
int32_t eval_batch_scaled(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                          const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                          int32_t flags, const double* df, const double* dc, const int32_t* row, void* stream,
                          const uint8_t* gate = nullptr);
// cpl_kernels.hip: cpl_eval_batch_ex whose pipelined-kernel launch is a no-op while *gate == 0
int32_t eval_batch_gated(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                         const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                         int32_t flags, void* stream, const uint8_t* gate);
bool kkt_wave_size(int nw, int m);
int64_t kkt_aug_workspace_doubles(int nw, int m);
int32_t kkt_aug_solve(int mode, int64_t batch, int nw, int m, const double* d_M, const double* d_A, const double* d_r1,
                      const double* d_r2, const double* d_mu, const double* d_dwl, const uint8_t* d_active, double* d_dw,
                      double* d_dy, double* d_delta_w, double* d_delta_c, int32_t* d_info, double* d_wsa,
                      hipStream_t st);
bool ls_post_prologue(int64_t batch);
// cpl_ipm.hip: the post-step kernel with the line-search setup (LsSetupArgs) as its tail
int32_t ipm_post_step_ex(int64_t batch, int32_t nw, const double* d_w, const double* d_dw, const double* d_zL,
                         const double* d_zU, const double* d_gphi, const double* d_mu, const double* d_tau,
                         const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                         const double* d_theta, const double* d_theta_min, const uint8_t* d_active,
                         const double* d_delta_w, double* d_dwl, double* d_dzL, double* d_dzU, double* d_a_max,
                         double* d_a_z, double* d_gd, uint8_t* d_switch_ok, const LsSetupArgs* ls, void* stream);
// cpl_ipm.hip: the optimality test + monotone barrier update with IPOPT's per-iteration rounds
double ipm_mu_min(double tol);
int32_t ipm_optimality_ex(int64_t batch, int32_t nw, int32_t m, int32_t fmax, int32_t nbounds, double tol,
                          double acceptable_tol, int32_t acceptable_iter, const double* d_A, const double* d_gw,
                          const double* d_c, const double* d_w, const double* d_y, const double* d_zL,
                          const double* d_zU, const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0,
                          const double* d_wu0, const double* d_mu, const double* d_filt_t, const double* d_filt_p,
                          const int64_t* d_fcount,
                          uint8_t* d_active, int64_t* d_status, int64_t* d_acc, double* d_dinf, double* d_err0,
                          double* d_base, double* d_mu_o, double* d_ft, double* d_fp, int64_t* d_fc,
                          int32_t mu_rounds, double mu_min, const uint8_t* d_tiny_flag, const uint8_t* d_skip,
                          const IpmUnpack* unpack, void* stream);
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
// IPOPT's gradient-based NLP scaling (GradientScaling::DetermineScalingParametersImpl, with
// nlp_scaling_max_gradient 100 and nlp_scaling_min_value 1e-8; batch_ipm.py nlp_scaling,
// oracle/cpl_solve_host.c nlp_scaling), from the callbacks at the starting point: one wave per
// instance.  df = max(1e-8, 100 / max|grad f|) when that maximum exceeds 100; per block of rows (the
// equalities, the inequalities) whose largest row gradient exceeds 100, dc_r = max(1e-8,
// 100 * (1 / max(100, max_j |J_rj|))) on each row of the block.  Gradients over the free variables
// (srp / srq: the free-column records of each row), a NaN entry counting as 0.  any[0] = 1 when an
// instance has a factor != 1.  Also (always) the NaN entries of the instance's Jacobian there — the
// 0/0 of a cone at F_t = 0, which the iteration takes as 0 — into nan_cnt[b] (scale = 0: that only).
__global__ __launch_bounds__(256) void k_nlp_scaling(int64_t B, int n, int m, int nnz_rec, int scale,
                                                     const uint8_t* __restrict__ is_fixed,
                                                     const int32_t* __restrict__ row_slack, const int32_t* __restrict__ srp,
                                                     const int32_t* __restrict__ srq, const double* __restrict__ grad,
                                                     const double* __restrict__ J, double* __restrict__ df,
                                                     double* __restrict__ dc, uint8_t* __restrict__ any,
                                                     int32_t* __restrict__ nan_cnt) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  int nans = 0;
  for (int q = lane; q < nnz_rec; q += 64) nans += J[b * nnz_rec + q] != J[b * nnz_rec + q];
  nans = (int)wave_sum((double)nans);
  if (lane == 0) nan_cnt[b] = nans;
  if (!scale) return;
  double gm = 0.0;
  for (int j = lane; j < n; j += 64)
    if (!is_fixed[j]) {
      const double v = grad[b * n + j];
      gm = fmax(gm, v == v ? fabs(v) : 0.0);
    }
  gm = wave_max(gm);
  const double d = gm > 100.0 ? fmax(100.0 / gm, 1e-8) : 1.0;
  double rm[2] = {0.0, 0.0}, emax = 0.0, imax = 0.0;  // m <= 128: two rows per lane at most
  for (int h = 0; h < 2; ++h) {
    const int r = lane + 64 * h;
    if (r >= m) break;
    double v = 0.0;
    for (int t = srp[r]; t < srp[r + 1]; ++t) {
      const double a = J[b * nnz_rec + srq[t]];
      v = fmax(v, a == a ? fabs(a) : 0.0);
    }
    rm[h] = v;
    if (row_slack[r] < 0) emax = fmax(emax, v);
    else imax = fmax(imax, v);
  }
  emax = wave_max(emax);
  imax = wave_max(imax);
  bool scaled = d != 1.0;
  for (int h = 0; h < 2; ++h) {
    const int r = lane + 64 * h;
    if (r >= m) break;
    const double bm = row_slack[r] < 0 ? emax : imax;
    const double s = bm > 100.0 ? fmax(100.0 * (1.0 / fmax(rm[h], 100.0)), 1e-8) : 1.0;
    dc[b * m + r] = s;
    scaled |= s != 1.0;
  }
  if (lane == 0) df[b] = d;
  if (__ballot(scaled) != 0 && lane == 0) any[0] = 1;
}

// the scaled problem's callback values in place: f, grad f times df; g, J (records, row rrow[q])
// times dc (any output may be nullptr)
__global__ __launch_bounds__(256) void k_apply_scaling(int64_t B, int n, int m, int nnz_rec, const int32_t* __restrict__ rrow,
                                                       const double* __restrict__ df, const double* __restrict__ dc,
                                                       double* __restrict__ f, double* __restrict__ grad,
                                                       double* __restrict__ g, double* __restrict__ J) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const double d = df[b];
  if (f && lane == 0) f[b] = f[b] * d;
  if (grad)
    for (int j = lane; j < n; j += 64) grad[b * n + j] = grad[b * n + j] * d;
  if (g)
    for (int r = lane; r < m; r += 64) g[b * m + r] = g[b * m + r] * dc[b * m + r];
  if (J)
    for (int q = lane; q < nnz_rec; q += 64) J[b * nnz_rec + q] = J[b * nnz_rec + q] * dc[b * m + rrow[q]];
}

// the Hessian callbacks' multipliers (dc y) / df [B, m]
__global__ void k_scale_y(int64_t total, int m, const double* __restrict__ dc, const double* __restrict__ df,
                          const double* __restrict__ y, double* __restrict__ yt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < total) yt[e] = (dc[e] * y[e]) / df[e / m];
}

// v [B, per] times df[b] row by row
__global__ void k_scale_rows(int64_t total, int64_t per, const double* __restrict__ df, double* __restrict__ v) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < total) v[e] = v[e] * df[e / per];
}

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

// A = [J_free | -P] (cpl_ipm_dense_a's entries) and k_prep in one launch: the first nblk_a
// workgroups take A's entries, the rest k_prep's instances (independent outputs, no ordering)
__global__ __launch_bounds__(256) void k_dense_a_prep(int64_t totalA, unsigned nblk_a, int m, int nw, int nf, int nnz,
                                                      const int32_t* __restrict__ amap,
                                                      const int32_t* __restrict__ row_slack,
                                                      const double* __restrict__ jac, double* __restrict__ A,
                                                      const uint8_t* __restrict__ active, int64_t B, int n, const int32_t* __restrict__ free_idx,
                                                      const double* __restrict__ gl, const double* __restrict__ grad,
                                                      const double* __restrict__ g, const double* __restrict__ w,
                                                      double* __restrict__ gradw, double* __restrict__ c) {
  if (blockIdx.x < nblk_a) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < totalA) dense_a_entry(e, m, nw, nf, nnz, amap, row_slack, jac, A, active);
    return;
  }
  const int64_t b = (int64_t)(blockIdx.x - nblk_a) * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) gradw[b * nw + k] = k < nf ? grad[b * n + free_idx[k]] : 0.0;
  for (int r = lane; r < m; r += 64) c[b * m + r] = cons_row(g + b * m, w + b * nw, nf, r, row_slack, gl);
}

// after the optimality kernel: tau = max(0.99, 1 - mu), the iteration's active snapshot, and the
// evaluation point X = unpack(w) for the Hessian (the solve loop has it fused into the optimality
// kernel: IpmUnpack)
__global__ void k_unpack_tau(int64_t total, int n, int nw, const int32_t* __restrict__ freepos,
                             const double* __restrict__ Xbase, const double* __restrict__ w,
                             const double* __restrict__ mu, const uint8_t* __restrict__ active,
                             const uint8_t* __restrict__ in_resto, double* __restrict__ X, double* __restrict__ tau,
                             uint8_t* __restrict__ act) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int64_t b = e / n;
  const int j = (int)(e - b * n);
  const int k = freepos[j];
  X[e] = k >= 0 ? w[b * nw + k] : Xbase[e];
  if (j == 0) {
    tau[b] = fmax(1.0 - mu[b], 0.99);
    act[b] = active[b] && !in_resto[b];  // the restoration phase's instances take their own step
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

// ---- IPOPT constants of the line search / restoration phase (batch_ipm.py restates them) ------
// (the acceptance test itself: cpl_accept.hpp)
constexpr double GAMMA_TH = LS_GAMMA_TH, GAMMA_PHI = LS_GAMMA_PHI, DELTA_SW = LS_DELTA, S_TH = LS_S_TH, S_PHI = LS_S_PHI;
constexpr double KAPPA_SOC = 0.99, KAPPA_SIGMA = 1e10;
constexpr double RHO_R = 1000.0, KAPPA_RESTO = 0.9, BOUND_MULT_RESET = 1000.0, SOFT_RESTO_FACTOR = 0.9999;
constexpr int MAX_SOFT_RESTO = LS_MAX_SOFT_RESTO, MU_ROUNDS = 6;

__device__ __forceinline__ double wave_min_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}

// IPOPT FilterLSAcceptor::CalculateAlphaMin (cpl_accept.hpp)
__device__ __forceinline__ double alpha_min_of(double theta, double gd, double theta_min) {
  return ls_alpha_min_of(theta, gd, theta_min);
}

// IPOPT FilterLSAcceptor::CheckAcceptabilityOfTrialPoint on one wave: theta_max, the filter (entries
// stored with their margins), switching condition / Armijo / sufficient decrease against the
// reference point with the obj_max_inc guard.  Returns ok; *h_type = the step augments the filter.
__device__ __forceinline__ bool acceptable_wave(double th, double ph, double tk, double pk, double g, double al,
                                                uint8_t switch_ok, double theta_max, const double* ft, const double* fp,
                                                bool* h_type) {
  return ls_acceptable_wave(th, ph, tk, pk, g, al, switch_ok, theta_max, ft, fp, FMAX, h_type);
}

// (the line-search setup after the Newton step: cpl_accept.hpp ls_setup_wave, run by the post-step
// kernel)

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

// second-order correction bookkeeping (batch_ipm.py: soc, c_soc, a_soc, th_old = theta of the first
// trial point as IPOPT's TrySecondOrderCorrection) and the first correction's right-hand side
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
    th_old[b] = th[b];
  }
}

__global__ void k_soc_after(int64_t B, uint8_t* __restrict__ soc, const uint8_t* __restrict__ ok,
                            const double* __restrict__ th, double* __restrict__ th_old) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  soc[b] = soc[b] && !ok[b] && th[b] <= KAPPA_SOC * th_old[b];
  th_old[b] = th[b];
}

// after a trial: alpha halved where still searching, the search given up below alpha_min (IPOPT
// tries the next point only while alpha > alpha_min); flags (zeroed by ls_setup_wave / k_resto_post):
// any[fi] = an instance is still searching; with soft_now, any[1] = an instance has no accepted
// point yet and will try the soft restoration step
__global__ void k_halve2(int64_t B, uint8_t* __restrict__ searching, double* __restrict__ alpha,
                         const double* __restrict__ a_min, const uint8_t* __restrict__ act,
                         const uint8_t* __restrict__ tiny, const uint8_t* __restrict__ soft_now,
                         const int32_t* __restrict__ soft_cnt, const double* __restrict__ st_alpha,
                         uint8_t* __restrict__ any, int fi) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  bool s = searching[b] != 0;
  if (s) {
    const double a = 0.5 * alpha[b];
    alpha[b] = a;
    if (!(a > a_min[b])) s = false;
    searching[b] = s ? 1 : 0;
  }
  if (s) any[fi] = 1;
  if (soft_now && act[b] && !tiny[b] &&
      ((soft_now[b] && soft_cnt[b] <= MAX_SOFT_RESTO) || (!soft_now[b] && !(st_alpha[b] > 0.0))))
    any[1] = 1;
}

// IPOPT's soft restoration step, part 1 (BacktrackingLineSearch::TrySoftRestoStep): the instances
// without an accepted trial (or in the soft phase, at most max_soft_resto_iters times) try the full
// primal-dual step alpha = min(alpha_primal_max, alpha_dual_max): its point w + alpha dw and X
__global__ __launch_bounds__(256) void k_soft_begin(
    int64_t B, int n, int nf, int nw, const uint8_t* __restrict__ act, const uint8_t* __restrict__ tiny,
    const uint8_t* __restrict__ soft_now, const int32_t* __restrict__ soft_cnt, const double* __restrict__ st_alpha,
    const double* __restrict__ a_max, const double* __restrict__ a_z, const double* __restrict__ w,
    const double* __restrict__ dw, const int32_t* __restrict__ freepos, const double* __restrict__ Xbase,
    uint8_t* __restrict__ soft_try, double* __restrict__ a_soft, double* __restrict__ ws, double* __restrict__ X) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const bool t = act[b] && !tiny[b] &&
                 ((soft_now[b] && soft_cnt[b] <= MAX_SOFT_RESTO) || (!soft_now[b] && !(st_alpha[b] > 0.0)));
  const double as = fmin(a_max[b], a_z[b]);
  for (int k = lane; k < nw; k += 64) ws[b * nw + k] = w[b * nw + k] + (t ? as : 0.0) * dw[b * nw + k];
  for (int j = lane; j < n; j += 64) {
    const int k = freepos[j];
    X[b * n + j] = k >= 0 ? w[b * nw + k] + (t ? as : 0.0) * dw[b * nw + k] : Xbase[b * n + j];
  }
  if (lane == 0) {
    soft_try[b] = t ? 1 : 0;
    a_soft[b] = as;
  }
}

// IPOPT's primal-dual error of the barrier problem (1-norms of the dual residual, the constraint
// residual and the mu-complementarity) of one instance on one wave.  A row r, column k: from the
// dense A (Ad != NULL) or from the values-only Jacobian records through amap (as cpl_ipm_dense_a).
__device__ __forceinline__ double pd_error_wave(int m, int nf, int nw, const double* Ad, const double* Jrec,
                                                const int32_t* amap, const int32_t* row_slack, const double* gw_free,
                                                int gw_stride_n, const int32_t* free32, const double* c,
                                                const double* w, const double* y, const double* zL, const double* zU,
                                                const double* alpha_dy, const double* dy, const double* dzL,
                                                const double* dzU, double a, const uint8_t* hasL, const uint8_t* hasU,
                                                const double* wl0, const double* wu0, double mu) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int k = lane; k < nw; k += 64) {
    double dual = k < nf ? (gw_stride_n ? gw_free[free32[k]] : gw_free[k]) : 0.0;
    for (int r = 0; r < m; ++r) {
      double akr;
      if (Ad) {
        akr = Ad[r * nw + k];
      } else if (k < nf) {
        const int q = amap[r * nf + k];
        akr = q == -1 ? 0.0 : (q == -2 ? 1.0 : Jrec[q]);
        akr = akr == akr ? akr : 0.0;
      } else {
        akr = row_slack[r] == k - nf ? -1.0 : 0.0;
      }
      const double yr = dy ? y[r] + a * dy[r] : y[r];
      dual += akr * yr;
    }
    const double zl = hasL[k] ? (dzL ? zL[k] + a * dzL[k] : zL[k]) : 0.0;
    const double zu = hasU[k] ? (dzU ? zU[k] + a * dzU[k] : zU[k]) : 0.0;
    dual = dual - zl + zu;
    s += fabs(dual);
    if (hasL[k]) s += fabs((w[k] - wl0[k]) * zl - mu);
    if (hasU[k]) s += fabs((wu0[k] - w[k]) * zu - mu);
  }
  for (int r = lane; r < m; r += 64) s += fabs(c[r]);
  (void)alpha_dy;
  return wave_sum(s);
}

// part 2: the soft step is taken when the original filter / current iterate accept it (the soft
// phase ends) or when it cuts the primal-dual error by soft_resto_pderror_reduction_factor (the
// soft phase starts or continues); the step's alpha then also moves the bound multipliers
__device__ __forceinline__ void soft_judge_wave(
    int64_t b, int64_t B, int n, int m, int nf, int nw, int nnz_rec, const uint8_t* __restrict__ soft_try,
    const uint8_t* __restrict__ soft_now, const double* __restrict__ a_soft, const int32_t* __restrict__ amap,
    const int32_t* __restrict__ row_slack, const int32_t* __restrict__ free32, const double* __restrict__ gl,
    const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU, const double* __restrict__ wl0,
    const double* __restrict__ wu0, const double* __restrict__ ws, const double* __restrict__ f_s,
    const double* __restrict__ grad_s, const double* __restrict__ g_s, const double* __restrict__ J_s,
    const double* __restrict__ A, const double* __restrict__ gradw, const double* __restrict__ c,
    const double* __restrict__ w, const double* __restrict__ y, const double* __restrict__ zL,
    const double* __restrict__ zU, const double* __restrict__ dy, const double* __restrict__ dzL,
    const double* __restrict__ dzU, const double* __restrict__ mu, const double* __restrict__ theta_k,
    const double* __restrict__ phi_k, const double* __restrict__ gd, const uint8_t* __restrict__ switch_ok,
    const double* __restrict__ theta_max, const double* __restrict__ ft, const double* __restrict__ fp,
    double* __restrict__ cs_tmp, uint8_t* __restrict__ in_soft, int32_t* __restrict__ soft_cnt,
    double* __restrict__ st_f, double* __restrict__ st_g, double* __restrict__ st_w, double* __restrict__ st_alpha,
    uint8_t* __restrict__ st_aug, double* __restrict__ a_z) {
  const int lane = threadIdx.x & 63;
  const double* wb = ws + b * nw;
  const double mub = mu[b], as = a_soft[b];
  double th = 0.0, lg = 0.0;
  for (int r = lane; r < m; r += 64) {
    const double cr = cons_row(g_s + b * m, wb, nf, r, row_slack, gl);
    cs_tmp[b * m + r] = cr;
    th += fabs(cr);
  }
  for (int k = lane; k < nw; k += 64) {
    if (hasL[k]) lg += log(wb[k] - wl0[k]);
    if (hasU[k]) lg += log(wu0[k] - wb[k]);
  }
  th = wave_sum(th);
  lg = wave_sum(lg);
  const double ph = f_s[b] - mub * lg;
  const bool orig_ok = acceptable_wave(th, ph, theta_k[b], phi_k[b], gd[b], 0.0, switch_ok[b], theta_max[b],
                                       ft + b * FMAX, fp + b * FMAX, nullptr);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const double pd_t = pd_error_wave(m, nf, nw, nullptr, J_s + b * (int64_t)nnz_rec, amap, row_slack, grad_s + b * n, 1,
                                    free32, cs_tmp + b * m, wb, y + b * m, zL + b * nw, zU + b * nw, nullptr,
                                    dy + b * m, dzL + b * nw, dzU + b * nw, as, hasL, hasU, wl0, wu0, mub);
  const double pd_c = pd_error_wave(m, nf, nw, A + b * (int64_t)m * nw, nullptr, amap, row_slack, gradw + b * nw, 0,
                                    free32, c + b * m, w + b * nw, y + b * m, zL + b * nw, zU + b * nw, nullptr,
                                    nullptr, nullptr, nullptr, 0.0, hasL, hasU, wl0, wu0, mub);
  const bool ok = isfinite(th) && isfinite(ph) && (orig_ok || pd_t <= SOFT_RESTO_FACTOR * pd_c);
  if (ok) {
    for (int r = lane; r < m; r += 64) st_g[b * m + r] = g_s[b * m + r];
    for (int k = lane; k < nw; k += 64) st_w[b * nw + k] = wb[k];
  }
  if (lane == 0) {
    if (ok) {
      st_f[b] = f_s[b];
      st_alpha[b] = as;
      st_aug[b] = 0;
      a_z[b] = as;
    }
    const bool left = ok && orig_ok;
    if (left) in_soft[b] = 0;
    else if (ok) in_soft[b] = 1;
    if (left || (ok && !soft_now[b])) soft_cnt[b] = 0;
  }
}

__global__ __launch_bounds__(256) void k_soft_judge(
    int64_t B, int n, int m, int nf, int nw, int nnz_rec, const uint8_t* __restrict__ soft_try,
    const uint8_t* __restrict__ soft_now, const double* __restrict__ a_soft, const int32_t* __restrict__ amap,
    const int32_t* __restrict__ row_slack, const int32_t* __restrict__ free32, const double* __restrict__ gl,
    const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU, const double* __restrict__ wl0,
    const double* __restrict__ wu0, const double* __restrict__ ws, const double* __restrict__ f_s,
    const double* __restrict__ grad_s, const double* __restrict__ g_s, const double* __restrict__ J_s,
    const double* __restrict__ A, const double* __restrict__ gradw, const double* __restrict__ c,
    const double* __restrict__ w, const double* __restrict__ y, const double* __restrict__ zL,
    const double* __restrict__ zU, const double* __restrict__ dy, const double* __restrict__ dzL,
    const double* __restrict__ dzU, const double* __restrict__ mu, const double* __restrict__ theta_k,
    const double* __restrict__ phi_k, const double* __restrict__ gd, const uint8_t* __restrict__ switch_ok,
    const double* __restrict__ theta_max, const double* __restrict__ ft, const double* __restrict__ fp,
    double* __restrict__ cs_tmp, uint8_t* __restrict__ in_soft, int32_t* __restrict__ soft_cnt,
    double* __restrict__ st_f, double* __restrict__ st_g, double* __restrict__ st_w, double* __restrict__ st_alpha,
    uint8_t* __restrict__ st_aug, double* __restrict__ a_z) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B || !soft_try[b]) return;
  soft_judge_wave(b, B, n, m, nf, nw, nnz_rec, soft_try, soft_now, a_soft, amap, row_slack, free32, gl, hasL, hasU, wl0,
                  wu0, ws, f_s, grad_s, g_s, J_s, A, gradw, c, w, y, zL, zU, dy, dzL, dzU, mu, theta_k, phi_k, gd,
                  switch_ok, theta_max, ft, fp, cs_tmp, in_soft, soft_cnt, st_f, st_g, st_w, st_alpha, st_aug, a_z);
}

// the end of the regular line search: failed = no accepted point (-> the restoration phase),
// moved = an accepted one; a failed search leaves the soft phase.  IPOPT calls no restoration phase
// at an acceptable point (BacktrackingLineSearch: "Restoration phase called at acceptable point" ->
// STOP_AT_ACCEPTABLE_POINT): an instance whose search failed there ends with status acceptable.
// Nor at an almost feasible point (theta <= 1e-2 tol): the backup acceptable point is restored and
// the solve stops there as acceptable (RestoreAcceptablePoint), or without one it ends as a
// restoration failure ("Restoration phase called, but point is almost feasible").
struct NearFeasible {
  const double* theta_k;
  double near_tol;  // 1e-2 tol
  int nw, m;
  uint8_t* has_acc;
  const double *acc_w, *acc_y, *acc_zL, *acc_zU;
  double *w, *y, *zL, *zU;
};
// The bookkeeping of instance b:
__device__ __forceinline__ void fail_book(int64_t b, const uint8_t* __restrict__ act,
                                          const double* __restrict__ st_alpha, const double* __restrict__ err0,
                                          double acc_tol, uint8_t* __restrict__ failed, uint8_t* __restrict__ moved,
                                          uint8_t* __restrict__ in_soft, int32_t* __restrict__ soft_cnt,
                                          int64_t* __restrict__ status, uint8_t* __restrict__ active,
                                          const NearFeasible& nf) {
  const bool a = act[b] != 0;
  bool f = a && !(st_alpha[b] > 0.0);
  const bool at_acc = f && err0[b] <= acc_tol;
  const bool near = f && !at_acc && nf.theta_k[b] <= nf.near_tol;
  if (at_acc || near) {
    const bool back = near && nf.has_acc[b] != 0;
    if (back) {  // (a rare branch: one thread copies the instance's backup point)
      const int nw = nf.nw, m = nf.m;
      for (int k = 0; k < nw; ++k) {
        nf.w[b * nw + k] = nf.acc_w[b * nw + k];
        nf.zL[b * nw + k] = nf.acc_zL[b * nw + k];
        nf.zU[b * nw + k] = nf.acc_zU[b * nw + k];
      }
      for (int r = 0; r < m; ++r) nf.y[b * m + r] = nf.acc_y[b * m + r];
      nf.has_acc[b] = 0;
    }
    status[b] = (at_acc || back) ? CPL_SOLVE_ACCEPTABLE : CPL_SOLVE_RESTO_FAILED;
    active[b] = 0;
    failed[b] = 0;
    moved[b] = 0;
    return;
  }
  failed[b] = f ? 1 : 0;
  moved[b] = (a && !f) ? 1 : 0;
  if (f) {
    in_soft[b] = 0;
    soft_cnt[b] = 0;
  }
}

// ... in the same launch as the accepted points' X = unpack(st_w) (an element per thread; the first
// element of each instance also does that instance's bookkeeping — which does not touch st_w)
__global__ void k_fail_unpack(int64_t total, int n, int nw, const int32_t* __restrict__ freepos,
                              const double* __restrict__ Xbase, const double* __restrict__ st_w, double* __restrict__ X,
                              const uint8_t* __restrict__ act, const double* __restrict__ st_alpha,
                              const double* __restrict__ err0, double acc_tol, uint8_t* __restrict__ failed,
                              uint8_t* __restrict__ moved, uint8_t* __restrict__ in_soft, int32_t* __restrict__ soft_cnt,
                              int64_t* __restrict__ status, uint8_t* __restrict__ active, const NearFeasible nf) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int64_t b = e / n;
  const int j = (int)(e - b * n);
  const int k = freepos[j];
  X[e] = k >= 0 ? st_w[b * nw + k] : Xbase[e];
  if (j != 0) return;
  fail_book(b, act, st_alpha, err0, acc_tol, failed, moved, in_soft, soft_cnt, status, active, nf);
}

// The small-batch iteration (P_FUSED) runs the soft step's judge and the end of the search as one
// wave per instance: the judge (soft_try instances), then — its st_w / st_alpha / soft counters
// written by the same wave, made visible to the wave's other lanes by a workgroup fence — the
// accepted point's X = unpack(st_w) and the bookkeeping.  The same operations on the same values
// as k_soft_judge + k_fail_unpack.
struct FailTail {
  const int32_t* freepos;
  const double* Xbase;
  double* X;
  const uint8_t* act;
  const double* err0;
  double acc_tol;
  uint8_t* failed;
  uint8_t* moved;
  int64_t* status;
  uint8_t* active;
  NearFeasible nf;
};
__global__ __launch_bounds__(256) void k_soft_judge_fail(
    int64_t B, int n, int m, int nf, int nw, int nnz_rec, const uint8_t* __restrict__ soft_try,
    const uint8_t* __restrict__ soft_now, const double* __restrict__ a_soft, const int32_t* __restrict__ amap,
    const int32_t* __restrict__ row_slack, const int32_t* __restrict__ free32, const double* __restrict__ gl,
    const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU, const double* __restrict__ wl0,
    const double* __restrict__ wu0, const double* __restrict__ ws, const double* __restrict__ f_s,
    const double* __restrict__ grad_s, const double* __restrict__ g_s, const double* __restrict__ J_s,
    const double* __restrict__ A, const double* __restrict__ gradw, const double* __restrict__ c,
    const double* __restrict__ w, const double* __restrict__ y, const double* __restrict__ zL,
    const double* __restrict__ zU, const double* __restrict__ dy, const double* __restrict__ dzL,
    const double* __restrict__ dzU, const double* __restrict__ mu, const double* __restrict__ theta_k,
    const double* __restrict__ phi_k, const double* __restrict__ gd, const uint8_t* __restrict__ switch_ok,
    const double* __restrict__ theta_max, const double* __restrict__ ft, const double* __restrict__ fp,
    double* __restrict__ cs_tmp, uint8_t* __restrict__ in_soft, int32_t* __restrict__ soft_cnt,
    double* __restrict__ st_f, double* __restrict__ st_g, double* __restrict__ st_w, double* __restrict__ st_alpha,
    uint8_t* __restrict__ st_aug, double* __restrict__ a_z, const FailTail ft2) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  if (soft_try[b])
    soft_judge_wave(b, B, n, m, nf, nw, nnz_rec, soft_try, soft_now, a_soft, amap, row_slack, free32, gl, hasL, hasU,
                    wl0, wu0, ws, f_s, grad_s, g_s, J_s, A, gradw, c, w, y, zL, zU, dy, dzL, dzU, mu, theta_k, phi_k,
                    gd, switch_ok, theta_max, ft, fp, cs_tmp, in_soft, soft_cnt, st_f, st_g, st_w, st_alpha, st_aug,
                    a_z);
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  const int lane = threadIdx.x & 63;
  for (int j = lane; j < n; j += 64) {
    const int k = ft2.freepos[j];
    ft2.X[b * n + j] = k >= 0 ? st_w[b * nw + k] : ft2.Xbase[b * n + j];
  }
  if (lane == 0)
    fail_book(b, ft2.act, st_alpha, ft2.err0, ft2.acc_tol, ft2.failed, ft2.moved, in_soft, soft_cnt, ft2.status,
              ft2.active, ft2.nf);
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
// NFX: the LDS row length of the pair vectors (64 for nf <= 64 — the 4-contact problem's 39 — else 128):
// 28.5 -> 15.5 KiB of LDS per workgroup, twice the resident workgroups per CU
template <int NFX>
__global__ __launch_bounds__(256) void k_lbfgs(int64_t B, int m, int nf, int nw, int nnz_rec,
                                               const int32_t* __restrict__ amap, const uint8_t* __restrict__ act,
                                               const double* __restrict__ w_old, const double* __restrict__ w_new,
                                               const double* __restrict__ y, const double* __restrict__ dy,
                                               const double* __restrict__ alpha, const double* __restrict__ gw_old,
                                               const double* __restrict__ J_old, const double* __restrict__ grad_new,
                                               const int32_t* __restrict__ free_idx, int n,
                                               const double* __restrict__ J_new, double* __restrict__ lm_s,
                                               double* __restrict__ lm_y, uint8_t* __restrict__ lm_cnt,
                                               uint8_t* __restrict__ lm_skip, const uint8_t* __restrict__ failed,
                                               double* __restrict__ Hq) {
  const int64_t b = blockIdx.x;
  if (b >= B || !act[b]) return;
  __shared__ double Ps[LM_HIST][NFX], Py[LM_HIST][NFX], yn[256], red[8];
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
    __shared__ double pjn[4][NFX], pjo[4][NFX];
    const int kp = nf <= 64 ? 64 : 128, parts = (int)blockDim.x / kp;
    const int k = tid % kp, part = tid / kp;
    if (k < nf && part < parts) {
      const double* jnb = J_new + b * (int64_t)nnz_rec;
      const double* job = J_old + b * (int64_t)nnz_rec;
      double jn = 0.0, jo = 0.0;
      // rows r = part, part + parts, ... in order, eight at a time: the eight amap indices, then the
      // eight record entries they name, are loads in flight together (one row at a time waited two
      // dependent L2 round trips per row); the accumulation is the plain loop's
      const int R = m > part ? (m - part + parts - 1) / parts : 0;
      for (int t0 = 0; t0 < R; t0 += 8) {
        int qv[8];
        double anv[8], aov[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) qv[u] = t0 + u < R ? amap[(part + (t0 + u) * parts) * nf + k] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          anv[u] = qv[u] >= 0 ? jnb[qv[u]] : 1.0;
          aov[u] = qv[u] >= 0 ? job[qv[u]] : 1.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (qv[u] == -1) continue;  // structural zero (or past the last row): A's entry is 0
          double an = anv[u], ao = aov[u];
          if (qv[u] >= 0) {
            an = an == an ? an : 0.0;
            ao = ao == ao ? ao : 0.0;
          }
          const int r = part + (t0 + u) * parts;
          jn += an * yn[r];
          jo += ao * yn[r];
        }
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
      // grad_w f at the new point: its free components (k_prep's gather), 0 without a cost (grad_new NULL)
      const double gn = grad_new ? grad_new[b * n + free_idx[k2]] : 0.0;
      Py[last][k2] = (gn + jn) - (gw_old[b * nw + k2] + jo);
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
  __shared__ double Pa[LM_HIST][NFX], s_sa[LM_HIST], s_sy[LM_HIST];
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

// k_lbfgs for nf <= 64 with one wave per instance (four instances per workgroup) and the pair vectors
// in registers (lane k holds entry k of every stored pair): the same operations in the same order as
// k_lbfgs (the workgroup form, NFX = 64) — the J^T y row partials in its four row groups summed in its order, its block dots as
// 0 + the wave sum, its recursion — so bitwise the same model, without its barriers and idle waves
// (that form ran its recursion on one wave of four and kept 15.5 KiB of LDS per instance).
constexpr int LBW_WAVES = 4;
__global__ __launch_bounds__(64 * LBW_WAVES) void k_lbfgs_wave(
    int64_t B, int m, int nf, int nw, int nnz_rec, const int32_t* __restrict__ amap, const uint8_t* __restrict__ act,
    const double* __restrict__ w_old, const double* __restrict__ w_new, const double* __restrict__ y,
    const double* __restrict__ dy, const double* __restrict__ alpha, const double* __restrict__ gw_old,
    const double* __restrict__ J_old, const double* __restrict__ grad_new, const int32_t* __restrict__ free_idx, int n,
    const double* __restrict__ J_new, double* __restrict__ lm_s, double* __restrict__ lm_y, uint8_t* __restrict__ lm_cnt,
    uint8_t* __restrict__ lm_skip, const uint8_t* __restrict__ failed, double* __restrict__ Hq) {
  extern __shared__ double ynw[];  // [LBW_WAVES][m]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * LBW_WAVES + wv;
  if (b >= B || !act[b]) return;
  double* yn = ynw + (size_t)wv * m;
  const double al = alpha[b];
  for (int r = lane; r < m; r += 64) yn[r] = y[b * m + r] + al * dy[b * m + r];
  const int cnt = lm_cnt[b], skipped = lm_skip[b] + 1;
  __builtin_amdgcn_wave_barrier();
  const int shift = cnt == LM_HIST ? 1 : 0, last = cnt - shift;
  double* gs = lm_s + b * (int64_t)LM_HIST * nf;
  double* gy = lm_y + b * (int64_t)LM_HIST * nf;
  const int k = lane;
  const bool hk = k < nf;
  double Ps[LM_HIST], Py[LM_HIST];
  {  // J_free^T y at both points: the workgroup form's four row groups (rows part, part + 4, ...), each in its
     // eight-row batches, the group partials summed in order
    constexpr int PARTS = 4;
    const double* jnb = J_new + b * (int64_t)nnz_rec;
    const double* job = J_old + b * (int64_t)nnz_rec;
    double pn[PARTS], po[PARTS];
#pragma unroll
    for (int part = 0; part < PARTS; ++part) {
      double jn = 0.0, jo = 0.0;
      const int R = m > part ? (m - part + PARTS - 1) / PARTS : 0;
      if (hk) {
        for (int t0 = 0; t0 < R; t0 += 8) {
          int qv[8];
          double anv[8], aov[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) qv[u] = t0 + u < R ? amap[(part + (t0 + u) * PARTS) * nf + k] : -1;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            anv[u] = qv[u] >= 0 ? jnb[qv[u]] : 1.0;
            aov[u] = qv[u] >= 0 ? job[qv[u]] : 1.0;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (qv[u] == -1) continue;
            double an = anv[u], ao = aov[u];
            if (qv[u] >= 0) {
              an = an == an ? an : 0.0;
              ao = ao == ao ? ao : 0.0;
            }
            const int r = part + (t0 + u) * PARTS;
            jn += an * yn[r];
            jo += ao * yn[r];
          }
        }
      }
      pn[part] = jn;
      po[part] = jo;
    }
    double jn = pn[0], jo = po[0];
#pragma unroll
    for (int q = 1; q < PARTS; ++q) {
      jn += pn[q];
      jo += po[q];
    }
#pragma unroll
    for (int j = 0; j < LM_HIST; ++j) {
      Ps[j] = 0.0;
      Py[j] = 0.0;
      if (hk && j < last) {
        Ps[j] = gs[(j + shift) * nf + k];
        Py[j] = gy[(j + shift) * nf + k];
      }
    }
    if (hk) {
      const double sl = w_new[b * nw + k] - w_old[b * nw + k];
      const double gn = grad_new ? grad_new[b * n + free_idx[k]] : 0.0;
      const double yl = (gn + jn) - (gw_old[b * nw + k] + jo);
#pragma unroll
      for (int j = 0; j < LM_HIST; ++j)
        if (j == last) {
          Ps[j] = sl;
          Py[j] = yl;
        }
    }
  }
  // the newest pair (slot `last`, wave-uniform) and the three dots as the workgroup form's block_dot: 0 + the
  // wave sum of the lanes' products (lanes >= nf contribute 0)
  double sL = 0.0, yL = 0.0;
#pragma unroll
  for (int j = 0; j < LM_HIST; ++j)
    if (j == last) {
      sL = Ps[j];
      yL = Py[j];
    }
  auto wdot = [&](double a, double c) {
    double v = 0.0;
    if (hk) v += a * c;
    return 0.0 + wave_sum(v);
  };
  const double sy = wdot(sL, yL);
  const double ss = wdot(sL, sL);
  const double yy = wdot(yL, yL);
  double* hc = Hq + b * (int64_t)LMC(nf);
  const bool skip = !(sy > sqrt(DBL_EPSILON) * sqrt(ss) * sqrt(yy));
  if (skip || failed[b]) {
    if (!failed[b] && skipped <= LM_MAX_SKIP) {
      if (lane == 0) lm_skip[b] = (uint8_t)skipped;
      return;
    }
    if (lane == 0) {
      hc[0] = 1.0;
      hc[1] = 0.0;
      lm_skip[b] = 0;
      lm_cnt[b] = 0;
    }
    return;
  }
  const int nc = last + 1;
  if (hk) {
#pragma unroll
    for (int j = 0; j < LM_HIST; ++j)
      if (j < nc) {
        gs[j * nf + k] = Ps[j];
        gy[j * nf + k] = Py[j];
      }
  }
  if (lane == 0) {
    lm_skip[b] = 0;
    lm_cnt[b] = (uint8_t)nc;
  }
  const double sigma = fmin(fmax(sy / ss, 1e-8), 1e8);
  // the recursion (the workgroup form's, lane k0 = k; its second entry k1 = k + 64 >= nf contributes zeros)
  double Pa[LM_HIST], s_sa[LM_HIST], s_sy[LM_HIST];
#pragma unroll
  for (int j = 0; j < LM_HIST; ++j) {
    Pa[j] = 0.0;
    s_sa[j] = 0.0;
    s_sy[j] = 0.0;
  }
#pragma unroll
  for (int j = 0; j < LM_HIST; ++j) {
    if (j >= nc) break;
    const double s0 = hk ? Ps[j] : 0.0, s1 = 0.0;
    double v0 = sigma * s0, v1 = sigma * s1;
#pragma unroll
    for (int i = 0; i < j; ++i) {
      if (!(s_sa[i] > 0.0)) continue;
      const double a0 = hk ? Pa[i] : 0.0, a1 = 0.0;
      const double y0 = hk ? Py[i] : 0.0, y1 = 0.0;
      const double as = wave_sum(a0 * s0 + a1 * s1) / s_sa[i];
      const double ys = wave_sum(y0 * s0 + y1 * s1) / s_sy[i];
      v0 = (v0 - a0 * as) + y0 * ys;
      v1 = (v1 - a1 * as) + y1 * ys;
    }
    if (hk) Pa[j] = v0;
    const double y0 = hk ? Py[j] : 0.0, y1 = 0.0;
    s_sa[j] = wave_sum(s0 * v0 + s1 * v1);
    s_sy[j] = wave_sum(s0 * y0 + s1 * y1);
  }
#pragma unroll
  for (int i = 0; i < LM_HIST; ++i) {
    if (i >= nc) break;
    if (!(s_sa[i] > 0.0)) continue;
    const double qa = sqrt(s_sa[i]), qy = sqrt(s_sy[i]);
    if (hk) {
      Pa[i] /= qa;
      Py[i] /= qy;
    }
  }
  int pos = 0;
#pragma unroll
  for (int i = 0; i < LM_HIST; ++i) {
    if (i >= nc) break;
    if (!(s_sa[i] > 0.0)) continue;
    if (hk) {
      hc[2 + pos * nf + k] = Pa[i];
      hc[2 + LM_HIST * nf + pos * nf + k] = Py[i];
    }
    ++pos;
  }
  if (lane == 0) {
    hc[0] = sigma;
    hc[1] = (double)pos;
  }
}

// ---- the restoration phase (IPOPT MinC_1NrmRestorationPhase; batch_ipm.py enter_resto /
// resto_step / leave_resto restate these kernels) -------------------------------------------
// The restoration problem of an instance whose line search failed at w_R:
//   min rho sum(p + n) + eta/2 |D_R (x - x_R)|^2  s.t.  c(w) - p + n = 0,  w in its bounds, p, n >= 0,
// eta = sqrt(mu_R), D_R = diag(1 / max(1, |x_R|)) over x_free; solved by the same interior-point
// method (its own barrier parameter, filter and line search; p and n eliminated from the Newton
// system) until the original infeasibility falls to kappa_resto of its value at the start and the
// point is acceptable to the original filter and to the iterate where the phase began.

// The accepted point's rows [f | grad (n) | g (m) | J (nnz_rec)] into the iterate's (k_accept_rows),
// entry q of instance b; k_resto_enter does it for the instances that moved (moved != NULL) in its
// launch — one launch fewer per iteration.
struct AcceptRows {
  const uint8_t* moved;
  int n, m, nnz;
  const double *f_n, *grad_n, *g_n, *J_n;
  double *f, *grad, *g, *J;
};
__device__ __forceinline__ void accept_row_entry(const AcceptRows& a, int64_t b, int64_t q) {
  if (q == 0) { a.f[b] = a.f_n[b]; return; }
  q -= 1;
  if (q < a.n) { a.grad[b * a.n + q] = a.grad_n[b * a.n + q]; return; }
  q -= a.n;
  if (q < a.m) { a.g[b * a.m + q] = a.g_n[b * a.m + q]; return; }
  q -= a.m;
  a.J[b * a.nnz + q] = a.J_n[b * a.nnz + q];
}

// Entry (RestoIterateInitializer): x_R = w; mu_R = max(mu, |c|inf); p, n from the closed form of the
// barrier subproblem at fixed x (p - n = c, both positive); their bound multipliers mu_R / p,
// mu_R / n; the x-bound multipliers min(rho, z); the original filter augmented with the current
// point (PrepareRestoPhaseStart); an empty restoration filter; a fresh quasi-Newton model; and the
// least-squares system of the constraint multipliers (W = I, Sigma_p = Sigma_n = 1) for
// cpl_kkt_qd_solve: r1 = zLR - zUR, r2 = zp - zn, D^-1 = 1/2.
struct RestoEnterArgs {
  int m, nw;
  const uint8_t* failed;
  const double *c, *w, *zL, *zU, *mu, *theta_k, *phi_k;
  const uint8_t *hasL, *hasU;
  double *filt_t, *filt_p;
  int64_t *fcount, *iters;
  uint8_t* in_resto;
  int64_t* n_resto;
  double *wR, *pR, *nR, *zp, *zn, *zLR, *zUR, *muR, *ftR, *fpR;
  int64_t* fcR;
  double *thmaxR, *thminR, *th_o0, *ph_o0, *dwlR;
  uint8_t *lm_cnt, *lm_skip;
  double* Hq;
  int64_t lmc;
  double *Mw, *r1, *r2, *Dinv;
  AcceptRows ar;
  IpmAcceptArgs acc;
  bool with_accept;
};
// instance b's entry by one wave (lane = its lane)
__device__ __forceinline__ void resto_enter_one(const RestoEnterArgs& E, int64_t b, int lane) {
  const int m = E.m, nw = E.nw;
  const uint8_t* __restrict__ failed = E.failed;
  const double* __restrict__ c = E.c;
  const double* __restrict__ w = E.w;
  const double* __restrict__ zL = E.zL;
  const double* __restrict__ zU = E.zU;
  const double* __restrict__ mu = E.mu;
  const double* __restrict__ theta_k = E.theta_k;
  const double* __restrict__ phi_k = E.phi_k;
  const uint8_t* __restrict__ hasL = E.hasL;
  const uint8_t* __restrict__ hasU = E.hasU;
  double* __restrict__ filt_t = E.filt_t;
  double* __restrict__ filt_p = E.filt_p;
  int64_t* __restrict__ fcount = E.fcount;
  int64_t* __restrict__ iters = E.iters;
  uint8_t* __restrict__ in_resto = E.in_resto;
  int64_t* __restrict__ n_resto = E.n_resto;
  double* __restrict__ wR = E.wR;
  double* __restrict__ pR = E.pR;
  double* __restrict__ nR = E.nR;
  double* __restrict__ zp = E.zp;
  double* __restrict__ zn = E.zn;
  double* __restrict__ zLR = E.zLR;
  double* __restrict__ zUR = E.zUR;
  double* __restrict__ muR = E.muR;
  double* __restrict__ ftR = E.ftR;
  double* __restrict__ fpR = E.fpR;
  int64_t* __restrict__ fcR = E.fcR;
  double* __restrict__ thmaxR = E.thmaxR;
  double* __restrict__ thminR = E.thminR;
  double* __restrict__ th_o0 = E.th_o0;
  double* __restrict__ ph_o0 = E.ph_o0;
  double* __restrict__ dwlR = E.dwlR;
  uint8_t* __restrict__ lm_cnt = E.lm_cnt;
  uint8_t* __restrict__ lm_skip = E.lm_skip;
  double* __restrict__ Hq = E.Hq;
  const int64_t lmc = E.lmc;
  double* __restrict__ Mw = E.Mw;
  double* __restrict__ r1 = E.r1;
  double* __restrict__ r2 = E.r2;
  double* __restrict__ Dinv = E.Dinv;
  const AcceptRows& ar = E.ar;
  if (E.with_accept) {  // (cpl_ipm_accept for this instance first, in the same launch)
    ipm_accept_one(E.acc, b, lane);
    __threadfence_block();  // its filter / count stores before the entry's loads of them
  }
  if (ar.moved && ar.moved[b]) {  // (k_accept_rows for the instances that moved, in the same launch)
    const int64_t L = 1 + ar.n + ar.m + ar.nnz;
    for (int64_t q = lane; q < L; q += 64) accept_row_entry(ar, b, q);
    return;
  }
  if (!failed[b]) return;
  const double mub = mu[b];
  double cinf = 0.0;
  for (int r = lane; r < m; r += 64) cinf = fmax(cinf, fabs(c[b * m + r]));
  cinf = wave_max(cinf);
  const double mr = fmax(mub, cinf);
  double th = 0.0;
  for (int r = lane; r < m; r += 64) {
    const double cr = c[b * m + r];
    const double a = (mr - RHO_R * cr) / (2.0 * RHO_R);
    const double nv = a + sqrt(a * a + mr * cr / (2.0 * RHO_R));
    const double pv = cr + nv;
    pR[b * m + r] = pv;
    nR[b * m + r] = nv;
    zp[b * m + r] = mr / pv;
    zn[b * m + r] = mr / nv;
    th += fabs(cr - pv + nv);
    r2[b * m + r] = mr / pv - mr / nv;
    Dinv[b * m + r] = 0.5;
  }
  th = wave_sum(th);
  for (int k = lane; k < nw; k += 64) {
    wR[b * nw + k] = w[b * nw + k];
    const double zl = hasL[k] ? fmin(zL[b * nw + k], RHO_R) : 0.0;
    const double zu = hasU[k] ? fmin(zU[b * nw + k], RHO_R) : 0.0;
    zLR[b * nw + k] = zl;
    zUR[b * nw + k] = zu;
    r1[b * nw + k] = zl - zu;
    for (int j = 0; j < nw; ++j) Mw[(b * nw + k) * nw + j] = j == k ? 1.0 : 0.0;
  }
  for (int k = lane; k < FMAX; k += 64) {
    ftR[b * FMAX + k] = INFINITY;
    fpR[b * FMAX + k] = INFINITY;
  }
  // the original filter augmented with the point where the phase begins
  const int64_t fc = fcount[b];
  const int slot = (int)(fc % FMAX);
  const double tk = theta_k[b], pk = phi_k[b];
  if (lane == 0) {
    filt_t[b * FMAX + slot] = (1.0 - GAMMA_TH) * tk;
    filt_p[b * FMAX + slot] = pk - GAMMA_PHI * tk;
    fcount[b] = fc + 1;
    iters[b] += 1;
    in_resto[b] = 1;
    n_resto[b] += 1;
    muR[b] = mr;
    fcR[b] = 0;
    thmaxR[b] = 1e4 * fmax(th, 1.0);
    thminR[b] = 1e-4 * fmax(th, 1.0);
    th_o0[b] = tk;
    ph_o0[b] = pk;
    dwlR[b] = 0.0;
    lm_cnt[b] = 0;
    lm_skip[b] = 0;
    if (Hq) {  // (limited-memory mode only)
      Hq[b * lmc] = 1.0;
      Hq[b * lmc + 1] = 0.0;
    }
  }
}
__global__ __launch_bounds__(256) void k_resto_enter(int64_t B, const RestoEnterArgs E) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  resto_enter_one(E, b, threadIdx.x & 63);
}

// the least-squares estimate kept when |y|max <= constr_mult_init_max = 1e3
__global__ __launch_bounds__(256) void k_resto_y0(int64_t B, int m, const uint8_t* __restrict__ failed,
                                                  const double* __restrict__ dy, double* __restrict__ y) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B || !failed[b]) return;
  const int lane = threadIdx.x & 63;
  double mx = 0.0;
  for (int r = lane; r < m; r += 64) mx = fmax(mx, fabs(dy[b * m + r]));
  mx = wave_max(mx);
  for (int r = lane; r < m; r += 64) y[b * m + r] = mx <= 1e3 ? dy[b * m + r] : 0.0;
}

// the restoration problem's optimality error, its monotone barrier update (resetting its filter) and
// the proximity term's gradient over w.  The restoration problem converged (IPOPT's
// RestoConvergenceCheck): a point of local infeasibility when the original problem's max |c| exceeds
// 1e2 tol; otherwise the point is feasible but unacceptable to the original filter — the first time the
// restoration tolerance is tightened to 1e-2 tol and the phase goes on (resto_tight), the second time
// the solve ends as a restoration failure (IPOPT's RESTORATION_CONVERGED_TO_FEASIBLE_POINT)
__global__ __launch_bounds__(256) void k_resto_prep1(
    int64_t B, int m, int nf, int nw, int nbounds, double tol, double mu_min, uint8_t* __restrict__ active,
    const uint8_t* __restrict__ in_resto, uint8_t* __restrict__ resto_tight, uint8_t* __restrict__ actR,
    int64_t* __restrict__ status,
    const double* __restrict__ A, const double* __restrict__ c, const double* __restrict__ w,
    const double* __restrict__ y, const double* __restrict__ wR, const double* __restrict__ pR,
    const double* __restrict__ nR, const double* __restrict__ zp, const double* __restrict__ zn,
    const double* __restrict__ zLR, const double* __restrict__ zUR, const uint8_t* __restrict__ hasL,
    const uint8_t* __restrict__ hasU, const double* __restrict__ wl0, const double* __restrict__ wu0,
    double* __restrict__ muR, double* __restrict__ ftR, double* __restrict__ fpR, int64_t* __restrict__ fcR,
    double* __restrict__ tauR, double* __restrict__ gfR) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const bool a = active[b] && in_resto[b];
  if (!a) {
    if (lane == 0) actR[b] = 0;
    return;
  }
  const double* Ab = A + b * (int64_t)m * nw;
  double mu = muR[b];
  double eta = sqrt(mu);
  double dmax = 0.0, zs = 0.0, cmax = 0.0, ys = 0.0, crmax = 0.0;
  double clv[2] = {0, 0}, cuv[2] = {0, 0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = lane + 64 * h;
    if (k < nw) {
      const double wk = w[b * nw + k];
      const double dr = k < nf ? 1.0 / fmax(fabs(wR[b * nw + k]), 1.0) : 0.0;
      double dual = k < nf ? eta * (dr * dr) * (wk - wR[b * nw + k]) : 0.0;
      dual = seq_dot_acc(dual, Ab + k, nw, y + b * m, m);
      const double zl = zLR[b * nw + k], zu = zUR[b * nw + k];
      dual = dual - zl + zu;
      dmax = fmax(dmax, fabs(dual));
      zs += fabs(zl) + fabs(zu);
      clv[h] = hasL[k] ? (wk - wl0[k]) * zl : 0.0;
      cuv[h] = hasU[k] ? (wu0[k] - wk) * zu : 0.0;
      cmax = fmax(cmax, fmax(clv[h], cuv[h]));
    }
  }
  double cp[2] = {0, 0}, cn[2] = {0, 0}, cinf = 0.0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = lane + 64 * h;
    if (r < m) {
      const double yr = y[b * m + r], pv = pR[b * m + r], nv = nR[b * m + r], zpv = zp[b * m + r], znv = zn[b * m + r];
      dmax = fmax(dmax, fmax(fabs(RHO_R - yr - zpv), fabs(RHO_R + yr - znv)));
      zs += fabs(zpv) + fabs(znv);
      ys += fabs(yr);
      crmax = fmax(crmax, fabs(c[b * m + r] - pv + nv));
      cinf = fmax(cinf, fabs(c[b * m + r]));
      cp[h] = pv * zpv;
      cn[h] = nv * znv;
      cmax = fmax(cmax, fmax(cp[h], cn[h]));
    }
  }
  dmax = wave_max(dmax);
  cmax = wave_max(cmax);
  crmax = wave_max(crmax);
  zs = wave_sum(zs);
  ys = wave_sum(ys);
  const int nbR = nbounds + 2 * m;
  const double sd = fmax((ys + zs) / (double)max(m + nbR, 1), 100.0) / 100.0;
  const double sc = fmax(zs / (double)max(nbR, 1), 100.0) / 100.0;
  const double base = fmax(dmax / sd, crmax);
  const double err0 = fmax(base, cmax / sc);
  const bool tight = resto_tight[b] != 0;
  if (err0 <= (tight ? 1e-2 * tol : tol)) {  // the restoration problem converged
    cinf = wave_max(cinf);
    const bool feasible = cinf <= 1e2 * tol;
    if (!feasible || tight) {
      if (lane == 0) {
        status[b] = feasible ? CPL_SOLVE_RESTO_FAILED : CPL_SOLVE_INFEASIBLE;
        active[b] = 0;
        actR[b] = 0;
      }
      return;
    }
    if (lane == 0) resto_tight[b] = 1;  // once: the restoration tolerance 1e-2 tol, and on
  }
  bool reset = false;
  for (int round = 0; round < MU_ROUNDS; ++round) {
    double em = 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = lane + 64 * h;
      if (k < nw) {
        if (hasL[k]) em = fmax(em, fabs(clv[h] - mu));
        if (hasU[k]) em = fmax(em, fabs(cuv[h] - mu));
      }
      if (lane + 64 * h < m) em = fmax(em, fmax(fabs(cp[h] - mu), fabs(cn[h] - mu)));
    }
    em = wave_max(em);
    if (fmax(base, em / sc) <= 10.0 * mu && mu > mu_min) {
      mu = fmax(fmin(0.2 * mu, pow(mu, 1.5)), mu_min);
      reset = true;
    }
  }
  if (reset) {
    for (int k = lane; k < FMAX; k += 64) {
      ftR[b * FMAX + k] = INFINITY;
      fpR[b * FMAX + k] = INFINITY;
    }
  }
  eta = sqrt(mu);
  for (int k = lane; k < nw; k += 64) {
    const double dr = k < nf ? 1.0 / fmax(fabs(wR[b * nw + k]), 1.0) : 0.0;
    gfR[b * nw + k] = k < nf ? eta * (dr * dr) * (w[b * nw + k] - wR[b * nw + k]) : 0.0;
  }
  if (lane == 0) {
    actR[b] = 1;
    muR[b] = mu;
    tauR[b] = fmax(1.0 - mu, 0.99);
    if (reset) fcR[b] = 0;
  }
}

// a restoration phase that failed (k_resto_prep1: RESTO_FAILED) with a backup acceptable point: IPOPT
// restores that point and stops there as acceptable (BacktrackingLineSearch: RestoreAcceptablePoint,
// STOP_AT_ACCEPTABLE_POINT); batch_ipm.py resto_step restates it
__global__ __launch_bounds__(256) void k_restore_acc(int64_t B, int m, int nw, int64_t* __restrict__ status,
                                                     uint8_t* __restrict__ has_acc, const double* __restrict__ acc_w,
                                                     const double* __restrict__ acc_y, const double* __restrict__ acc_zL,
                                                     const double* __restrict__ acc_zU, double* __restrict__ w,
                                                     double* __restrict__ y, double* __restrict__ zL,
                                                     double* __restrict__ zU) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B || status[b] != CPL_SOLVE_RESTO_FAILED || !has_acc[b]) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) {
    w[b * nw + k] = acc_w[b * nw + k];
    zL[b * nw + k] = acc_zL[b * nw + k];
    zU[b * nw + k] = acc_zU[b * nw + k];
  }
  for (int r = lane; r < m; r += 64) y[b * m + r] = acc_y[b * m + r];
  __builtin_amdgcn_wave_barrier();  // (one wave per instance: its lanes read status / has_acc above)
  if (lane == 0) {
    status[b] = CPL_SOLVE_ACCEPTABLE;
    has_acc[b] = 0;
  }
}

// after the Newton setup (M = diag(Sigma_R) + H_c, r1 = -(grad phi_R,w + A^T y)): the proximity
// term's Hessian eta D_R^2 on M's diagonal, the eliminated p / n blocks (Sigma_p = zp / p,
// Sigma_n = zn / n, D^-1 = 1 / (1/Sigma_p + 1/Sigma_n), r2 = -(c - p + n) + r_p / Sigma_p - r_n / Sigma_n)
// and the restoration problem's theta and barrier objective phi_R
__global__ __launch_bounds__(256) void k_resto_prep2(
    int64_t B, int m, int nf, int nw, const uint8_t* __restrict__ actR, const double* __restrict__ c,
    const double* __restrict__ w, const double* __restrict__ y, const double* __restrict__ wR,
    const double* __restrict__ pR, const double* __restrict__ nR, const double* __restrict__ zp,
    const double* __restrict__ zn, const double* __restrict__ muR, const uint8_t* __restrict__ hasL,
    const uint8_t* __restrict__ hasU, const double* __restrict__ wl0, const double* __restrict__ wu0,
    double* __restrict__ M, double* __restrict__ rp, double* __restrict__ rn, double* __restrict__ Dinv,
    double* __restrict__ r2, double* __restrict__ thetaR, double* __restrict__ phiR) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B || !actR[b]) return;
  const int lane = threadIdx.x & 63;
  const double mu = muR[b], eta = sqrt(mu);
  double prox = 0.0, lg = 0.0, th = 0.0, pn = 0.0, lpn = 0.0;
  for (int k = lane; k < nw; k += 64) {
    const double wk = w[b * nw + k];
    if (k < nf) {
      const double dr = 1.0 / fmax(fabs(wR[b * nw + k]), 1.0);
      const double d2 = dr * dr;
      M[(b * nw + k) * nw + k] += eta * d2;
      const double dx = wk - wR[b * nw + k];
      prox += d2 * (dx * dx);
    }
    if (hasL[k]) lg += log(wk - wl0[k]);
    if (hasU[k]) lg += log(wu0[k] - wk);
  }
  for (int r = lane; r < m; r += 64) {
    const double pv = pR[b * m + r], nv = nR[b * m + r], yr = y[b * m + r];
    const double sp = zp[b * m + r] / pv, sn = zn[b * m + r] / nv;
    const double a = -((RHO_R - mu / pv) - yr), q = -((RHO_R - mu / nv) + yr);
    const double cr = c[b * m + r] - pv + nv;
    rp[b * m + r] = a;
    rn[b * m + r] = q;
    Dinv[b * m + r] = 1.0 / (1.0 / sp + 1.0 / sn);
    r2[b * m + r] = -cr + a / sp - q / sn;
    th += fabs(cr);
    pn += pv + nv;
    lpn += log(pv) + log(nv);
  }
  prox = wave_sum(prox);
  lg = wave_sum(lg);
  th = wave_sum(th);
  pn = wave_sum(pn);
  lpn = wave_sum(lpn);
  if (lane == 0) {
    thetaR[b] = th;
    phiR[b] = RHO_R * pn + 0.5 * eta * prox - mu * lg - mu * lpn;
  }
}

// after the restoration Newton step: dp, dn, the bound-multiplier steps, the fraction-to-the-boundary
// steps (primal over w, p, n; dual over zLR, zUR, zp, zn), gd = grad phi_R . (dw, dp, dn), the
// switching condition, alpha_min and the line search's state
__global__ __launch_bounds__(256) void k_resto_post(
    int64_t B, int m, int nw, const uint8_t* __restrict__ actR, const double* __restrict__ w,
    const double* __restrict__ dw, const double* __restrict__ dy, const double* __restrict__ gphi,
    const double* __restrict__ pR, const double* __restrict__ nR, const double* __restrict__ zp,
    const double* __restrict__ zn, const double* __restrict__ zLR, const double* __restrict__ zUR,
    const double* __restrict__ rp, const double* __restrict__ rn, const double* __restrict__ muR,
    const double* __restrict__ tauR, const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU,
    const double* __restrict__ wl0, const double* __restrict__ wu0, const double* __restrict__ thetaR,
    const double* __restrict__ thminR, const double* __restrict__ f, const double* __restrict__ g,
    double* __restrict__ dp, double* __restrict__ dn, double* __restrict__ dzL, double* __restrict__ dzU,
    double* __restrict__ dzp, double* __restrict__ dzn, double* __restrict__ a_max, double* __restrict__ a_z,
    double* __restrict__ gdR, uint8_t* __restrict__ switchR, double* __restrict__ a_min,
    uint8_t* __restrict__ searching, double* __restrict__ st_f, double* __restrict__ st_g, double* __restrict__ st_w,
    double* __restrict__ st_p, double* __restrict__ st_n, double* __restrict__ st_alpha, uint8_t* __restrict__ st_aug,
    double* __restrict__ alpha, uint8_t* __restrict__ any) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  if (b == 0 && lane == 0 && any) any[2] = 0;
  if (!actR[b]) return;
  const double mu = muR[b], t = tauR[b];
  double rpmax = INFINITY, rz = INFINITY, gd = 0.0;
  for (int k = lane; k < nw; k += 64) {
    const double wk = w[b * nw + k], dk = dw[b * nw + k];
    gd += gphi[b * nw + k] * dk;
    double dzl = 0.0, dzu = 0.0;
    if (hasL[k]) {
      const double dl = wk - wl0[k], zl = zLR[b * nw + k];
      dzl = mu / dl - zl - zl / dl * dk;
      if (dk < 0.0) rpmax = fmin(rpmax, -t * dl / dk);
      if (dzl < 0.0) rz = fmin(rz, -t * zl / dzl);
    }
    if (hasU[k]) {
      const double du = wu0[k] - wk, zu = zUR[b * nw + k];
      dzu = mu / du - zu + zu / du * dk;
      if (dk > 0.0) rpmax = fmin(rpmax, -t * du / -dk);
      if (dzu < 0.0) rz = fmin(rz, -t * zu / dzu);
    }
    dzL[b * nw + k] = dzl;
    dzU[b * nw + k] = dzu;
    st_w[b * nw + k] = wk;
  }
  for (int r = lane; r < m; r += 64) {
    const double pv = pR[b * m + r], nv = nR[b * m + r], zpv = zp[b * m + r], znv = zn[b * m + r];
    const double dyr = dy[b * m + r];
    const double sp = zpv / pv, sn = znv / nv;
    const double dpv = (rp[b * m + r] + dyr) / sp, dnv = (rn[b * m + r] - dyr) / sn;
    const double dzpv = mu / pv - zpv - zpv / pv * dpv, dznv = mu / nv - znv - znv / nv * dnv;
    dp[b * m + r] = dpv;
    dn[b * m + r] = dnv;
    dzp[b * m + r] = dzpv;
    dzn[b * m + r] = dznv;
    gd += (RHO_R - mu / pv) * dpv + (RHO_R - mu / nv) * dnv;
    if (dpv < 0.0) rpmax = fmin(rpmax, -t * pv / dpv);
    if (dnv < 0.0) rpmax = fmin(rpmax, -t * nv / dnv);
    if (dzpv < 0.0) rz = fmin(rz, -t * zpv / dzpv);
    if (dznv < 0.0) rz = fmin(rz, -t * znv / dznv);
    st_g[b * m + r] = g[b * m + r];
    st_p[b * m + r] = pv;
    st_n[b * m + r] = nv;
  }
  rpmax = wave_min_d(rpmax);
  rz = wave_min_d(rz);
  gd = wave_sum(gd);
  if (lane == 0) {
    const double am = fmin(rpmax, 1.0);
    a_max[b] = am;
    a_z[b] = fmin(rz, 1.0);
    gdR[b] = gd;
    const double th = thetaR[b];
    switchR[b] = ls_switch_flags(th, thminR[b], gd);
    a_min[b] = alpha_min_of(th, gd, thminR[b]);
    searching[b] = 1;
    st_f[b] = f[b];
    st_alpha[b] = 0.0;
    st_aug[b] = 0;
    alpha[b] = am;
  }
}

// the restoration line search's acceptance test at one trial point (p, n along with w) and the take
__global__ __launch_bounds__(256) void k_resto_judge(
    int64_t B, int m, int nf, int nw, const uint8_t* __restrict__ searching_in, const int32_t* __restrict__ row_slack,
    const double* __restrict__ gl, const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU,
    const double* __restrict__ wl0, const double* __restrict__ wu0, const double* __restrict__ wt,
    const double* __restrict__ f_t, const double* __restrict__ g_t, const double* __restrict__ alpha,
    const double* __restrict__ pR, const double* __restrict__ nR, const double* __restrict__ dp,
    const double* __restrict__ dn, const double* __restrict__ wR, const double* __restrict__ muR,
    const double* __restrict__ thetaR, const double* __restrict__ phiR, const double* __restrict__ gdR,
    const uint8_t* __restrict__ switchR, const double* __restrict__ thmaxR, const double* __restrict__ ftR,
    const double* __restrict__ fpR, uint8_t* __restrict__ searching, double* __restrict__ st_f,
    double* __restrict__ st_g, double* __restrict__ st_w, double* __restrict__ st_p, double* __restrict__ st_n,
    double* __restrict__ st_alpha, uint8_t* __restrict__ st_aug) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B || !searching_in[b]) return;
  const int lane = threadIdx.x & 63;
  const double al = alpha[b], mu = muR[b], eta = sqrt(mu);
  const double* wb = wt + b * nw;
  double th = 0.0, pn = 0.0, lpn = 0.0, prox = 0.0, lg = 0.0;
  for (int r = lane; r < m; r += 64) {
    const double pt = pR[b * m + r] + al * dp[b * m + r], nt = nR[b * m + r] + al * dn[b * m + r];
    th += fabs(cons_row(g_t + b * m, wb, nf, r, row_slack, gl) - pt + nt);
    pn += pt + nt;
    lpn += log(pt) + log(nt);
  }
  for (int k = lane; k < nw; k += 64) {
    if (k < nf) {
      const double dr = 1.0 / fmax(fabs(wR[b * nw + k]), 1.0);
      const double dx = wb[k] - wR[b * nw + k];
      prox += (dr * dr) * (dx * dx);
    }
    if (hasL[k]) lg += log(wb[k] - wl0[k]);
    if (hasU[k]) lg += log(wu0[k] - wb[k]);
  }
  th = wave_sum(th);
  pn = wave_sum(pn);
  lpn = wave_sum(lpn);
  prox = wave_sum(prox);
  lg = wave_sum(lg);
  const double ph = RHO_R * pn + 0.5 * eta * prox - mu * lg - mu * lpn;
  bool h = false;
  const bool ok = acceptable_wave(th, ph, thetaR[b], phiR[b], gdR[b], al, switchR[b], thmaxR[b], ftR + b * FMAX,
                                  fpR + b * FMAX, &h);
  if (!ok) return;
  for (int r = lane; r < m; r += 64) {
    st_g[b * m + r] = g_t[b * m + r];
    st_p[b * m + r] = pR[b * m + r] + al * dp[b * m + r];
    st_n[b * m + r] = nR[b * m + r] + al * dn[b * m + r];
  }
  for (int k = lane; k < nw; k += 64) st_w[b * nw + k] = wb[k];
  if (lane == 0) {
    st_f[b] = f_t[b];
    st_alpha[b] = al;
    st_aug[b] = h ? 1 : 0;
    searching[b] = 0;
  }
}

// the restoration iteration's acceptance: a failed line search ends the instance (restoration
// failed); otherwise y, the bound multipliers (kappa_Sigma safeguard at mu_R), p, n, w, the
// restoration filter; then the return test (RestoConvergenceCheck: the original theta at most
// kappa_resto of its value where the phase began, the point acceptable to the original filter and
// to that iterate) and the return (ComputeBoundMultiplierStep for the original bound multipliers, a
// reset to 1 when any exceeds 1000, y = 0, a fresh quasi-Newton model)
__global__ __launch_bounds__(256) void k_resto_accept(
    int64_t B, int m, int nf, int nw, const uint8_t* __restrict__ actR, uint8_t* __restrict__ movedR,
    uint8_t* __restrict__ active, int64_t* __restrict__ status, int64_t* __restrict__ iters,
    const double* __restrict__ st_alpha, const uint8_t* __restrict__ st_aug, const double* __restrict__ st_w,
    const double* __restrict__ st_p, const double* __restrict__ st_n, const double* __restrict__ dy,
    const double* __restrict__ dzL, const double* __restrict__ dzU, const double* __restrict__ dzp,
    const double* __restrict__ dzn, const double* __restrict__ a_z, const double* __restrict__ muR,
    const double* __restrict__ thetaR, const double* __restrict__ phiR, double* __restrict__ ftR,
    double* __restrict__ fpR, int64_t* __restrict__ fcR, double* __restrict__ w, double* __restrict__ y,
    double* __restrict__ pR, double* __restrict__ nR, double* __restrict__ zp, double* __restrict__ zn,
    double* __restrict__ zLR, double* __restrict__ zUR, const uint8_t* __restrict__ hasL,
    const uint8_t* __restrict__ hasU, const double* __restrict__ wl0, const double* __restrict__ wu0,
    const int32_t* __restrict__ row_slack, const double* __restrict__ gl, const double* __restrict__ f_n,
    const double* __restrict__ g_n, const double* __restrict__ mu, const double* __restrict__ filt_t,
    const double* __restrict__ filt_p, const double* __restrict__ th_o0, const double* __restrict__ ph_o0,
    const double* __restrict__ wR, double* __restrict__ zL, double* __restrict__ zU, uint8_t* __restrict__ in_resto,
    int64_t* __restrict__ acc, uint8_t* __restrict__ lm_cnt, uint8_t* __restrict__ lm_skip, double* __restrict__ Hq,
    int64_t lmc) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  if (!actR[b]) {
    if (lane == 0) movedR[b] = 0;
    return;
  }
  const double al = st_alpha[b];
  if (!(al > 0.0)) {
    // the restoration phase's line search failed: IPOPT's restoration phase for the restoration problem
    // (RestoRestorationPhase::PerformRestoration) — x (here w) and every multiplier stay, p and n take
    // the closed-form minimisers of the barrier subproblem at the current c(w) and mu_R (the
    // restoration phase's start, RestoIterateInitializer), and that is the next iterate.  (g_n = g(w):
    // the search state's point is the iterate when no trial was taken.)
    const double mur = muR[b];
    for (int r = lane; r < m; r += 64) {
      const double c = cons_row(g_n + b * m, st_w + b * nw, nf, r, row_slack, gl);
      const double a = (mur - RHO_R * c) / (2.0 * RHO_R);
      const double nn = a + sqrt(a * a + mur * c / (2.0 * RHO_R));
      nR[b * m + r] = nn;
      pR[b * m + r] = c + nn;
    }
    if (lane == 0) {
      movedR[b] = 0;
      iters[b] += 1;
    }
    return;
  }
  const double mur = muR[b], az = a_z[b];
  for (int r = lane; r < m; r += 64) {
    y[b * m + r] += al * dy[b * m + r];
    const double pn = st_p[b * m + r], nn = st_n[b * m + r];
    zp[b * m + r] = fmin(fmax(zp[b * m + r] + az * dzp[b * m + r], mur / (KAPPA_SIGMA * pn)), KAPPA_SIGMA * mur / pn);
    zn[b * m + r] = fmin(fmax(zn[b * m + r] + az * dzn[b * m + r], mur / (KAPPA_SIGMA * nn)), KAPPA_SIGMA * mur / nn);
    pR[b * m + r] = pn;
    nR[b * m + r] = nn;
  }
  for (int k = lane; k < nw; k += 64) {
    const double wn = st_w[b * nw + k];
    if (hasL[k]) {
      const double dl = wn - wl0[k];
      zLR[b * nw + k] = fmin(fmax(zLR[b * nw + k] + az * dzL[b * nw + k], mur / (KAPPA_SIGMA * dl)), KAPPA_SIGMA * mur / dl);
    }
    if (hasU[k]) {
      const double du = wu0[k] - wn;
      zUR[b * nw + k] = fmin(fmax(zUR[b * nw + k] + az * dzU[b * nw + k], mur / (KAPPA_SIGMA * du)), KAPPA_SIGMA * mur / du);
    }
    w[b * nw + k] = wn;
  }
  if (lane == 0) {
    movedR[b] = 1;
    iters[b] += 1;
    if (st_aug[b]) {
      const int64_t fc = fcR[b];
      const int slot = (int)(fc % FMAX);
      const double tk = thetaR[b], pk = phiR[b];
      ftR[b * FMAX + slot] = (1.0 - GAMMA_TH) * tk;
      fpR[b * FMAX + slot] = pk - GAMMA_PHI * tk;
      fcR[b] = fc + 1;
    }
  }
  // ---- back to the regular iteration?
  const double mub = mu[b];
  double th = 0.0, lg = 0.0;
  for (int r = lane; r < m; r += 64) th += fabs(cons_row(g_n + b * m, st_w + b * nw, nf, r, row_slack, gl));
  for (int k = lane; k < nw; k += 64) {
    const double wn = st_w[b * nw + k];
    if (hasL[k]) lg += log(wn - wl0[k]);
    if (hasU[k]) lg += log(wu0[k] - wn);
  }
  th = wave_sum(th);
  lg = wave_sum(lg);
  const double ph = f_n[b] - mub * lg;
  bool rejected = false;
  for (int k = lane; k < FMAX; k += 64) rejected |= !((th <= filt_t[b * FMAX + k]) || (ph <= filt_p[b * FMAX + k]));
  const bool in_filter = __ballot(rejected) == 0;
  const double t0 = th_o0[b];
  const double p0 = ph_o0[b];
  const bool vs_start = (th - (1.0 - GAMMA_TH) * t0 <= 10.0 * DBL_EPSILON * fabs(t0)) ||
                        ((ph - p0) - (-GAMMA_PHI * t0) <= 10.0 * DBL_EPSILON * fabs(p0));
  const bool back = isfinite(th) && isfinite(ph) && th <= KAPPA_RESTO * t0 && in_filter && vs_start;
  if (!back) return;
  const double tau = fmax(1.0 - mub, 0.99);
  double ad = INFINITY;
  double dzl[2] = {0, 0}, dzu[2] = {0, 0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = lane + 64 * h;
    if (k < nw) {
      const double wr = wR[b * nw + k], wn = st_w[b * nw + k];
      if (hasL[k]) {
        const double s0 = wr - wl0[k], s1 = wn - wl0[k], z = zL[b * nw + k];
        dzl[h] = (z * (s0 - s1) + mub) / s0 - z;
        if (dzl[h] < 0.0) ad = fmin(ad, -tau * z / dzl[h]);
      }
      if (hasU[k]) {
        const double s0 = wu0[k] - wr, s1 = wu0[k] - wn, z = zU[b * nw + k];
        dzu[h] = (z * (s0 - s1) + mub) / s0 - z;
        if (dzu[h] < 0.0) ad = fmin(ad, -tau * z / dzu[h]);
      }
    }
  }
  ad = fmin(wave_min_d(ad), 1.0);
  double zmax = -INFINITY, zl_n[2] = {0, 0}, zu_n[2] = {0, 0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = lane + 64 * h;
    if (k < nw) {
      zl_n[h] = hasL[k] ? zL[b * nw + k] + ad * dzl[h] : zL[b * nw + k];
      zu_n[h] = hasU[k] ? zU[b * nw + k] + ad * dzu[h] : zU[b * nw + k];
      zmax = fmax(zmax, fmax(zl_n[h], zu_n[h]));
    }
  }
  zmax = wave_max(zmax);
  const bool big = zmax > BOUND_MULT_RESET;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = lane + 64 * h;
    if (k < nw) {
      zL[b * nw + k] = (big && hasL[k]) ? 1.0 : zl_n[h];
      zU[b * nw + k] = (big && hasU[k]) ? 1.0 : zu_n[h];
    }
  }
  for (int r = lane; r < m; r += 64) y[b * m + r] = 0.0;
  if (lane == 0) {
    in_resto[b] = 0;
    acc[b] = 0;
    lm_cnt[b] = 0;
    lm_skip[b] = 0;
    if (Hq) {  // (limited-memory mode only)
      Hq[b * lmc] = 1.0;
      Hq[b * lmc + 1] = 0.0;
    }
  }
}

// the number of instances still active, and of those in the restoration phase, into two ints
// (read by the host after each iteration): up to COUNT1_MAX instances one workgroup counts them.
// With a mailbox (coherent pinned host memory: [count, resto, seq]) the two counts also go straight
// to the host, then the iteration's sequence number (count[2], incremented here) behind a
// system-scope fence: the host polls seq instead of a D2H copy + stream synchronisation (a blit
// kernel and two host wake-ups per iteration, ~35 us of a single solve's ~200 us iteration).
constexpr int64_t COUNT1_MAX = 65536;
constexpr int64_t TRACK_FUSE_ROWS = 64;  // batches up to this size track the best iterate inside k_count1
struct TrackBest {  // (small batches) k_track_best's work inside k_count1; best_w == NULL: none
  int nw;
  double vtol;
  const double *w, *f, *g, *gl, *gu;
  double *best_w, *best_f;
  const double* dc;  // (scaled solves) the row factors: the violation is the unscaled g's; else NULL
};
__device__ __forceinline__ double orig_violation_wave(int m, const double* __restrict__ gb,
                                                      const double* __restrict__ gl, const double* __restrict__ gu,
                                                      const double* __restrict__ dcb);
// k_track_best's work for instance b (one wave)
__device__ __forceinline__ void track_best_one(const TrackBest& tb, const uint8_t* __restrict__ active, int m,
                                               int64_t b, int lane) {
  if (!active[b]) return;
  const double v = orig_violation_wave(m, tb.g + b * m, tb.gl, tb.gu, tb.dc ? tb.dc + b * m : nullptr);
  const double fb = tb.f[b];
  if (!(v <= tb.vtol) || !(fb < tb.best_f[b])) return;
  for (int k = lane; k < tb.nw; k += 64) tb.best_w[b * tb.nw + k] = tb.w[b * tb.nw + k];
  if (lane == 0) tb.best_f[b] = fb;
}
// k_resto_y0's work for a failed instance b (one wave)
__device__ __forceinline__ void resto_y0_one(int m, const double* __restrict__ dy, double* __restrict__ y, int64_t b,
                                             int lane) {
  double mx = 0.0;
  for (int r = lane; r < m; r += 64) mx = fmax(mx, fabs(dy[b * m + r]));
  mx = wave_max(mx);
  for (int r = lane; r < m; r += 64) y[b * m + r] = mx <= 1e3 ? dy[b * m + r] : 0.0;
}
// the two counts into count[0..1] and, with a mailbox, to the host behind the sequence number
__device__ __forceinline__ void post_counts(int t, int tr, int32_t* __restrict__ count, int32_t* __restrict__ mail) {
  count[0] = t;
  count[1] = tr;
  if (mail) {
    const int32_t seq = count[2] + 1;
    count[2] = seq;
    volatile int32_t* mb = mail;
    mb[0] = t;
    mb[1] = tr;
    __threadfence_system();
    mb[2] = seq;
  }
}
// the counts by the NT threads of one workgroup into count[0..1], and the mailbox post
template <int NT>
__device__ __forceinline__ void count_post(int64_t B, const uint8_t* __restrict__ active,
                                           const uint8_t* __restrict__ in_resto, int32_t* __restrict__ count,
                                           int32_t* __restrict__ mail) {
  __shared__ int s_w[NT / 64], s_r[NT / 64];
  int c = 0, cr = 0;
  for (int64_t b = threadIdx.x; b < B; b += NT) {
    c += active[b] ? 1 : 0;
    cr += (active[b] && in_resto[b]) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    cr += __shfl_xor(cr, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s_w[threadIdx.x >> 6] = c;
    s_r[threadIdx.x >> 6] = cr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0, tr = 0;
    for (int q = 0; q < NT / 64; ++q) {
      t += s_w[q];
      tr += s_r[q];
    }
    post_counts(t, tr, count, mail);
  }
}
__global__ __launch_bounds__(1024) void k_count1(int64_t B, const uint8_t* __restrict__ active,
                                                 const uint8_t* __restrict__ in_resto, int32_t* __restrict__ count,
                                                 int32_t* __restrict__ mail, int m, const uint8_t* __restrict__ failed,
                                                 const double* __restrict__ dy, double* __restrict__ y,
                                                 const TrackBest tb) {
  const int lane = threadIdx.x & 63;
  if (tb.best_w)  // k_track_best's work, a wave per instance (the same operations)
    for (int64_t b = threadIdx.x >> 6; b < B; b += 16) track_best_one(tb, active, m, b, lane);
  if (failed)  // k_resto_y0's work, a wave per instance (no dependence on the counts below)
    for (int64_t b = threadIdx.x >> 6; b < B; b += 16)
      if (failed[b]) resto_y0_one(m, dy, y, b, lane);
  count_post<1024>(B, active, in_resto, count, mail);
}

// The small-batch iteration's tail (B <= FUSE_ROWS: a single-instance Solve(), every solve's
// compacted tail) in ONE launch instead of three (k_resto_enter, cpl_kkt_qd_kernel, k_count1: ~4.5
// us each at B = 1, latency only), one workgroup per instance: k_resto_enter's work (the accept,
// the accepted rows, the restoration entry) by its first wave; for an instance whose search failed
// the entry's least-squares multipliers by the workgroup (qd_solve_block, cpl_kkt_qd_kernel's
// solve) and k_resto_y0's estimate; k_count1's best-iterate tracking.  Per instance these are the
// three launches' operations in their order (bitwise the same state).  The last workgroup to arrive
// (a 64-bit arrival word at count + 4 that also carries the counts, reset by that workgroup for the
// next replay) posts the active / restoration counts: k_count1's counting.
constexpr int TAIL_THREADS = 256;
struct QdSolveArgs {
  int nw, m;
  const double *W, *A, *Dinv, *r1, *r2;
  double *dwl, *dw, *dy, *delta_w, *Kws;
};
__global__ __launch_bounds__(TAIL_THREADS) void k_tail_small(int64_t B, const RestoEnterArgs E, const QdSolveArgs Q,
                                                             const uint8_t* __restrict__ active,
                                                             const uint8_t* __restrict__ in_resto,
                                                             int32_t* __restrict__ count, int32_t* __restrict__ mail,
                                                             double* __restrict__ y, const TrackBest tb) {
  extern __shared__ __align__(16) double qd_lds[];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 64) resto_enter_one(E, b, lane);
  __syncthreads();  // (its global stores before the solve's and the tracking's loads of them)
  const bool fl = E.failed[b] != 0;
  if (fl) {
    qd_solve_block<TAIL_THREADS>(b, Q.nw, Q.m, Q.W, Q.A, Q.Dinv, Q.r1, Q.r2, Q.dwl, Q.dw, Q.dy, Q.delta_w, Q.Kws,
                                 qd_lds);
    __syncthreads();  // (dy)
  }
  if (tid < 64) {
    if (tb.best_w) track_best_one(tb, active, E.m, b, lane);
    if (fl) resto_y0_one(E.m, Q.dy, y, b, lane);
  }
  // the arrival: ONE 64-bit atomic carries the instance's counts and the arrival itself (bits 0-20
  // active, 21-41 in the restoration phase, 42- arrivals; B <= FUSE_ROWS), so the last workgroup
  // reads the totals from its return value — nothing else crosses workgroups, so no device-scope
  // fences (each an L2 write-back: with them this launch cost as much as the three it replaces)
  if (tid == 0) {
    const unsigned long long a = active[b] ? 1ull : 0ull;
    const unsigned long long r = (a && in_resto[b]) ? 1ull : 0ull;  // (in_resto[b]: this thread's own store)
    const unsigned long long mine = (1ull << 42) | (r << 21) | a;
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(count + 4);
    const unsigned long long tot = atomicAdd(acc, mine) + mine;
    if ((tot >> 42) == (unsigned long long)B) {
      atomicExch(acc, 0ull);  // (every workgroup has arrived: reset for the next launch)
      post_counts((int)(tot & 0x1fffffull), (int)((tot >> 21) & 0x1fffffull), count, mail);
    }
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
  if (threadIdx.x == 0 && blockIdx.x == 0) count[0] = count[1] = 0;
}
__global__ __launch_bounds__(256) void k_count(int64_t B, const uint8_t* __restrict__ active,
                                               const uint8_t* __restrict__ in_resto, int32_t* __restrict__ count) {
  __shared__ int s_cnt[2];
  if (threadIdx.x < 2) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int a = (b < B && active[b]) ? 1 : 0;
  const int r = (a && in_resto[b]) ? 1 : 0;
  const unsigned long long bal = __ballot(a), balr = __ballot(r);
  if ((threadIdx.x & 63) == 0) {
    if (bal) atomicAdd(&s_cnt[0], __popcll(bal));
    if (balr) atomicAdd(&s_cnt[1], __popcll(balr));
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_cnt[0]) atomicAdd(count, s_cnt[0]);
    if (s_cnt[1]) atomicAdd(count + 1, s_cnt[1]);
  }
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
                                                       const double* __restrict__ dc, const double* __restrict__ df,
                                                       const double* __restrict__ Xbase, const double* __restrict__ d_inf,
                                                       const int64_t* __restrict__ status, const int64_t* __restrict__ iters,
                                                       const int64_t* __restrict__ n_resto,
                                                       double* __restrict__ fw, double* __restrict__ fy,
                                                       double* __restrict__ fX, double* __restrict__ fdinf,
                                                       int64_t* __restrict__ fstatus, int64_t* __restrict__ fiters,
                                                       int64_t* __restrict__ fresto) {
  const int64_t r = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int32_t o = orig[r];
  if (o < 0 || (finished_only && active[r])) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) fw[(int64_t)o * nw + k] = w[r * nw + k];
  // the multipliers of the unscaled problem: (dc y) / df (nlp_scaling; dc = nullptr: unscaled)
  for (int k = lane; k < m; k += 64) fy[(int64_t)o * m + k] = dc ? (dc[r * m + k] * y[r * m + k]) / df[r] : y[r * m + k];
  for (int k = lane; k < n; k += 64) fX[(int64_t)o * n + k] = Xbase[r * n + k];
  if (lane == 0) {
    fdinf[o] = d_inf[r];
    fstatus[o] = status[r];
    fiters[o] = iters[r];
    fresto[o] = n_resto[r];
  }
}

// the restoration-phase instances whose trial was accepted in the current search
__global__ void k_moved_r(int64_t B, const uint8_t* __restrict__ actR, const double* __restrict__ st_alpha,
                          uint8_t* __restrict__ movedR) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) movedR[b] = actR[b] && st_alpha[b] > 0.0;
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

// max violation of the constraint values g_b [m] against their original bounds (NaN: infinite), on
// one wave.  dcb (scaled solves: the instance's row factors, else NULL): g_b holds the scaled problem's
// values dc g, so the original constraint's value is g_b / dc (the bounds, 0 or infinite, are the
// original ones either way) — fallback_viol_tol applies to the original constraints
__device__ __forceinline__ double orig_violation_wave(int m, const double* __restrict__ gb,
                                                      const double* __restrict__ gl, const double* __restrict__ gu,
                                                      const double* __restrict__ dcb) {
  double v = 0.0;
  for (int r = threadIdx.x & 63; r < m; r += 64) {
    const double gv = dcb ? gb[r] / dcb[r] : gb[r];
    v = fmax(v, fmax(fmax(gl[r] - gv, gv - gu[r]), 0.0));
    if (gv != gv) v = INFINITY;
  }
  return wave_max(v);
}

// The best iterate of every active instance: after each iteration's acceptance, the current point
// (w, f, g in sync) replaces the kept one when its original constraints hold to `vtol` and its
// objective is lower.  (Not IPOPT: a solve that ends without convergence at an infeasible iterate
// returns this one instead, k_fallback.)
__global__ __launch_bounds__(256) void k_track_best(int64_t B, int m, int nw, double vtol,
                                                    const uint8_t* __restrict__ active, const double* __restrict__ w,
                                                    const double* __restrict__ f, const double* __restrict__ g,
                                                    const double* __restrict__ gl, const double* __restrict__ gu,
                                                    double* __restrict__ best_w, double* __restrict__ best_f,
                                                    const double* __restrict__ dc) {
  const int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (b >= B || !active[b]) return;
  const double v = orig_violation_wave(m, g + b * m, gl, gu, dc ? dc + b * m : nullptr);
  const double fb = f[b];
  if (!(v <= vtol) || !(fb < best_f[b])) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) best_w[b * nw + k] = w[b * nw + k];
  if (lane == 0) best_f[b] = fb;
}

// Rows leaving the batch (finished ones, or every row at the end): an instance that stopped without
// converging (max_iter, local infeasibility, restoration failure) at an iterate violating its
// constraints by more than `vtol` returns its best feasible iterate (k_track_best) when it met one;
// fbest[orig] records it
__global__ __launch_bounds__(256) void k_fallback(int64_t rows, int m, int nw, double vtol, bool finished_only,
                                                  const int32_t* __restrict__ orig, const uint8_t* __restrict__ active,
                                                  const int64_t* __restrict__ status, const double* __restrict__ g,
                                                  const double* __restrict__ gl, const double* __restrict__ gu,
                                                  const double* __restrict__ best_w, const double* __restrict__ best_f,
                                                  double* __restrict__ w, uint8_t* __restrict__ fbest,
                                                  const double* __restrict__ dc) {
  const int64_t r = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int32_t o = orig[r];
  if (o < 0 || (finished_only && active[r]) || status[r] <= CPL_SOLVE_ACCEPTABLE) return;
  const double v = orig_violation_wave(m, g + r * m, gl, gu, dc ? dc + r * m : nullptr);
  if (v <= vtol || !(best_f[r] < INFINITY)) return;
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nw; k += 64) w[r * nw + k] = best_w[r * nw + k];
  if (lane == 0) fbest[o] = 1;
}

__global__ void k_fill(int64_t B, double v, double* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = v;
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
  cpl_problem_desc desc_R;  // the template with zero cost weights: y^T g's Hessian for the restoration phase
  cpl_solve_options opt;
  int64_t B = 0;
  int64_t Bcur = 0;  // rows in play: B, shrunk by active-set compaction
  int n = 0, m = 0, nnz = 0, nnz_rec = 0, nf = 0, nI = 0, nw = 0, nbounds = 0;
  bool analytic_H = false, bfgs = false, fd = false, fd_fused = true;
  bool ls_fusable = false;  // the one-wave KKT size: the fused line-search kernel can re-solve with its factors
  bool jreg = false;        // IPOPT's Jacobian regularisation (cpl_kkt_aug_kernel after every KKT call)
  double* ws_aug = nullptr; // its workspace
  double mu_min = 0.0;
  hipStream_t stream = nullptr;
  bool captured = false;  // an iteration graph exists
  std::map<int64_t, std::pair<hipGraph_t, hipGraphExec_t>> graphs;  // (size, inputs, phase) -> graph
  uint8_t* h_flag = nullptr;  // pinned: the device's 4 flag bytes
  cpl::Arena arena;
  const double* mass = nullptr;       // per solve
  const uint8_t* tag = nullptr;
  // problem constants (device)
  int32_t *free32, *ineq_row, *row_slack, *freepos, *amap, *col_ptr, *csc_k, *csc_row;
  int64_t *free64, *fixed64;
  uint8_t *is_fixed, *hasL, *hasU, *zeros_u8;
  double *xl, *xu, *gl, *gu, *wl0, *wu0, *zeros_w, *zeros_B;
  // state
  double *Xbase, *w, *y, *zL, *zU, *mu, *filt_t, *filt_p, *dwl, *f, *grad, *g, *J, *d_inf, *Hq, *lm_s, *lm_y, *theta_max,
      *theta_min;
  int64_t *status, *iters, *acc, *fcount, *n_resto;
  // d_any [4]: batch-wide "any instance" flags the host reads once per phase (h_flag):
  //   [0] an instance is still searching after its trials, [1] an instance needs the soft restoration
  //   step (both set by the search kernels, cpl_kernels.hip cpl_ls_backtrack_kernel / cpl_ipm_judge_take),
  //   [2] an instance is searching inside the restoration phase.  Who clears them, per iteration:
  //   * fused search with the post-step prologue (post_in_ls): block 0 of the OPTIMALITY kernel clears
  //     [0..1] (IpmUnpack.any) — several launches before the search kernel sets them.  Invariant: no
  //     launch between the two (Hessian / FD evaluation, Newton setup, KKT factorisation) reads or
  //     writes d_any; the search kernel's own prologue cannot clear them (its other blocks set them
  //     concurrently: setup.any = nullptr there);
  //   * fused search without the prologue: the post-step kernel's tail clears [0..1] (LsSetup.any);
  //   * step-by-step search: a memset of [0..1] before the first trial;
  //   * [2]: a memset before the restoration phase's search, or block 0 of k_resto_post.
  //   tests/test_gpu_solve_engine.py covers the fused paths on both sides of LS_GF_MIN (B 2047 / 2048).
  uint8_t *active, *lm_cnt, *lm_skip, *d_any, *in_soft, *tiny_last, *tiny_flag, *in_resto, *resto_tight;
  double *best_w, *best_f;  // the best iterate feasible to fallback_viol_tol (lowest f) and its f
  double *acc_w, *acc_y, *acc_zL, *acc_zU;  // IPOPT's backup acceptable point
  uint8_t* has_acc;
  uint8_t* fbest;           // [B] full-batch: the solve returned that iterate instead of its last one
  int32_t* soft_cnt;
  // restoration state
  double *wR, *pR, *nR, *zp, *zn, *zLR, *zUR, *muR, *ftR, *fpR, *th_o0, *ph_o0, *dwlR, *thmaxR, *thminR;
  int64_t* fcR;
  // iteration temporaries
  double *A, *gradw, *c, *err0, *base, *mu_o, *ft, *fp, *tau, *X, *H, *M, *Kqd, *r1, *r2, *gphi,
      *mr_diag, *theta_k, *phi_k, *dw, *dy, *delta_w, *delta_c, *dzL, *dzU, *a_max, *a_z, *gd, *ws, *a_min, *a_soft,
      *cs_tmp, *scr1, *scr2;
  int64_t* fc;
  int32_t* info;
  uint8_t *act, *switch_ok, *searching, *st_aug, *ok, *soc, *ok_s, *failed, *moved, *tiny_now, *soft_now, *soft_try;
  double *st_f, *st_g, *st_w, *st_alpha, *alpha, *th, *wt, *Xt, *f_t, *g_t;
  double *c_soc, *a_soc, *th_old, *r2s, *dws, *dys, *ws_, *Xs, *f_s, *g_s, *th_s;
  double *Xn, *f_n, *grad_n, *g_n, *J_n, *Xp, *hfd, *gL, *mass_fd, *jac_fd, *grad_fd;
  uint8_t* tag_fd;
  // restoration temporaries
  double *gfR, *tauR, *rp, *rn, *Dinv, *dp, *dn, *dzp, *dzn, *st_p, *st_n, *thetaR, *phiR, *gdR, *a_maxR, *a_zR,
      *a_minR, *alphaR;
  uint8_t *actR, *movedR, *searchingR, *switchR;
  double *fin_f, *fin_g;
  int32_t *st32, *it32;
  // compaction: original instance of each row, compacted masses / tags, full-batch results
  int32_t *orig, *pos, *d_count, *h_count = nullptr;
  bool tail_fused = false;  // P_FUSED: the soft judge launch also ends the search (k_soft_judge_fail)
  bool soft_fused = false;  // P_FUSED(_R): the search kernel starts the soft step (no k_soft_begin)
  bool soft_begun = false;  // ... and the Newton phase's search kernel did (P_SOFT skips k_soft_begin)
  double *mass_c, *fw, *fy, *fX, *fdinf;
  uint8_t* tag_c;
  int64_t *fstatus, *fiters, *fresto;
  uint64_t* scratch;
  int64_t scratch_words = 0;
  int32_t compactions = 0;
  // IPOPT's gradient-based NLP scaling (cpl_solve_options.nlp_scaling): df [B], dc [B, m] (rows
  // compacted with the batch), the Hessian callbacks' multipliers (dc y) / df [B, m]; the records' row
  // [nnz_rec]; the free-column records of every row (CSR: srp [m + 1], srq); scaled: this solve has a
  // factor != 1 (the scaling kernels run; graphs keyed by it)
  double *df, *dc, *ytil;
  int32_t *rrow, *srp, *srq;
  int32_t* nan_cnt;  // [B] full batch: NaN Jacobian entries at each instance's start point
  uint8_t* sc_any;
  bool scaled = false;
  bool sc_fused = true;  // the evaluations apply the scaling themselves (until a path says unsupported)
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

// the scaled problem's values (IPOPT's scaled NLP): df f, df grad f, dc g, dc J (one product each)
int32_t apply_scaling(cpl_solver* S, double* fo, double* grado, double* go, double* jo) {
  if (!S->scaled) return CPL_OK;
  hipLaunchKernelGGL(k_apply_scaling, dim3(blocks_for(S->Bcur)), dim3(256), 0, S->stream, S->Bcur, S->n, S->m,
                     S->nnz_rec, S->rrow, S->df, S->dc, fo, grado, go, jo);
  LAUNCHED("k_apply_scaling");
  return CPL_OK;
}
// (scaled: the pipelined evaluation applies the factors in its tile image — one launch fewer per
// evaluation; other paths evaluate, then k_apply_scaling)
int32_t eval_fg(cpl_solver* S, const double* X, double* fo, double* go) {
  if (S->scaled && S->sc_fused) {
    const int32_t rc = eval_batch_scaled(&S->desc, S->Bcur, X, S->mass, S->tag, go, nullptr, fo, nullptr, 0, S->df,
                                         S->dc, S->rrow, S->stream);
    if (rc != CPL_ERR_UNSUPPORTED) return rc;
    S->sc_fused = false;
  }
  CK(cpl_eval_batch(&S->desc, S->Bcur, X, S->mass, S->tag, go, nullptr, fo, nullptr, S->stream));
  return apply_scaling(S, fo, nullptr, go, nullptr);
}
// gate (device byte, or nullptr): the evaluation is skipped where the pipelined kernel runs it and the
// byte is 0 — the outputs are then left as they were, and so are they scaled again (callers gate only
// an evaluation whose outputs nobody reads when the byte is 0)
int32_t eval_full(cpl_solver* S, const double* X, double* fo, double* grado, double* go, double* jo,
                  const uint8_t* gate = nullptr) {
  if (S->scaled && S->sc_fused) {
    const int32_t rc = eval_batch_scaled(&S->desc, S->Bcur, X, S->mass, S->tag, go, jo, fo, grado,
                                         CPL_EVAL_JAC_FOLDED, S->df, S->dc, S->rrow, S->stream, gate);
    if (rc != CPL_ERR_UNSUPPORTED) return rc;
    S->sc_fused = false;
  }
  CK(eval_batch_gated(&S->desc, S->Bcur, X, S->mass, S->tag, go, jo, fo, grado, CPL_EVAL_JAC_FOLDED, S->stream, gate));
  return apply_scaling(S, fo, grado, go, jo);
}

// The phases of one lock-step iteration (each graph-capturable, no host synchronisation inside):
//   P_NEWTON    the convergence test, barrier update, Newton step, tiny-step test, the first trial
//               with its second-order corrections, then the rest of every instance's backtracking
//               search in one kernel (cpl_kernels.hip ls_backtrack); flags: any instance with no
//               accepted trial (a soft-restoration candidate) / still searching
//   P_SOFT      IPOPT's soft restoration step (launched when a flag was raised)
//   P_RNEWTON   one restoration-phase iteration of the instances inside it: Newton step, first trial,
//               the rest of the search in one kernel, the acceptance and the return test (P_RACCEPT)
//   P_ACCEPT    the accepted points' evaluation, L-BFGS, the state update, the restoration phase's
//               entry for failed searches, the active / restoration counts; P_ACCEPT_NR the same
//               without the entry (no flag raised: no instance can have failed)
// Per iteration: P_NEWTON, [P_SOFT], [P_RNEWTON], P_ACCEPT | P_ACCEPT_NR; the host reads the flag
// bytes after P_NEWTON and the two counts after the accept.  Small batches (at most FUSE_ROWS rows,
// where every launch is latency and a host round trip costs as much as several kernels) run the
// whole iteration as one graph instead, P_FUSED = P_NEWTON + P_SOFT + P_ACCEPT (P_FUSED_R with the
// restoration iteration as well): the soft step's kernels and the restoration entry's run masked
// whether or not an instance needs them, and the host reads only the counts.
constexpr int64_t FUSE_ROWS = 256;  // (see the phase list above)
enum Phase { P_NEWTON = 1, P_SOFT, P_ACCEPT, P_RNEWTON, P_RACCEPT, P_ACCEPT_NR, P_FUSED, P_FUSED_R };

int32_t hessian_into(cpl_solver* S, const cpl_problem_desc* d, const uint8_t* mask, const double** Hblk, int* h_sym) {
  const int64_t B = S->Bcur;
  const int n = S->n, nf = S->nf;
  hipStream_t st = S->stream;
  const cpl_solve_options& o = S->opt;
  *Hblk = nullptr;
  *h_sym = 0;
  if (S->bfgs) return CPL_OK;  // the compact model is expanded inside the Newton setup
  // scaled: the callbacks' Hessian at the multipliers (dc y) / df, times df (the scaled Lagrangian
  // df f + (dc y)^T g is df (f + ((dc y) / df)^T g))
  const double* yh = S->y;
  if (S->scaled) {
    hipLaunchKernelGGL(k_scale_y, dim3(blocks_elems(B * S->m)), dim3(256), 0, st, B * S->m, S->m, S->dc, S->df, S->y,
                       S->ytil);
    LAUNCHED("k_scale_y");
    yh = S->ytil;
  }
  auto scale_H = [&]() -> int32_t {
    if (!S->scaled) return CPL_OK;
    hipLaunchKernelGGL(k_scale_rows, dim3(blocks_elems(B * nf * nf)), dim3(256), 0, st, B * nf * nf, nf * nf, S->df,
                       S->H);
    LAUNCHED("k_scale_rows");
    return CPL_OK;
  };
  if (S->analytic_H) {
    CK(cpl_lagrangian_hessian(d, B, S->X, yh, mask, S->free32, nf, S->H, st));
    CK(scale_H());
    *Hblk = S->H;
    return CPL_OK;
  }
  // central differences of grad f + J^T y (the 2 nf points of every instance in one launch)
  CK(cpl_ipm_fd_points(B, n, nf, o.fd_step, S->freepos, S->X, S->Xp, S->hfd, mask, st));
  int32_t rc = CPL_ERR_UNSUPPORTED;
  if (S->fd_fused)
    rc = cpl_eval_lagrangian_grad(d, B * 2 * nf, S->Xp, S->mass ? S->mass_fd : nullptr, S->tag ? S->tag_fd : nullptr,
                                  S->col_ptr, S->csc_k, S->csc_row, yh, 2 * nf, mask, S->gL, st);
  if (rc == CPL_ERR_UNSUPPORTED) {  // Superquadric / mixed: eval + J^T y in two launches
    S->fd_fused = false;
    CK(cpl_eval_batch(d, B * 2 * nf, S->Xp, S->mass ? S->mass_fd : nullptr, S->tag ? S->tag_fd : nullptr, nullptr,
                      S->jac_fd, nullptr, S->grad_fd, st));
    CK(cpl_lagrangian_grad(B * 2 * nf, n, S->m, S->nnz, S->col_ptr, S->csc_k, S->csc_row, S->grad_fd, S->jac_fd, yh,
                           2 * nf, S->gL, st));
  } else {
    CK(rc);
  }
  CK(cpl_ipm_fd_hessian_raw(B, n, nf, S->free64, S->gL, S->hfd, S->H, mask, st));
  CK(scale_H());
  *Hblk = S->H;
  *h_sym = 1;
  return CPL_OK;
}

static NearFeasible near_feasible(cpl_solver* S, const cpl_solve_options& o) {
  return NearFeasible{S->theta_k, 1e-2 * o.tol, S->nw, S->m, S->has_acc, S->acc_w, S->acc_y, S->acc_zL, S->acc_zU,
                      S->w, S->y, S->zL, S->zU};
}

int32_t step_phase(cpl_solver* S, int phase) {
  const int64_t B = S->Bcur;
  const int n = S->n, m = S->m, nf = S->nf, nw = S->nw;
  hipStream_t st = S->stream;
  const cpl_solve_options& o = S->opt;
  const int64_t lmc = S->bfgs ? LMC(nf) : 0;
  auto judge = [&](const double* wt, const double* ft_, const double* gt_, const double* al, const uint8_t* extra,
                   double* th, uint8_t* ok) {
    return cpl_ipm_judge_take(B, nw, m, nf, FMAX, S->row_slack, S->gl, S->hasL, S->hasU, S->wl0, S->wu0, wt, ft_, gt_,
                              al, S->mu_o, S->theta_k, S->phi_k, S->gd, S->switch_ok, S->theta_max, S->ft, S->fp,
                              extra, S->searching, S->st_f, S->st_g, S->st_w, S->st_alpha, S->st_aug, th, ok, 0, st);
  };
  auto halve = [&](uint8_t* searching, double* alpha, const double* a_min, int fi, bool soft) -> int32_t {
    hipLaunchKernelGGL(k_halve2, dim3(blocks_elems(B)), dim3(256), 0, st, B, searching, alpha, a_min, S->act,
                       S->tiny_now, soft ? S->soft_now : nullptr, S->soft_cnt, S->st_alpha, S->d_any, fi);
    LAUNCHED("k_halve2");
    return CPL_OK;
  };
  // the first regular trial: the point, f and g there, IPOPT's acceptance test and the take, its
  // second-order corrections, the halving
  auto first_trial = [&]() -> int32_t {
    CK(cpl_ipm_trial_point(B, n, nf, nw, S->free64, S->fixed64, S->Xbase, S->w, S->dw, S->alpha, S->searching,
                           S->st_w, S->wt, S->Xt, st));
    CK(eval_fg(S, S->Xt, S->f_t, S->g_t));
    CK(judge(S->wt, S->f_t, S->g_t, S->alpha, nullptr, S->th, S->ok));
    if (o.max_soc > 0) {  // second-order corrections on the first trial (IPOPT's max_soc)
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
        if (S->jreg)
          CK(kkt_aug_solve(1, B, nw, m, S->M, S->A, S->r1, S->r2s, nullptr, nullptr, S->soc, S->dws, S->dys, nullptr,
                           S->delta_c, nullptr, S->ws_aug, st));
        CK(cpl_ipm_max_step(B, nw, S->w, S->dws, nullptr, nullptr, S->hasL, S->hasU, S->wl0, S->wu0, S->tau, S->a_soc,
                            st));
        CK(cpl_ipm_trial_point(B, n, nf, nw, S->free64, S->fixed64, S->Xbase, S->w, S->dws, S->a_soc, S->soc, S->st_w,
                               S->ws_, S->Xs, st));
        CK(eval_fg(S, S->Xs, S->f_s, S->g_s));
        CK(judge(S->ws_, S->f_s, S->g_s, S->alpha, S->soc, S->th_s, S->ok_s));
        hipLaunchKernelGGL(k_soc_after, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->soc, S->ok_s, S->th_s,
                           S->th_old);
        LAUNCHED("k_soc_after");
        cg = S->g_s;
        cw = S->ws_;
      }
    }
    return halve(S->searching, S->alpha, S->a_min, 0, true);
  };
  // the first restoration trial: the point (w along dw; p, n in the judge), f and g, the test and the take
  auto rtrial = [&]() -> int32_t {
    CK(cpl_ipm_trial_point(B, n, nf, nw, S->free64, S->fixed64, S->Xbase, S->w, S->dw, S->alphaR, S->searchingR,
                           S->st_w, S->wt, S->Xt, st));
    CK(eval_fg(S, S->Xt, S->f_t, S->g_t));
    hipLaunchKernelGGL(k_resto_judge, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nf, nw, S->searchingR, S->row_slack,
                       S->gl, S->hasL, S->hasU, S->wl0, S->wu0, S->wt, S->f_t, S->g_t, S->alphaR, S->pR, S->nR, S->dp,
                       S->dn, S->wR, S->muR, S->thetaR, S->phiR, S->gdR, S->switchR, S->thmaxR, S->ftR, S->fpR,
                       S->searchingR, S->st_f, S->st_g, S->st_w, S->st_p, S->st_n, S->st_alpha, S->st_aug);
    LAUNCHED("k_resto_judge");
    return halve(S->searchingR, S->alphaR, S->a_minR, 2, false);
  };

  switch (phase) {
    case P_NEWTON: {
      {  // A (active instances) and k_prep's gradw / c in one launch
        const int64_t totalA = B * (int64_t)m * nw;
        const unsigned nblk_a = (unsigned)((totalA + 255) / 256);
        hipLaunchKernelGGL(k_dense_a_prep, dim3(nblk_a + blocks_for(B)), dim3(256), 0, st, totalA, nblk_a, m, nw, nf,
                           S->nnz_rec, S->amap, S->row_slack, S->J, S->A, S->active, B, n, S->free32, S->gl, S->grad, S->g, S->w,
                           S->gradw, S->c);
        LAUNCHED("k_dense_a_prep");
      }
      // (with k_unpack_tau's X = unpack(w), tau and the active snapshot fused into its tail)
      // the whole search in one launch (first trial, its corrections, the backtracking), the post-step
      // quantities and the search's setup in that launch's prologue; or the first trial step by step
      // and the remaining trials in one launch
      const bool fused = o.ls_kernel == 2 || (o.ls_kernel == 1 && B <= FUSE_ROWS);  // (2: the default)
      const bool fused_ls = fused && S->ls_fusable;
      const bool post_in_ls = fused_ls && ls_post_prologue(B);  // (the search kernel's prologue)
      const IpmUnpack unp{n, S->freepos, S->Xbase, S->in_resto, S->X, S->tau, S->act,
                          S->acc_w, S->acc_y, S->acc_zL, S->acc_zU, S->has_acc, post_in_ls ? S->d_any : nullptr,
                          S->in_soft};
      CK(ipm_optimality_ex(B, nw, m, FMAX, S->nbounds, o.tol, o.acceptable_tol, o.acceptable_iter, S->A, S->gradw,
                           S->c, S->w, S->y, S->zL, S->zU, S->hasL, S->hasU, S->wl0, S->wu0, S->mu, S->filt_t,
                           S->filt_p, S->fcount, S->active, S->status, S->acc, S->d_inf, S->err0, S->base, S->mu_o,
                           S->ft, S->fp, S->fc, MU_ROUNDS, S->mu_min, S->tiny_flag, S->in_resto, &unp, st));
      const double* Hblk = nullptr;
      int h_sym = 0;
      CK(hessian_into(S, &S->desc, S->act, &Hblk, &h_sym));
      if (S->bfgs)
        CK(ipm_newton_setup_lm(B, nw, m, nf, S->w, S->zL, S->zU, S->gradw, S->A, S->y, S->c, S->f, S->mu_o, S->hasL,
                               S->hasU, S->wl0, S->wu0, S->Hq, LM_HIST, S->M, S->r1, S->r2, S->gphi, S->mr_diag,
                               S->theta_k, S->phi_k, S->act, st));
      else
        CK(cpl_ipm_newton_setup(B, nw, m, nf, S->w, S->zL, S->zU, S->gradw, S->A, S->y, S->c, S->f, S->mu_o, S->hasL,
                                S->hasU, S->wl0, S->wu0, Hblk, h_sym, S->M, S->r1, S->r2, S->gphi, S->mr_diag,
                                S->theta_k, S->phi_k, S->act, st));
      CK(cpl_kkt_solve(0, B, nw, m, S->M, S->A, S->r1, S->r2, S->mu_o, S->dwl, S->act, S->dw, S->dy, S->delta_w,
                       S->delta_c, S->info, S->ws, st));
      if (S->jreg)
        CK(kkt_aug_solve(0, B, nw, m, S->M, S->A, S->r1, S->r2, S->mu_o, S->dwl, S->act, S->dw, S->dy, S->delta_w,
                         S->delta_c, S->info, S->ws_aug, st));
      // the step's multipliers / fraction-to-the-boundary, then the search's setup: a launch of their
      // own, or the fused search kernel's prologue
      LsSetupArgs ls;
      ls.m = m; ls.act = S->act; ls.w = S->w; ls.dw = S->dw; ls.dy = S->dy; ls.c = S->c; ls.f = S->f; ls.g = S->g;
      ls.theta_k = S->theta_k; ls.theta_min = S->theta_min; ls.in_soft = S->in_soft; ls.soft_cnt = S->soft_cnt;
      ls.tiny_last = S->tiny_last; ls.tiny_flag = S->tiny_flag; ls.tiny_now = S->tiny_now; ls.soft_now = S->soft_now;
      ls.a_min = S->a_min; ls.searching = S->searching; ls.st_f = S->st_f; ls.st_g = S->st_g; ls.st_w = S->st_w;
      ls.st_alpha = S->st_alpha; ls.st_aug = S->st_aug; ls.alpha = S->alpha; ls.any = S->d_any;
      const PostStepArgs post{nw, S->w, S->dw, S->zL, S->zU, S->gphi, S->mu_o, S->tau, S->hasL, S->hasU, S->wl0,
                              S->wu0, S->theta_k, S->theta_min, S->act, S->delta_w, S->dwl, S->dzL, S->dzU,
                              S->a_max, S->a_z, S->gd, S->switch_ok};
      if (!post_in_ls)
        CK(ipm_post_step_ex(B, nw, S->w, S->dw, S->zL, S->zU, S->gphi, S->mu_o, S->tau, S->hasL, S->hasU, S->wl0,
                            S->wu0, S->theta_k, S->theta_min, S->act, S->delta_w, S->dwl, S->dzL, S->dzU, S->a_max,
                            S->a_z, S->gd, S->switch_ok, &ls, st));
      if (!fused_ls) CK(first_trial());
      if (fused && S->ls_fusable) {
        LsBacktrackArgs la;
        la.batch = B; la.n = n; la.m = m; la.nf = nf; la.nw = nw; la.nfilt = FMAX; la.max_trials = o.max_ls - 1;
        if (la.max_trials < 0) la.max_trials = 0;
        la.act = S->act; la.tiny = S->tiny_now; la.soft_now = S->soft_now; la.soft_cnt = S->soft_cnt;
        la.searching = S->searching; la.alpha = S->alpha; la.a_min = S->a_min;
        la.w = S->w; la.dw = S->dw; la.Xbase = S->Xbase; la.freepos = S->freepos; la.row_slack = S->row_slack;
        la.gl = S->gl; la.hasL = S->hasL; la.hasU = S->hasU; la.wl0 = S->wl0; la.wu0 = S->wu0;
        la.mu = S->mu_o; la.theta_k = S->theta_k; la.phi_k = S->phi_k; la.gd = S->gd; la.switch_ok = S->switch_ok;
        la.theta_max = S->theta_max; la.filt_t = S->ft; la.filt_p = S->fp;
        la.mass = S->mass; la.env_tag = S->tag;
        if (S->scaled) { la.df = S->df; la.dc = S->dc; }
        la.st_f = S->st_f; la.st_g = S->st_g; la.st_w = S->st_w; la.st_alpha = S->st_alpha; la.st_aug = S->st_aug;
        la.any = S->d_any;
        la.resto = 0;
        la.rho = 0.0;
        la.pR = la.nR = la.dp = la.dn = la.wR = nullptr;
        la.st_p = la.st_n = nullptr;
        la.first = 1;
        la.max_soc = o.max_soc;
        la.c = S->c; la.M = S->M; la.r1 = S->r1; la.kkt_ws = S->ws; la.tau = S->tau;
        if (S->jreg) { la.aug_dc = S->delta_c; la.aug_ws = S->ws_aug; }  // (the regularised systems' re-solves)
        la.a_max = S->a_max; la.a_z = S->a_z;
        la.soft_ws = la.soft_X = la.a_soft = nullptr; la.soft_try = nullptr;
        if (S->soft_fused) {
          la.soft_ws = S->ws_; la.soft_X = S->Xs; la.soft_try = S->soft_try; la.a_soft = S->a_soft;
          S->soft_begun = true;
        }
        la.post = post;
        la.setup = ls;
        la.setup.any = nullptr;  // (cleared by the optimality kernel: other waves set them concurrently)
        la.with_post = post_in_ls ? 1 : 0;
        CK(ls_backtrack(&S->desc, la, st));
      } else if (o.max_ls > 1) {  // the remaining trials of every instance still searching, in one launch
        HK(hipMemsetAsync(S->d_any, 0, 2, st), "hipMemsetAsync flags");
        LsBacktrackArgs la;
        la.batch = B; la.n = n; la.m = m; la.nf = nf; la.nw = nw; la.nfilt = FMAX; la.max_trials = o.max_ls - 1;
        la.act = S->act; la.tiny = S->tiny_now; la.soft_now = S->soft_now; la.soft_cnt = S->soft_cnt;
        la.searching = S->searching; la.alpha = S->alpha; la.a_min = S->a_min;
        la.w = S->w; la.dw = S->dw; la.Xbase = S->Xbase; la.freepos = S->freepos; la.row_slack = S->row_slack;
        la.gl = S->gl; la.hasL = S->hasL; la.hasU = S->hasU; la.wl0 = S->wl0; la.wu0 = S->wu0;
        la.mu = S->mu_o; la.theta_k = S->theta_k; la.phi_k = S->phi_k; la.gd = S->gd; la.switch_ok = S->switch_ok;
        la.theta_max = S->theta_max; la.filt_t = S->ft; la.filt_p = S->fp;
        la.mass = S->mass; la.env_tag = S->tag;
        if (S->scaled) { la.df = S->df; la.dc = S->dc; }
        la.st_f = S->st_f; la.st_g = S->st_g; la.st_w = S->st_w; la.st_alpha = S->st_alpha; la.st_aug = S->st_aug;
        la.any = S->d_any;
        la.resto = 0;
        la.rho = 0.0;
        la.pR = la.nR = la.dp = la.dn = la.wR = nullptr;
        la.st_p = la.st_n = nullptr;
        la.first = 0; la.max_soc = 0; la.c = la.M = la.r1 = la.kkt_ws = la.tau = nullptr;
        la.with_post = 0;
        la.a_max = la.a_z = nullptr; la.soft_ws = la.soft_X = la.a_soft = nullptr; la.soft_try = nullptr;
        CK(ls_backtrack(&S->desc, la, st));
      }
      return CPL_OK;
    }
    case P_SOFT: {
      if (!S->soft_begun) {  // (else the Newton phase's search kernel started the soft step)
        hipLaunchKernelGGL(k_soft_begin, dim3(blocks_for(B)), dim3(256), 0, st, B, n, nf, nw, S->act, S->tiny_now,
                           S->soft_now, S->soft_cnt, S->st_alpha, S->a_max, S->a_z, S->w, S->dw, S->freepos, S->Xbase,
                           S->soft_try, S->a_soft, S->ws_, S->Xs);
        LAUNCHED("k_soft_begin");
      }
      // (the fused search kernel raised d_any[1] exactly where it set soft_try: with no soft-step candidate
      // this evaluation's outputs are read by nobody, and its launch returns at once)
      CK(eval_full(S, S->Xs, S->f_n, S->grad_n, S->g_n, S->J_n, S->soft_begun ? S->d_any + 1 : nullptr));
      if (S->tail_fused) {
        const FailTail tail{S->freepos, S->Xbase, S->Xn, S->act, S->err0, o.acceptable_tol, S->failed, S->moved,
                            S->status, S->active, near_feasible(S, o)};
        hipLaunchKernelGGL(k_soft_judge_fail, dim3(blocks_for(B)), dim3(256), 0, st, B, n, m, nf, nw, S->nnz_rec,
                           S->soft_try, S->soft_now, S->a_soft, S->amap, S->row_slack, S->free32, S->gl, S->hasL,
                           S->hasU, S->wl0, S->wu0, S->ws_, S->f_n, S->grad_n, S->g_n, S->J_n, S->A, S->gradw, S->c,
                           S->w, S->y, S->zL, S->zU, S->dy, S->dzL, S->dzU, S->mu_o, S->theta_k, S->phi_k, S->gd,
                           S->switch_ok, S->theta_max, S->ft, S->fp, S->cs_tmp, S->in_soft, S->soft_cnt, S->st_f,
                           S->st_g, S->st_w, S->st_alpha, S->st_aug, S->a_z, tail);
        LAUNCHED("k_soft_judge_fail");
        return CPL_OK;
      }
      hipLaunchKernelGGL(k_soft_judge, dim3(blocks_for(B)), dim3(256), 0, st, B, n, m, nf, nw, S->nnz_rec, S->soft_try,
                         S->soft_now, S->a_soft, S->amap, S->row_slack, S->free32, S->gl, S->hasL, S->hasU, S->wl0,
                         S->wu0, S->ws_, S->f_n, S->grad_n, S->g_n, S->J_n, S->A, S->gradw, S->c, S->w, S->y, S->zL,
                         S->zU, S->dy, S->dzL, S->dzU, S->mu_o, S->theta_k, S->phi_k, S->gd, S->switch_ok,
                         S->theta_max, S->ft, S->fp, S->cs_tmp, S->in_soft, S->soft_cnt, S->st_f, S->st_g, S->st_w,
                         S->st_alpha, S->st_aug, S->a_z);
      LAUNCHED("k_soft_judge");
      return CPL_OK;
    }
    case P_ACCEPT:
    case P_ACCEPT_NR: {
      // the failed-search bookkeeping and the accepted points (done by the soft judge's launch in
      // P_FUSED), then one full evaluation there
      if (!S->tail_fused) {
        hipLaunchKernelGGL(k_fail_unpack, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, nw, S->freepos,
                           S->Xbase, S->st_w, S->Xn, S->act, S->st_alpha, S->err0, o.acceptable_tol, S->failed,
                           S->moved, S->in_soft, S->soft_cnt, S->status, S->active, near_feasible(S, o));
        LAUNCHED("k_fail_unpack");
      }
      CK(eval_full(S, S->Xn, S->f_n, S->grad_n, S->g_n, S->J_n));
      if (S->bfgs) {
        if (nf <= 64)
          hipLaunchKernelGGL(k_lbfgs_wave, dim3((unsigned)((B + LBW_WAVES - 1) / LBW_WAVES)), dim3(64 * LBW_WAVES),
                             sizeof(double) * LBW_WAVES * (size_t)m, st, B, m, nf, nw, S->nnz_rec, S->amap, S->moved,
                             S->w, S->st_w, S->y, S->dy, S->st_alpha, S->gradw, S->J, S->grad_n, S->free32, n, S->J_n,
                             S->lm_s, S->lm_y, S->lm_cnt, S->lm_skip, S->zeros_u8, S->Hq);
        else
          hipLaunchKernelGGL(k_lbfgs<128>, dim3((unsigned)B), dim3(256), 0, st, B, m, nf, nw, S->nnz_rec, S->amap, S->moved,
                             S->w, S->st_w, S->y, S->dy, S->st_alpha, S->gradw, S->J, S->grad_n, S->free32, n, S->J_n,
                             S->lm_s, S->lm_y, S->lm_cnt, S->lm_skip, S->zeros_u8, S->Hq);
        LAUNCHED("k_lbfgs");
      }
      const IpmAcceptArgs acc{nw, m, FMAX, S->moved, S->st_aug, nullptr, nullptr, S->st_alpha, S->a_z, S->theta_k,
                              S->phi_k, S->ft, S->fp, S->fc, S->st_w, S->dy, S->dzL, S->dzU, S->mu_o, S->hasL,
                              S->hasU, S->wl0, S->wu0, S->w, S->y, S->zL, S->zU, S->mu, S->iters, S->filt_t,
                              S->filt_p, S->fcount};
      AcceptRows ar{S->moved, n, m, S->nnz_rec, S->f_n, S->grad_n, S->g_n, S->J_n, S->f, S->grad, S->g, S->J};
      if (phase == P_ACCEPT_NR) {  // no instance can have failed its search: no entry
        CK(cpl_ipm_accept(B, nw, m, FMAX, S->moved, S->st_aug, nullptr, nullptr, S->st_alpha, S->a_z, S->theta_k,
                          S->phi_k, S->ft, S->fp, S->fc, S->st_w, S->dy, S->dzL, S->dzU, S->mu_o, S->hasL, S->hasU,
                          S->wl0, S->wu0, S->w, S->y, S->zL, S->zU, S->mu, S->iters, S->filt_t, S->filt_p, S->fcount,
                          st));
        hipLaunchKernelGGL(k_accept_rows, dim3(blocks_elems(B * (1 + n + m + S->nnz_rec))), dim3(256), 0, st, B, n,
                           m, S->nnz_rec, S->moved, S->f_n, S->grad_n, S->g_n, S->J_n, S->f, S->grad, S->g, S->J);
        LAUNCHED("k_accept_rows");
        goto count;
      }
      {  // the restoration phase starts where the line search failed
      RestoEnterArgs E{m, nw, S->failed, S->c, S->w, S->zL, S->zU, S->mu_o, S->theta_k, S->phi_k, S->hasL, S->hasU,
                       S->filt_t, S->filt_p, S->fcount, S->iters, S->in_resto, S->n_resto, S->wR, S->pR, S->nR, S->zp,
                       S->zn, S->zLR, S->zUR, S->muR, S->ftR, S->fpR, S->fcR, S->thmaxR, S->thminR, S->th_o0, S->ph_o0,
                       S->dwlR, S->lm_cnt, S->lm_skip, S->bfgs ? S->Hq : nullptr, lmc, S->M, S->r1, S->r2, S->Dinv, ar,
                       acc, true};
      if (B <= FUSE_ROWS && sizeof(double) * qd_lds_doubles(nw, m) <= 160 * 1024) {
        // the entry, its least-squares multipliers and the counts in one launch (k_tail_small)
        const QdSolveArgs Q{nw, m, S->M, S->A, S->Dinv, S->r1, S->r2, S->dwlR, S->dw, S->dy, S->scr1, S->Kqd};
        TrackBest tb{};
        if (o.fallback_viol_tol > 0.0)
          tb = TrackBest{nw, o.fallback_viol_tol, S->w, S->f, S->g, S->gl, S->gu, S->best_w, S->best_f,
                         S->scaled ? S->dc : nullptr};
        hipLaunchKernelGGL(k_tail_small, dim3((unsigned)B), dim3(TAIL_THREADS), sizeof(double) * qd_lds_doubles(nw, m),
                           st, B, E, Q, S->active, S->in_resto, S->d_count, S->h_count, S->y, tb);
        LAUNCHED("k_tail_small (the entry, its multipliers, the counts)");
        return CPL_OK;
      }
      hipLaunchKernelGGL(k_resto_enter, dim3(blocks_for(B)), dim3(256), 0, st, B, E);
      LAUNCHED("k_resto_enter (+ the accept, the accepted rows)");
      CK(cpl_kkt_qd_solve(B, nw, m, S->M, S->A, S->Dinv, S->r1, S->r2, S->failed, S->dwlR, S->dw, S->dy, S->scr1,
                          S->Kqd, st));
      if (B > COUNT1_MAX) {
        hipLaunchKernelGGL(k_resto_y0, dim3(blocks_for(B)), dim3(256), 0, st, B, m, S->failed, S->dy, S->y);
        LAUNCHED("k_resto_y0");
      }
      }
    count:
      const bool track_fused = o.fallback_viol_tol > 0.0 && B <= TRACK_FUSE_ROWS;
      TrackBest tb{};
      if (track_fused) tb = TrackBest{nw, o.fallback_viol_tol, S->w, S->f, S->g, S->gl, S->gu, S->best_w, S->best_f,
                         S->scaled ? S->dc : nullptr};
      if (o.fallback_viol_tol > 0.0 && !track_fused) {
        hipLaunchKernelGGL(k_track_best, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nw, o.fallback_viol_tol,
                           S->active, S->w, S->f, S->g, S->gl, S->gu, S->best_w, S->best_f, S->scaled ? S->dc : nullptr);
        LAUNCHED("k_track_best");
      }
      if (B > COUNT1_MAX) {
        hipLaunchKernelGGL(k_count_zero, dim3(1), dim3(64), 0, st, S->d_count);
        LAUNCHED("k_count_zero");
        hipLaunchKernelGGL(k_count, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->active, S->in_resto, S->d_count);
      } else {
        // (with the restoration entry's multiplier reset fused in: P_ACCEPT)
        hipLaunchKernelGGL(k_count1, dim3(1), dim3(1024), 0, st, B, S->active, S->in_resto, S->d_count, S->h_count, m,
                           phase == P_ACCEPT ? S->failed : nullptr, S->dy, S->y, tb);
      }
      LAUNCHED("k_count");
      return CPL_OK;
    }
    case P_RNEWTON: {
      hipLaunchKernelGGL(k_resto_prep1, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nf, nw, S->nbounds, o.tol,
                         S->mu_min, S->active, S->in_resto, S->resto_tight, S->actR, S->status, S->A, S->c, S->w, S->y,
                         S->wR, S->pR,
                         S->nR, S->zp, S->zn, S->zLR, S->zUR, S->hasL, S->hasU, S->wl0, S->wu0, S->muR, S->ftR,
                         S->fpR, S->fcR, S->tauR, S->gfR);
      LAUNCHED("k_resto_prep1");
      hipLaunchKernelGGL(k_restore_acc, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nw, S->status, S->has_acc,
                         S->acc_w, S->acc_y, S->acc_zL, S->acc_zU, S->w, S->y, S->zL, S->zU);
      LAUNCHED("k_restore_acc");
      const double* Hblk = nullptr;
      int h_sym = 0;
      CK(hessian_into(S, &S->desc_R, S->actR, &Hblk, &h_sym));
      if (S->bfgs)
        CK(ipm_newton_setup_lm(B, nw, m, nf, S->w, S->zLR, S->zUR, S->gfR, S->A, S->y, S->c, S->f, S->muR, S->hasL,
                               S->hasU, S->wl0, S->wu0, S->Hq, LM_HIST, S->M, S->r1, S->scr2, S->gphi, S->mr_diag,
                               S->scr1, S->scr1 + S->B, S->actR, st));
      else
        CK(cpl_ipm_newton_setup(B, nw, m, nf, S->w, S->zLR, S->zUR, S->gfR, S->A, S->y, S->c, S->f, S->muR, S->hasL,
                                S->hasU, S->wl0, S->wu0, Hblk, h_sym, S->M, S->r1, S->scr2, S->gphi, S->mr_diag,
                                S->scr1, S->scr1 + S->B, S->actR, st));
      hipLaunchKernelGGL(k_resto_prep2, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nf, nw, S->actR, S->c, S->w, S->y,
                         S->wR, S->pR, S->nR, S->zp, S->zn, S->muR, S->hasL, S->hasU, S->wl0, S->wu0, S->M, S->rp,
                         S->rn, S->Dinv, S->r2, S->thetaR, S->phiR);
      LAUNCHED("k_resto_prep2");
      CK(cpl_kkt_qd_solve(B, nw, m, S->M, S->A, S->Dinv, S->r1, S->r2, S->actR, S->dwlR, S->dw, S->dy, S->scr1,
                          S->Kqd, st));
      hipLaunchKernelGGL(k_resto_post, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nw, S->actR, S->w, S->dw, S->dy,
                         S->gphi, S->pR, S->nR, S->zp, S->zn, S->zLR, S->zUR, S->rp, S->rn, S->muR, S->tauR, S->hasL,
                         S->hasU, S->wl0, S->wu0, S->thetaR, S->thminR, S->f, S->g, S->dp, S->dn, S->dzL, S->dzU,
                         S->dzp, S->dzn, S->a_maxR, S->a_zR, S->gdR, S->switchR, S->a_minR, S->searchingR, S->st_f,
                         S->st_g, S->st_w, S->st_p, S->st_n, S->st_alpha, S->st_aug, S->alphaR, S->d_any);
      LAUNCHED("k_resto_post");
      CK(rtrial());
      if (o.max_ls > 1) {  // the restoration search's remaining trials, in one launch
        HK(hipMemsetAsync(S->d_any + 2, 0, 1, st), "hipMemsetAsync flag");
        LsBacktrackArgs la;
        la.batch = B; la.n = n; la.m = m; la.nf = nf; la.nw = nw; la.nfilt = FMAX; la.max_trials = o.max_ls - 1;
        la.act = S->actR; la.tiny = S->tiny_now; la.soft_now = S->soft_now; la.soft_cnt = S->soft_cnt;
        la.searching = S->searchingR; la.alpha = S->alphaR; la.a_min = S->a_minR;
        la.w = S->w; la.dw = S->dw; la.Xbase = S->Xbase; la.freepos = S->freepos; la.row_slack = S->row_slack;
        la.gl = S->gl; la.hasL = S->hasL; la.hasU = S->hasU; la.wl0 = S->wl0; la.wu0 = S->wu0;
        la.mu = S->muR; la.theta_k = S->thetaR; la.phi_k = S->phiR; la.gd = S->gdR; la.switch_ok = S->switchR;
        la.theta_max = S->thmaxR; la.filt_t = S->ftR; la.filt_p = S->fpR;
        la.mass = S->mass; la.env_tag = S->tag;
        if (S->scaled) { la.df = S->df; la.dc = S->dc; }
        la.st_f = S->st_f; la.st_g = S->st_g; la.st_w = S->st_w; la.st_alpha = S->st_alpha; la.st_aug = S->st_aug;
        la.any = S->d_any;
        la.resto = 1;
        la.rho = RHO_R;
        la.pR = S->pR; la.nR = S->nR; la.dp = S->dp; la.dn = S->dn; la.wR = S->wR;
        la.st_p = S->st_p; la.st_n = S->st_n;
        la.first = 0; la.max_soc = 0; la.c = la.M = la.r1 = la.kkt_ws = la.tau = nullptr;
        la.with_post = 0;
        la.a_max = la.a_z = nullptr; la.soft_ws = la.soft_X = la.a_soft = nullptr; la.soft_try = nullptr;
        CK(ls_backtrack(&S->desc, la, st));
      }
      return step_phase(S, P_RACCEPT);
    }
    case P_RACCEPT: {
      hipLaunchKernelGGL(k_unpack, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, nw, S->freepos, S->Xbase,
                         S->st_w, nullptr, nullptr, S->Xn);
      LAUNCHED("k_unpack (resto)");
      CK(eval_full(S, S->Xn, S->f_n, S->grad_n, S->g_n, S->J_n));
      if (S->bfgs) {  // the restoration phase's own model: pairs from J^T y (its constraint curvature)
        hipLaunchKernelGGL(k_moved_r, dim3(blocks_elems(B)), dim3(256), 0, st, B, S->actR, S->st_alpha, S->movedR);
        LAUNCHED("k_moved_r");
        if (nf <= 64)
          hipLaunchKernelGGL(k_lbfgs_wave, dim3((unsigned)((B + LBW_WAVES - 1) / LBW_WAVES)), dim3(64 * LBW_WAVES),
                             sizeof(double) * LBW_WAVES * (size_t)m, st, B, m, nf, nw, S->nnz_rec, S->amap, S->movedR,
                             S->w, S->st_w, S->y, S->dy, S->st_alpha, S->zeros_w, S->J, nullptr, S->free32, n, S->J_n,
                             S->lm_s, S->lm_y, S->lm_cnt, S->lm_skip, S->zeros_u8, S->Hq);
        else
          hipLaunchKernelGGL(k_lbfgs<128>, dim3((unsigned)B), dim3(256), 0, st, B, m, nf, nw, S->nnz_rec, S->amap,
                             S->movedR, S->w, S->st_w, S->y, S->dy, S->st_alpha, S->zeros_w, S->J, nullptr, S->free32, n,
                             S->J_n, S->lm_s, S->lm_y, S->lm_cnt, S->lm_skip, S->zeros_u8, S->Hq);
        LAUNCHED("k_lbfgs (resto)");
      }
      hipLaunchKernelGGL(k_resto_accept, dim3(blocks_for(B)), dim3(256), 0, st, B, m, nf, nw, S->actR, S->movedR,
                         S->active, S->status, S->iters, S->st_alpha, S->st_aug, S->st_w, S->st_p, S->st_n, S->dy,
                         S->dzL, S->dzU, S->dzp, S->dzn, S->a_zR, S->muR, S->thetaR, S->phiR, S->ftR, S->fpR, S->fcR,
                         S->w, S->y, S->pR, S->nR, S->zp, S->zn, S->zLR, S->zUR, S->hasL, S->hasU, S->wl0, S->wu0,
                         S->row_slack, S->gl, S->f_n, S->g_n, S->mu, S->filt_t, S->filt_p, S->th_o0, S->ph_o0, S->wR,
                         S->zL, S->zU, S->in_resto, S->acc, S->lm_cnt, S->lm_skip, S->bfgs ? S->Hq : nullptr, lmc);
      LAUNCHED("k_resto_accept");
      hipLaunchKernelGGL(k_accept_rows, dim3(blocks_elems(B * (1 + n + m + S->nnz_rec))), dim3(256), 0, st, B, n, m,
                         S->nnz_rec, S->movedR, S->f_n, S->grad_n, S->g_n, S->J_n, S->f, S->grad, S->g, S->J);
      LAUNCHED("k_accept_rows (resto)");
      return CPL_OK;
    }
    case P_FUSED:
    case P_FUSED_R: {
      S->soft_fused = true;
      S->soft_begun = false;
      {
        const int32_t rc0 = step_phase(S, P_NEWTON);
        if (rc0 != CPL_OK) {
          S->soft_fused = S->soft_begun = false;
          return rc0;
        }
      }
      // P_SOFT and P_ACCEPT adjacent (no restoration iteration between): one launch ends the search
      S->tail_fused = phase == P_FUSED;
      int32_t rc = step_phase(S, P_SOFT);
      S->soft_fused = S->soft_begun = false;
      if (rc == CPL_OK && phase == P_FUSED_R) rc = step_phase(S, P_RNEWTON);
      if (rc == CPL_OK) rc = step_phase(S, P_ACCEPT);
      S->tail_fused = false;
      return rc;
    }
    default:
      return fail(CPL_ERR_INVALID_ARGUMENT, "step_phase: bad phase");
  }
}

// the graph of one phase at the current batch size (captured once per (size, inputs, phase), then
// replayed); without graphs the phase is launched directly
int32_t run_phase(cpl_solver* S, int phase) {
  if (!S->opt.use_graph) return step_phase(S, phase);
  const int64_t key = ((S->Bcur * 8 + (S->scaled ? 4 : 0) + (S->mass ? 2 : 0) + (S->tag ? 1 : 0)) * 16) + phase;
  auto it = S->graphs.find(key);
  if (it == S->graphs.end()) {
    HK(hipStreamBeginCapture(S->stream, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
    const int32_t rc = step_phase(S, phase);
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
    S->captured = true;
  }
  HK(hipGraphLaunch(it->second.second, S->stream), "hipGraphLaunch");
  return CPL_OK;
}

// the device's flags (any still searching / soft candidates / restoration searching) to the host
// wait for iteration `seq`'s counts in the mailbox (k_count1), polling; the stream is queried
// every 1024 polls so that a failed launch ends the wait with its error
int32_t wait_mail(cpl_solver* S, int32_t seq) {
  volatile int32_t* mb = S->h_count;
  for (uint32_t k = 1;; ++k) {
    if (mb[2] == seq) break;
    if ((k & 1023u) == 0) {
      const hipError_t q = hipStreamQuery(S->stream);
      if (q == hipSuccess) {
        if (mb[2] == seq) break;
        return fail(CPL_ERR_RUNTIME, "cpl_solver_solve: the iteration's counts never reached the host");
      }
      if (q != hipErrorNotReady) return hip_err(q, "hipStreamQuery");
    }
    __builtin_ia32_pause();
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return CPL_OK;
}

int32_t read_flags(cpl_solver* S) {
  HK(hipMemcpyAsync(S->h_flag, S->d_any, 4, hipMemcpyDeviceToHost, S->stream), "hipMemcpyAsync flags");
  HK(hipStreamSynchronize(S->stream), "hipStreamSynchronize");
  return CPL_OK;
}

// Active-set compaction: the finished rows' results go to the full-batch arrays, the `count` active
// rows move to the front (every per-instance state buffer gathered), the batch shrinks to Bn rows
// (the rows past `count` padded inactive), so later iterations cost what their active instances do.
int32_t compact(cpl_solver* S, int64_t count, int64_t Bn) {
  hipStream_t st = S->stream;
  const int64_t Bc = S->Bcur;
  const int n = S->n, m = S->m, nw = S->nw;
  if (S->opt.fallback_viol_tol > 0.0) {
    hipLaunchKernelGGL(k_fallback, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, m, nw, S->opt.fallback_viol_tol, true,
                       S->orig, S->active, S->status, S->g, S->gl, S->gu, S->best_w, S->best_f, S->w, S->fbest,
                       S->scaled ? S->dc : nullptr);
    LAUNCHED("k_fallback");
  }
  hipLaunchKernelGGL(k_scatter_final, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, n, m, nw, true, S->orig, S->active,
                     S->w, S->y, S->scaled ? S->dc : nullptr, S->df, S->Xbase, S->d_inf, S->status, S->iters, S->n_resto, S->fw, S->fy,
                     S->fX, S->fdinf,
                     S->fstatus, S->fiters, S->fresto);
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
  CK(move(S->status, 1)); CK(move(S->iters, 1)); CK(move(S->acc, 1)); CK(move(S->fcount, 1)); CK(move(S->n_resto, 1));
  // the restoration phase's state
  CK(move(S->wR, nw)); CK(move(S->pR, m)); CK(move(S->nR, m)); CK(move(S->zp, m)); CK(move(S->zn, m));
  CK(move(S->zLR, nw)); CK(move(S->zUR, nw)); CK(move(S->muR, 1)); CK(move(S->ftR, FMAX)); CK(move(S->fpR, FMAX));
  CK(move(S->fcR, 1)); CK(move(S->th_o0, 1)); CK(move(S->ph_o0, 1)); CK(move(S->dwlR, 1)); CK(move(S->thmaxR, 1));
  CK(move(S->thminR, 1)); CK(move(S->best_w, nw)); CK(move(S->best_f, 1));
  CK(move(S->acc_w, nw)); CK(move(S->acc_y, m)); CK(move(S->acc_zL, nw)); CK(move(S->acc_zU, nw));
  if (S->scaled) {
    CK(move(S->df, 1));
    CK(move(S->dc, m));
  }
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
  CK(move_bytes(S->in_soft));
  CK(move_bytes(S->tiny_last));
  CK(move_bytes(S->tiny_flag));
  CK(move_bytes(S->in_resto));
  CK(move_bytes(S->resto_tight));
  CK(move_bytes(S->has_acc));
  if (S->tag) CK(move_bytes(S->tag_c));
  auto move_i32 = [&](int32_t* buf) -> int32_t {
    hipLaunchKernelGGL(k_gather_i32, dim3(blocks_elems(count)), dim3(256), 0, st, count, S->pos, buf,
                       (int32_t*)S->scratch);
    LAUNCHED("k_gather_i32");
    HK(hipMemcpyAsync(buf, S->scratch, 4 * (size_t)count, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
    return CPL_OK;
  };
  CK(move_i32(S->orig));
  CK(move_i32(S->soft_cnt));
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
  o->max_ls = 40;   // backtracking trials at most (IPOPT stops at alpha_min, ~20 halvings typically)
  o->max_soc = 4;   // IPOPT's max_soc
  o->acceptable_iter = 15;
  o->use_graph = 1;
  o->compact = 1;
  o->ls_kernel = 2;
  o->tol = 1e-8;
  o->acceptable_tol = 1e-6;
  o->mu_init = 0.1;
  o->fd_step = 1e-6;
  o->fallback_viol_tol = 0.0;  // off: IPOPT returns its last iterate
  o->nlp_scaling = 1;          // IPOPT's default nlp_scaling_method gradient-based
  o->jacobian_regularization = 0;  // R's pivots (the restatements' default); 1: IPOPT's (2,2) block
}

int32_t cpl_solver_destroy(cpl_solver* S) {
  if (!S) return CPL_OK;
  for (auto& g : S->graphs) {
    (void)hipGraphExecDestroy(g.second.second);
    (void)hipGraphDestroy(g.second.first);
  }
  S->graphs.clear();
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
  if (graph_captured) *graph_captured = S->captured ? 1 : 0;
  return CPL_OK;
}

int32_t cpl_solver_stats(const cpl_solver* S, int32_t* compactions, int64_t* final_rows) {
  if (!S) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_stats: null solver");
  if (compactions) *compactions = S->compactions;
  if (final_rows) *final_rows = S->Bcur;
  return CPL_OK;
}

int32_t cpl_solver_fallbacks(const cpl_solver* S, uint8_t* d_out, void* stream) {
  if (!S || !d_out) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_fallbacks: null argument");
  HK(hipMemcpyAsync(d_out, S->fbest, (size_t)S->B, hipMemcpyDeviceToDevice, (hipStream_t)stream),
     "hipMemcpyAsync fallbacks");
  return CPL_OK;
}

int32_t cpl_solver_nan_jacobian(const cpl_solver* S, int32_t* d_out, void* stream) {
  if (!S || !d_out) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_nan_jacobian: null argument");
  HK(hipMemcpyAsync(d_out, S->nan_cnt, 4 * (size_t)S->B, hipMemcpyDeviceToDevice, (hipStream_t)stream),
     "hipMemcpyAsync nan_jacobian");
  return CPL_OK;
}

int32_t cpl_solver_restorations(const cpl_solver* S, int64_t* d_out, void* stream) {
  if (!S || !d_out) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_solver_restorations: null argument");
  HK(hipMemcpyAsync(d_out, S->fresto, 8 * (size_t)S->B, hipMemcpyDeviceToDevice, (hipStream_t)stream),
     "hipMemcpyAsync restorations");
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
      opt.max_ls < 0 || !(opt.tol > 0.0) || opt.ls_kernel < 0 || opt.ls_kernel > 2 || opt.nlp_scaling < 0 ||
      opt.nlp_scaling > 1 || opt.jacobian_regularization < 0 || opt.jacobian_regularization > 1)
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

  // nlp_scaling: each record's row, and the free-column records of each row (CSR)
  std::vector<int32_t> rrow(nnz_rec), srp(m + 1, 0), srq;
  for (int q = 0; q < nnz_rec; ++q) {
    rrow[q] = iRow[var_k[q]];
    if (freepos[jCol[var_k[q]]] >= 0) ++srp[rrow[q] + 1];
  }
  for (int r = 0; r < m; ++r) srp[r + 1] += srp[r];
  srq.resize(srp[m]);
  {
    std::vector<int32_t> fill(srp.begin(), srp.end() - 1);
    for (int q = 0; q < nnz_rec; ++q)
      if (freepos[jCol[var_k[q]]] >= 0) srq[fill[rrow[q]]++] = q;
  }

  cpl_solver* S = new cpl_solver();
  S->desc = *d;
  S->desc_R = *d;  // zero cost weights: the Hessian of y^T g alone (the restoration phase)
  S->desc_R.W_com = 0.0;
  for (int i = 0; i < CPL_MAX_CONTACTS; ++i) S->desc_R.W_p[i] = S->desc_R.W_F[i] = 0.0;
  S->opt = opt;
  S->B = batch;
  S->n = n; S->m = m; S->nnz = nnz; S->nnz_rec = nnz_rec; S->nf = nf; S->nI = nI; S->nw = nw; S->nbounds = nbounds;
  S->jreg = opt.jacobian_regularization == 1;
  if (S->jreg && kkt_aug_workspace_doubles(nw, m) < 0) {
    delete S;
    return fail(CPL_ERR_UNSUPPORTED, "cpl_solver_create: jacobian_regularization needs nw + m <= 128");
  }
  S->ls_fusable = kkt_wave_size(nw, m);
  S->mu_min = ipm_mu_min(opt.tol);
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
  if ((e = hipHostMalloc(&S->h_flag, 4)) != hipSuccess) return bad(e, "hipHostMalloc");
  // [count, resto, seq, -]: the per-iteration mailbox k_count1 writes (coherent, GPU-mapped)
  if ((e = hipHostMalloc(&S->h_count, 4 * sizeof(int32_t), hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
    return bad(e, "hipHostMalloc");
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
  S->zeros_u8 = a.take<uint8_t>(Bz);
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
  S->fcount = a.take<int64_t>(Bz); S->fc = a.take<int64_t>(Bz); S->n_resto = a.take<int64_t>(Bz);
  S->active = a.take<uint8_t>(Bz); S->lm_cnt = a.take<uint8_t>(Bz); S->lm_skip = a.take<uint8_t>(Bz); S->d_any = a.take<uint8_t>(4);
  S->in_soft = a.take<uint8_t>(Bz); S->tiny_last = a.take<uint8_t>(Bz); S->tiny_flag = a.take<uint8_t>(Bz);
  S->in_resto = a.take<uint8_t>(Bz); S->soft_cnt = a.take<int32_t>(Bz); S->resto_tight = a.take<uint8_t>(Bz);
  S->best_w = a.take<double>(Bz * nw); S->best_f = a.take<double>(Bz); S->fbest = a.take<uint8_t>(Bz);
  S->acc_w = a.take<double>(Bz * nw); S->acc_y = a.take<double>(Bz * m); S->acc_zL = a.take<double>(Bz * nw);
  S->acc_zU = a.take<double>(Bz * nw); S->has_acc = a.take<uint8_t>(Bz);
  // the restoration phase's state
  S->wR = a.take<double>(Bz * nw); S->pR = a.take<double>(Bz * m); S->nR = a.take<double>(Bz * m);
  S->zp = a.take<double>(Bz * m); S->zn = a.take<double>(Bz * m); S->zLR = a.take<double>(Bz * nw);
  S->zUR = a.take<double>(Bz * nw); S->muR = a.take<double>(Bz); S->ftR = a.take<double>(Bz * FMAX);
  S->fpR = a.take<double>(Bz * FMAX); S->fcR = a.take<int64_t>(Bz); S->th_o0 = a.take<double>(Bz);
  S->ph_o0 = a.take<double>(Bz); S->dwlR = a.take<double>(Bz); S->thmaxR = a.take<double>(Bz);
  S->thminR = a.take<double>(Bz);
  // temporaries
  S->A = a.take<double>(Bz * m * nw);
  S->gradw = a.take<double>(Bz * nw); S->c = a.take<double>(Bz * m);
  S->err0 = a.take<double>(Bz); S->base = a.take<double>(Bz); S->mu_o = a.take<double>(Bz);
  S->ft = a.take<double>(Bz * FMAX); S->fp = a.take<double>(Bz * FMAX); S->tau = a.take<double>(Bz);
  S->X = a.take<double>(Bz * n); S->H = a.take<double>(Bz * nf * nf); S->M = a.take<double>(Bz * nw * nw);
  S->Kqd = a.take<double>(Bz * nw * nw); S->r1 = a.take<double>(Bz * nw); S->r2 = a.take<double>(Bz * m);
  S->gphi = a.take<double>(Bz * nw); S->mr_diag = a.take<double>(Bz * nw); S->theta_k = a.take<double>(Bz);
  S->phi_k = a.take<double>(Bz); S->dw = a.take<double>(Bz * nw); S->dy = a.take<double>(Bz * m);
  S->delta_w = a.take<double>(Bz); S->delta_c = a.take<double>(Bz); S->dzL = a.take<double>(Bz * nw);
  S->dzU = a.take<double>(Bz * nw); S->a_max = a.take<double>(Bz); S->a_z = a.take<double>(Bz);
  S->gd = a.take<double>(Bz); S->ws = a.take<double>(Bz * kws);
  S->ws_aug = a.take<double>(S->jreg ? Bz * (size_t)kkt_aug_workspace_doubles(nw, m) : 0); S->info = a.take<int32_t>(Bz);
  S->a_min = a.take<double>(Bz); S->a_soft = a.take<double>(Bz); S->cs_tmp = a.take<double>(Bz * m);
  S->scr1 = a.take<double>(2 * Bz); S->scr2 = a.take<double>(Bz * m);
  S->act = a.take<uint8_t>(Bz); S->switch_ok = a.take<uint8_t>(Bz); S->searching = a.take<uint8_t>(Bz);
  S->st_aug = a.take<uint8_t>(Bz); S->ok = a.take<uint8_t>(Bz); S->soc = a.take<uint8_t>(Bz);
  S->ok_s = a.take<uint8_t>(Bz); S->failed = a.take<uint8_t>(Bz); S->moved = a.take<uint8_t>(Bz);
  S->tiny_now = a.take<uint8_t>(Bz); S->soft_now = a.take<uint8_t>(Bz); S->soft_try = a.take<uint8_t>(Bz);
  S->st_f = a.take<double>(Bz); S->st_g = a.take<double>(Bz * m); S->st_w = a.take<double>(Bz * nw);
  S->st_alpha = a.take<double>(Bz); S->alpha = a.take<double>(Bz);
  S->th = a.take<double>(Bz); S->wt = a.take<double>(Bz * nw); S->Xt = a.take<double>(Bz * n);
  S->f_t = a.take<double>(Bz); S->g_t = a.take<double>(Bz * m);
  S->c_soc = a.take<double>(Bz * m); S->a_soc = a.take<double>(Bz); S->th_old = a.take<double>(Bz);
  S->r2s = a.take<double>(Bz * m); S->dws = a.take<double>(Bz * nw); S->dys = a.take<double>(Bz * m);
  S->ws_ = a.take<double>(Bz * nw); S->Xs = a.take<double>(Bz * n); S->f_s = a.take<double>(Bz);
  S->g_s = a.take<double>(Bz * m); S->th_s = a.take<double>(Bz);
  S->Xn = a.take<double>(Bz * n); S->f_n = a.take<double>(Bz); S->grad_n = a.take<double>(Bz * n);
  S->g_n = a.take<double>(Bz * m); S->J_n = a.take<double>(Bz * nnz_rec);
  S->zeros_w = a.take<double>(Bz * nw); S->zeros_B = a.take<double>(Bz);
  // the restoration phase's temporaries
  S->gfR = a.take<double>(Bz * nw); S->tauR = a.take<double>(Bz); S->rp = a.take<double>(Bz * m);
  S->rn = a.take<double>(Bz * m); S->Dinv = a.take<double>(Bz * m); S->dp = a.take<double>(Bz * m);
  S->dn = a.take<double>(Bz * m); S->dzp = a.take<double>(Bz * m); S->dzn = a.take<double>(Bz * m);
  S->st_p = a.take<double>(Bz * m); S->st_n = a.take<double>(Bz * m); S->thetaR = a.take<double>(Bz);
  S->phiR = a.take<double>(Bz); S->gdR = a.take<double>(Bz); S->a_maxR = a.take<double>(Bz);
  S->a_zR = a.take<double>(Bz); S->a_minR = a.take<double>(Bz); S->alphaR = a.take<double>(Bz);
  S->actR = a.take<uint8_t>(Bz); S->movedR = a.take<uint8_t>(Bz); S->searchingR = a.take<uint8_t>(Bz);
  S->switchR = a.take<uint8_t>(Bz);
  S->fin_f = a.take<double>(Bz); S->fin_g = a.take<double>(Bz * m);
  S->st32 = a.take<int32_t>(Bz); S->it32 = a.take<int32_t>(Bz);
  S->Xp = a.take<double>(nfd * n); S->gL = a.take<double>(nfd * n); S->hfd = a.take<double>(Bz * nf);
  S->mass_fd = a.take<double>(nfd); S->jac_fd = a.take<double>(nfd * nnz); S->grad_fd = a.take<double>(nfd * n);
  S->tag_fd = a.take<uint8_t>(nfd);
  S->orig = a.take<int32_t>(Bz); S->pos = a.take<int32_t>(Bz); S->d_count = a.take<int32_t>(6);
  S->mass_c = a.take<double>(Bz); S->tag_c = a.take<uint8_t>(Bz);
  S->fw = a.take<double>(Bz * nw); S->fy = a.take<double>(Bz * m); S->fX = a.take<double>(Bz * n);
  S->fdinf = a.take<double>(Bz); S->fstatus = a.take<int64_t>(Bz); S->fiters = a.take<int64_t>(Bz);
  S->fresto = a.take<int64_t>(Bz);
  S->scratch = a.take<uint64_t>(Bz * (size_t)S->scratch_words);
  S->df = a.take<double>(Bz); S->dc = a.take<double>(Bz * m); S->ytil = a.take<double>(S->bfgs ? 0 : Bz * m);
  S->rrow = a.take<int32_t>(nnz_rec); S->srp = a.take<int32_t>(m + 1); S->srq = a.take<int32_t>(srq.size());
  S->sc_any = a.take<uint8_t>(4); S->nan_cnt = a.take<int32_t>(Bz);
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
      {S->gu, gu.data(), 8 * (size_t)m}, {S->wl0, wl0.data(), 8 * (size_t)nw}, {S->wu0, wu0.data(), 8 * (size_t)nw},
      {S->rrow, rrow.data(), 4 * rrow.size()}, {S->srp, srp.data(), 4 * srp.size()}, {S->srq, srq.data(), 4 * srq.size()}};
  for (const Up& u : ups)
    if (u.bytes && (e = hipMemcpy(u.dst, u.src, u.bytes, hipMemcpyHostToDevice)) != hipSuccess) return bad(e, "hipMemcpy");
  if ((e = hipMemset(S->zeros_w, 0, 8 * Bz * nw)) != hipSuccess || (e = hipMemset(S->zeros_B, 0, 8 * Bz)) != hipSuccess ||
      (e = hipMemset(S->zeros_u8, 0, Bz)) != hipSuccess)
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
  // per-instance flags of the line search and the restoration phase start cleared
  HK(hipMemsetAsync(S->in_soft, 0, (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->tiny_last, 0, (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->tiny_flag, 0, (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->in_resto, 0, (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->resto_tight, 0, (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->fbest, 0, (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->has_acc, 0, (size_t)B, st), "hipMemsetAsync");
  hipLaunchKernelGGL(k_fill, dim3(blocks_elems(B)), dim3(256), 0, st, B, INFINITY, S->best_f);
  LAUNCHED("k_fill best_f");
  HK(hipMemsetAsync(S->soft_cnt, 0, 4 * (size_t)B, st), "hipMemsetAsync");
  HK(hipMemsetAsync(S->n_resto, 0, 8 * (size_t)B, st), "hipMemsetAsync");
  int64_t evals = 0;
  if (S->fd && (d_mass || d_env_tag)) {
    hipLaunchKernelGGL(k_repeat, dim3(blocks_elems(B * 2 * nf)), dim3(256), 0, st, B, 2 * nf, S->mass, S->mass_fd,
                       S->tag, S->tag_fd);
    LAUNCHED("k_repeat");
  }
  // starting point: x pushed into its bounds, slacks = g_I(x) pushed into theirs, least-squares y
  hipLaunchKernelGGL(k_xbase, dim3(blocks_elems(B * n)), dim3(256), 0, st, B * n, n, d_x0, S->is_fixed, S->xl, S->Xbase);
  LAUNCHED("k_xbase");
  // IPOPT's gradient-based NLP scaling from the callbacks at the starting point (fixed variables at
  // their value); the iteration runs on the scaled problem when any instance has a factor != 1
  // (and the NaN Jacobian entries there: cpl_solver_nan_jacobian)
  S->scaled = false;
  CK(eval_full(S, S->Xbase, S->f, S->grad, S->g, S->J));
  ++evals;
  HK(hipMemsetAsync(S->sc_any, 0, 4, st), "hipMemsetAsync");
  hipLaunchKernelGGL(k_nlp_scaling, dim3(blocks_for(B)), dim3(256), 0, st, B, n, m, S->nnz_rec, S->opt.nlp_scaling,
                     S->is_fixed, S->row_slack, S->srp, S->srq, S->grad, S->J, S->df, S->dc, S->sc_any, S->nan_cnt);
  LAUNCHED("k_nlp_scaling");
  if (S->opt.nlp_scaling) {
    HK(hipMemcpyAsync(S->h_flag, S->sc_any, 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    HK(hipStreamSynchronize(st), "hipStreamSynchronize");
    S->scaled = S->h_flag[0] != 0;
  }
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
  if (S->jreg)
    CK(kkt_aug_solve(0, B, nw, m, S->M, S->A, S->r1, S->r2, S->mu, S->zeros_B, nullptr, S->dw, S->dy, S->delta_w,
                     S->delta_c, S->info, S->ws_aug, st));
  hipLaunchKernelGGL(k_y0, dim3(blocks_for(B)), dim3(256), 0, st, B, m, S->dy, S->info, S->y);
  LAUNCHED("k_y0");
  if (S->bfgs) {  // model initialised to init_val I (IPOPT's limited_memory_init_val = 1)
    hipLaunchKernelGGL(k_lm_init, dim3(blocks_elems(B)), dim3(256), 0, st, B, nf, S->Hq);
    LAUNCHED("k_lm_init");
  }
  const int64_t ev_newton = (S->fd ? 1 : 0) + 1 + S->opt.max_soc;
  int it = 0;
  const int max_iter = S->opt.max_iter;
  const bool compacting = S->opt.compact != 0 && S->opt.use_graph;
  const int64_t min_rows = 256;  // (below it a compaction costs more than its smaller iterations save: profiles/r5/compact_floor)
  int32_t resto_rows = 0;  // instances in the restoration phase after the previous iteration
  // the mailbox's sequence: the device counter restarts with this solve (the previous solve ended
  // with a stream synchronisation, so nothing is still writing the host side)
  int32_t seq = 0;
  ((volatile int32_t*)S->h_count)[2] = 0;
  HK(hipMemsetAsync(S->d_count + 2, 0, 4 * sizeof(int32_t), st), "hipMemsetAsync seq");  // (+ k_tail_small's arrivals)
  while (it < max_iter) {
    if (S->Bcur <= FUSE_ROWS && S->opt.use_graph) {  // one graph, one host round trip
      CK(run_phase(S, resto_rows > 0 ? P_FUSED_R : P_FUSED));
      evals += ev_newton + 2 + (resto_rows > 0 ? (S->fd ? 1 : 0) + 3 : 0);
    } else {
      CK(run_phase(S, P_NEWTON));  // the Newton step and the whole regular line search
      evals += ev_newton;
      CK(read_flags(S));
      if (S->h_flag[1] || S->h_flag[0]) {  // an instance found no acceptable trial: the soft restoration step
        CK(run_phase(S, P_SOFT));
        ++evals;
      }
      const bool may_fail = S->h_flag[1] || S->h_flag[0];
      if (resto_rows > 0) {  // one restoration-phase iteration of the instances inside it
        CK(run_phase(S, P_RNEWTON));
        evals += (S->fd ? 1 : 0) + 3;
      }
      CK(run_phase(S, may_fail ? P_ACCEPT : P_ACCEPT_NR));
      ++evals;
    }
    ++it;
    if (S->Bcur <= COUNT1_MAX) {  // k_count1 delivered the counts to the mailbox
      CK(wait_mail(S, ++seq));
    } else {
      HK(hipMemcpyAsync(S->h_count, S->d_count, 8, hipMemcpyDeviceToHost, st), "hipMemcpyAsync count");
      HK(hipStreamSynchronize(st), "hipStreamSynchronize");
    }
    const int64_t cnt = ((volatile int32_t*)S->h_count)[0];
    resto_rows = ((volatile int32_t*)S->h_count)[1];
    if (cnt == 0) break;
    if (compacting && S->Bcur > min_rows && 2 * cnt <= S->Bcur) {
      // shrink to the smallest halving of the current size that holds the active instances
      int64_t Bn = S->Bcur;
      while (Bn / 2 >= cnt && Bn / 2 >= min_rows) Bn = (Bn + 1) / 2;
      if (Bn < S->Bcur) CK(compact(S, cnt, Bn));
    }
  }
  // final convergence test at the last iterate (the barrier update outputs go to scratch)
  const int64_t Bc = S->Bcur;
  CK(cpl_ipm_dense_a(Bc, m, nw, nf, S->nnz_rec, S->amap, S->row_slack, S->J, S->A, S->active, st));
  hipLaunchKernelGGL(k_prep, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, n, m, nf, nw, S->free32, S->row_slack, S->gl,
                     S->grad, S->g, S->w, S->gradw, S->c);
  LAUNCHED("k_prep");
  CK(ipm_optimality_ex(Bc, nw, m, FMAX, S->nbounds, S->opt.tol, S->opt.acceptable_tol, S->opt.acceptable_iter, S->A,
                       S->gradw, S->c, S->w, S->y, S->zL, S->zU, S->hasL, S->hasU, S->wl0, S->wu0, S->mu, S->filt_t,
                       S->filt_p, S->fcount, S->active, S->status, S->acc, S->d_inf, S->err0, S->base, S->mu_o, S->ft,
                       S->fp, S->fc, MU_ROUNDS, S->mu_min, nullptr, S->in_resto, nullptr, st));
  if (S->opt.fallback_viol_tol > 0.0) {
    hipLaunchKernelGGL(k_fallback, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, m, nw, S->opt.fallback_viol_tol, false,
                       S->orig, S->active, S->status, S->g, S->gl, S->gu, S->best_w, S->best_f, S->w, S->fbest,
                       S->scaled ? S->dc : nullptr);
    LAUNCHED("k_fallback");
  }
  // every row still in the batch to its instance's place in the full-batch results
  hipLaunchKernelGGL(k_scatter_final, dim3(blocks_for(Bc)), dim3(256), 0, st, Bc, n, m, nw, false, S->orig, S->active,
                     S->w, S->y, S->scaled ? S->dc : nullptr, S->df, S->Xbase, S->d_inf, S->status, S->iters, S->n_resto, S->fw, S->fy,
                     S->fX, S->fdinf,
                     S->fstatus, S->fiters, S->fresto);
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
