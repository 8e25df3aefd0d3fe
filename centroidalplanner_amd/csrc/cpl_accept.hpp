// cpl_accept.hpp — IPOPT's filter line-search acceptance test on one wave (FilterLSAcceptor
// [IPOPT]; batch_ipm.py `acceptable` restates it), shared by the solve engine's kernels
// (cpl_ipm.hip's judge, cpl_solver.hip's soft / restoration judges, cpl_kernels.hip's backtracking
// kernel), and the argument block of that backtracking kernel (cpl_kernels.hip ls_backtrack, called
// by cpl_solver.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "cpl_wave.hpp"

namespace cpl {

// gamma_theta, gamma_phi, delta, s_theta, s_phi, eta_phi, obj_max_inc [IPOPT defaults]
constexpr double LS_GAMMA_TH = 1e-5, LS_GAMMA_PHI = 1e-8, LS_DELTA = 1.0, LS_S_TH = 1.1, LS_S_PHI = 2.3;
constexpr double LS_ETA_PHI = 1e-8, LS_OBJ_MAX_INC = 5.0;
constexpr int LS_MAX_SOFT_RESTO = 10;  // max_soft_resto_iters
constexpr double LS_KAPPA_SOC = 0.99;  // kappa_soc

// The accepted step's state commit for instance b on one wave (cpl_ipm_accept_kernel; the solve
// engine's k_resto_enter runs it in its launch): the filter (augmented / reset), y, z with the
// kappa_Sigma safeguard, w, mu and the iteration count.
struct IpmAcceptArgs {
  int nw, m, nfilt;
  const uint8_t *active, *aug, *failed, *rest;
  const double *alpha, *a_z, *theta, *phi, *filt_t_in, *filt_p_in;
  const int64_t* fcount_in;
  const double *w_new, *dy, *dzL, *dzU, *mu;
  const uint8_t *hasL, *hasU;
  const double *wl0, *wu0;
  double *w, *y, *zL, *zU, *mu_state;
  int64_t* iters;
  double *filt_t, *filt_p;
  int64_t* fcount;
};
__device__ __forceinline__ void ipm_accept_one(const IpmAcceptArgs& a, int64_t b, int lane) {
  const int nw = a.nw, m = a.m, nfilt = a.nfilt;
  const bool act = a.active[b] != 0;
  const bool addm = act && a.aug[b];
  const bool fail = a.failed && a.failed[b] != 0;
  const int64_t fc = a.fcount_in[b];
  const int slot = (int)(fc % nfilt);
  const double tk = a.theta[b], pk = a.phi[b];
  for (int k = lane; k < nfilt; k += 64) {
    double ft = a.filt_t_in[b * nfilt + k], fp = a.filt_p_in[b * nfilt + k];
    if (addm && k == slot) {
      ft = (1.0 - 1e-5) * tk;
      fp = pk - 1e-8 * tk;
    }
    if (fail) ft = fp = INFINITY;
    a.filt_t[b * nfilt + k] = ft;
    a.filt_p[b * nfilt + k] = fp;
  }
  const double al = a.alpha[b], az = (a.rest && a.rest[b]) ? 0.0 : a.a_z[b], mub = a.mu[b];
  for (int r = lane; r < m; r += 64)
    if (act) a.y[b * m + r] += al * a.dy[b * m + r];
  for (int k = lane; k < nw; k += 64) {
    const double wn = a.w_new[b * nw + k];
    if (act) {
      if (a.hasL[k]) {
        const double dl = wn - a.wl0[k];
        a.zL[b * nw + k] = fmin(fmax(a.zL[b * nw + k] + az * a.dzL[b * nw + k], mub / (1e10 * dl)), 1e10 * mub / dl);
      }
      if (a.hasU[k]) {
        const double du = a.wu0[k] - wn;
        a.zU[b * nw + k] = fmin(fmax(a.zU[b * nw + k] + az * a.dzU[b * nw + k], mub / (1e10 * du)), 1e10 * mub / du);
      }
      a.w[b * nw + k] = wn;
    }
  }
  if (lane == 0) {
    a.fcount[b] = fail ? 0 : fc + (addm ? 1 : 0);
    a.mu_state[b] = mub;
    if (act) a.iters[b] += 1;
  }
}

// theta_max; the filter (entries stored with their margins ((1 - gamma_theta) theta, phi - gamma_phi
// theta): acceptable when, for every entry, theta or phi is not larger — IPOPT's Filter::Acceptable);
// the switching condition; Armijo on the barrier objective for an f-type step at a reference point
// with theta <= theta_min, else sufficient decrease of theta or phi against the reference point, both
// with IPOPT's round-off tolerance Compare_le(lhs, rhs, base) = lhs - rhs <= 10 eps |base|;
// obj_max_inc.  *h_type: the step augments the filter — IPOPT's UpdateForNextIteration augments
// unless the step is f-type (IsFtype: the switching condition alone, no theta_min term) AND Armijo
// holds.  sw: LS_SW_DESCENT (grad phi . dw < 0) | LS_SW_THETA_MIN (theta_k <= theta_min), the
// post-step kernel's flags.  Every lane of the wave must call it (a ballot).
constexpr uint8_t LS_SW_DESCENT = 1, LS_SW_THETA_MIN = 2;
__device__ __forceinline__ uint8_t ls_switch_flags(double theta, double theta_min, double gd) {
  return (uint8_t)((gd < 0.0 ? LS_SW_DESCENT : 0) | (theta <= theta_min ? LS_SW_THETA_MIN : 0));
}
__device__ __forceinline__ bool ls_acceptable_wave(double th, double ph, double tk, double pk, double g, double al,
                                                   uint8_t sw, double theta_max, const double* ft,
                                                   const double* fp, int nfilt, bool* h_type) {
  const int lane = threadIdx.x & 63;
  bool rejected = false;
  for (int k = lane; k < nfilt; k += 64) rejected |= !((th <= ft[k]) || (ph <= fp[k]));
  const bool in_filter = __ballot(rejected) == 0;
  const bool fin = isfinite(ph) && isfinite(th);
  const bool is_ftype = (sw & LS_SW_DESCENT) && (al * pow(fmax(-g, 0.0), LS_S_PHI) > LS_DELTA * pow(tk, LS_S_TH));
  const bool ftype = is_ftype && (sw & LS_SW_THETA_MIN);
  const double ro_p = 10.0 * DBL_EPSILON * fabs(pk), ro_t = 10.0 * DBL_EPSILON * fabs(tk);
  bool armijo = (ph - pk) - LS_ETA_PHI * al * g <= ro_p;
  bool suff = (th - (1.0 - LS_GAMMA_TH) * tk <= ro_t) || ((ph - pk) - (-LS_GAMMA_PHI * tk) <= ro_p);
  if (ph > pk) {  // IsAcceptableToCurrentIterate: no jump of more than obj_max_inc orders of magnitude
    const double basval = fabs(pk) > 10.0 ? log10(fabs(pk)) : 1.0;
    if (log10(ph - pk) > LS_OBJ_MAX_INC + basval) armijo = suff = false;
  }
  if (h_type) *h_type = !(is_ftype && armijo);
  return fin && th <= theta_max && in_filter && (ftype ? armijo : suff);
}

// The line search's per-instance setup after the Newton step (ls_setup_wave below)
struct LsSetupArgs {
  int32_t m;
  const uint8_t* act;
  const double *w, *dw, *dy, *c, *f, *g, *theta_k, *theta_min;
  uint8_t* in_soft;
  int32_t* soft_cnt;
  uint8_t *tiny_last, *tiny_flag, *tiny_now, *soft_now;
  double* a_min;
  uint8_t* searching;
  double *st_f, *st_g, *st_w, *st_alpha;
  uint8_t* st_aug;
  double* alpha;
  uint8_t* any;
};

// The post-step quantities (cpl_ipm.hip's post-step kernel; the fused line-search kernel runs it as
// its prologue: ipm_post_step_one below)
struct PostStepArgs {
  int32_t nw;
  const double *w, *dw, *zL, *zU, *gphi, *mu, *tau;
  const uint8_t *hasL, *hasU;
  const double *wl0, *wu0, *theta, *theta_min;
  const uint8_t* active;
  const double* delta_w;
  double *dwl, *dzL, *dzU, *a_max, *a_z, *gd_out;
  uint8_t* switch_ok;
};

// The rest of the regular backtracking line search of every instance still searching after its
// first trial (and that trial's second-order corrections), in one launch: trials at alpha, alpha / 2,
// ... until one is acceptable, alpha falls to alpha_min, or max_trials more trials were made
// (batch_ipm.py regular_step, trials ls = 1 .. max_ls - 1).  Device pointers, rows of the batch.
struct LsBacktrackArgs {
  int64_t batch;
  int32_t n, m, nf, nw, nfilt, max_trials;
  const uint8_t* act;         // the instance iterates this iteration (active, not in restoration)
  const uint8_t* tiny;        // tiny step this iteration (no line search)
  const uint8_t* soft_now;    // in the soft restoration phase this iteration
  const int32_t* soft_cnt;
  uint8_t* searching;         // in/out
  double* alpha;              // in/out: the next trial's step
  const double* a_min;
  const double* w;            // [batch, nw] the iterate
  const double* dw;           // [batch, nw] the Newton step
  const double* Xbase;        // [batch, n] fixed variables
  const int32_t* freepos;     // [n] position in w of each variable, -1 fixed
  const int32_t* row_slack;   // [m] slack of each inequality row, -1 equality
  const double* gl;
  const uint8_t* hasL;
  const uint8_t* hasU;
  const double* wl0;
  const double* wu0;
  const double* mu;
  const double* theta_k;
  const double* phi_k;
  const double* gd;
  const uint8_t* switch_ok;
  const double* theta_max;
  const double* filt_t;       // [batch, nfilt] the filter (after this iteration's barrier update)
  const double* filt_p;
  const double* mass;         // [batch] or NULL
  const uint8_t* env_tag;     // [batch] (mixed batches) or NULL
  double* st_f;               // the accepted trial: f, g, w, alpha, filter-augmenting
  double* st_g;
  double* st_w;
  double* st_alpha;
  uint8_t* st_aug;
  uint8_t* any;               // any[0] |= still searching (trials exhausted), any[1] |= soft candidate
  // restoration-phase search (resto != 0; batch_ipm.py resto_step): the trial also moves p, n along
  // dp, dn; theta = sum |c(w_t) - p_t + n_t|, phi = rho sum(p_t + n_t) + eta/2 |D_R (x_t - x_R)|^2 -
  // mu_R (sum log slacks + sum log p_t n_t); the flag is any[2]; no soft restoration
  int32_t resto;
  double rho;
  const double* pR;
  const double* nR;
  const double* dp;
  const double* dn;
  const double* wR;
  double* st_p;
  double* st_n;
  // first != 0 (regular search; systems the one-wave KKT kernel factorises): the kernel also makes
  // the first trial at alpha (alpha_max) and its up to max_soc second-order corrections (batch_ipm.py
  // regular_step, IPOPT's TrySecondOrderCorrection), re-solving with the factors the iteration's
  // factorisation kept (kkt_ws), before it backtracks — one launch for the whole search
  int32_t first;
  int32_t max_soc;
  const double* c;            // [batch, m] c(w) at the iterate
  const double* M;            // [batch, nw, nw] the Newton system's M
  const double* r1;           // [batch, nw] its first right-hand side
  const double* kkt_ws;       // cpl_kkt_solve's factor workspace (mode 0 of this iteration)
  const double* tau;          // [batch] fraction-to-the-boundary parameter
  // soft_ws != NULL (the small-batch iteration, P_FUSED): the kernel's tail also starts IPOPT's soft
  // restoration step (the solver's k_soft_begin, which would be the next launch): soft_try = no
  // accepted trial (or in the soft phase within its budget), a_soft = min(alpha_max, alpha_z), the
  // point soft_ws = w + a_soft dw on those instances (= w elsewhere) and its X = unpack(soft_ws)
  const double* a_max;
  const double* a_z;
  double* soft_ws;
  double* soft_X;
  uint8_t* soft_try;
  double* a_soft;
  // (FIRST) the post-step quantities and the search's setup of every instance, computed in the
  // kernel's prologue (with_post) instead of a launch of their own
  PostStepArgs post;
  LsSetupArgs setup;
  int32_t with_post;
  // IPOPT's NLP scaling (cpl_solve_options.nlp_scaling): the trial's f times df[b], its g times
  // dc[b, r] (the scaled problem's values, as the solver's k_apply_scaling); nullptr: unscaled
  const double* df = nullptr;
  const double* dc = nullptr;
  // IPOPT's Jacobian regularisation (cpl_solve_options.jacobian_regularization): a system whose
  // factorisation marked it rank deficient (aug_dc[b] != 0) re-solves its corrections with the augmented
  // factors cpl_kkt_aug_kernel kept in aug_ws (cpl_kkt_block.hpp kkt_aug_resolve_wave); nullptr: off
  const double* aug_dc = nullptr;
  double* aug_ws = nullptr;
  // which instances this launch searches (set by ls_backtrack): 0 all; 1 the unmarked (aug_dc == 0),
  // 2 the marked — large batches run the two in separate instantiations (the default one keeps its
  // occupancy), small ones all in the AUGR one
  int32_t aug_sel = 0;
};

// s + sum_{r < m} a[r * stride] * v[r], accumulated in r order exactly as the plain loop
// (s += a v: the same roundings), with the loads issued eight at a time: the plain loop's load ->
// multiply -> add chain waited one L2 round trip per row (a one-wave-per-instance kernel at small
// batch sizes is that chain)
__device__ __forceinline__ double seq_dot_acc(double s, const double* __restrict__ a, int stride,
                                              const double* __restrict__ v, int m) {
  int r = 0;
  for (; r + 8 <= m; r += 8) {
    double av[8], vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      av[u] = a[(r + u) * stride];
      vv[u] = v[r + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += av[u] * vv[u];
  }
  for (; r < m; ++r) s += a[r * stride] * v[r];
  return s;
}

// IPOPT FilterLSAcceptor::CalculateAlphaMin (alpha_min_frac 0.05)
constexpr double LS_ALPHA_MIN_FRAC = 0.05;
__device__ __forceinline__ double ls_alpha_min_of(double theta, double gd, double theta_min) {
  if (!(gd < 0.0)) return LS_ALPHA_MIN_FRAC * LS_GAMMA_TH;
  double a = fmin(LS_GAMMA_TH, LS_GAMMA_PHI * theta / -gd);
  if (theta <= theta_min) a = fmin(a, LS_DELTA * pow(theta, LS_S_TH) / pow(-gd, LS_S_PHI));
  return LS_ALPHA_MIN_FRAC * a;
}

// IPOPT's tiny-step test tolerances (tiny_step_tol, tiny_step_y_tol)
constexpr double LS_TINY_STEP_TOL = 10.0 * DBL_EPSILON, LS_TINY_STEP_Y_TOL = 1e-2;

__device__ __forceinline__ double ls_xor_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

// After the Newton step (batch_ipm.py regular_step): IPOPT's tiny-step test (every primal component
// below 10 eps relative, the multiplier step below 1e-2, the point feasible to 1e-4; two in a row
// force the next barrier decrease), the soft restoration phase's counter, alpha_min, and the line
// search state (searching unless tiny or in the soft phase; a tiny step is taken whole: alpha_max).
// One wave per instance, at the end of cpl_ipm.hip's post-step kernel (am = alpha_max and gd = the
// directional derivative it has just computed).
__device__ __forceinline__ void ls_setup_wave(int64_t b, int nw, const LsSetupArgs& L, double am, double gd) {
  const int m = L.m;
  const int lane = threadIdx.x & 63;
  const bool a = L.act[b] != 0;
  double rel = 0.0, dym = 0.0, cin = 0.0;
  for (int k = lane; k < nw; k += 64) rel = fmax(rel, fabs(L.dw[b * nw + k]) / (1.0 + fabs(L.w[b * nw + k])));
  for (int r = lane; r < m; r += 64) {
    dym = fmax(dym, fabs(L.dy[b * m + r]));
    cin = fmax(cin, fabs(L.c[b * m + r]));
  }
  rel = ls_xor_max(rel);
  dym = ls_xor_max(dym);
  cin = ls_xor_max(cin);
  const bool tiny = a && rel < LS_TINY_STEP_TOL && dym < LS_TINY_STEP_Y_TOL && cin < 1e-4;
  const bool sn = a && L.in_soft[b] && !tiny;
  for (int r = lane; r < m; r += 64) L.st_g[b * m + r] = L.g[b * m + r];
  for (int k = lane; k < nw; k += 64)
    L.st_w[b * nw + k] = tiny ? L.w[b * nw + k] + am * L.dw[b * nw + k] : L.w[b * nw + k];
  if (lane == 0) {
    if (b == 0 && L.any) L.any[0] = L.any[1] = 0;
    if (a) {
      const bool tl = L.tiny_last[b] != 0;
      L.tiny_flag[b] = (tiny && tl) ? 1 : 0;
      L.tiny_last[b] = (tiny && !tl) ? 1 : 0;
    }
    L.tiny_now[b] = tiny ? 1 : 0;
    L.soft_now[b] = sn ? 1 : 0;
    if (sn) L.soft_cnt[b] += 1;
    L.a_min[b] = ls_alpha_min_of(L.theta_k[b], gd, L.theta_min[b]);
    L.searching[b] = (a && !tiny && !sn) ? 1 : 0;
    L.st_f[b] = L.f[b];
    L.st_alpha[b] = tiny ? am : 0.0;
    L.st_aug[b] = 0;
    L.alpha[b] = am;
  }
}

// After the Newton step (batch_ipm.py step): bound-multiplier steps dzL = mu/dl - zL - zL/dl dw,
// dzU = mu/du - zU + zU/du dw, their fraction-to-the-boundary step a_z, the primal one a_max,
// gd = grad_phi . dw, switch_ok = ls_switch_flags (gd < 0, theta <= theta_min), and delta_w_last <-
// delta_w on the active instances; then (ls.act != NULL) the line search's setup.  One wave, instance b.
__device__ __forceinline__ void ipm_post_step_one(const PostStepArgs& P, int64_t b, const LsSetupArgs& ls) {
  const int nw = P.nw;
  const int lane = threadIdx.x & 63;
  const double mub = P.mu[b], t = P.tau[b];
  double rp = INFINITY, rz = INFINITY, gd = 0.0;
  for (int k = lane; k < nw; k += 64) {
    const double wk = P.w[b * nw + k], dk = P.dw[b * nw + k];
    gd += P.gphi[b * nw + k] * dk;
    double dzl = 0.0, dzu = 0.0;
    if (P.hasL[k]) {
      const double dl = wk - P.wl0[k], zl = P.zL[b * nw + k];
      dzl = mub / dl - zl - zl / dl * dk;
      if (dk < 0.0) rp = fmin(rp, -t * dl / dk);
      if (dzl < 0.0) rz = fmin(rz, -t * zl / dzl);
    }
    if (P.hasU[k]) {
      const double du = P.wu0[k] - wk, zu = P.zU[b * nw + k];
      dzu = mub / du - zu + zu / du * dk;
      if (dk > 0.0) rp = fmin(rp, -t * du / -dk);
      if (dzu < 0.0) rz = fmin(rz, -t * zu / dzu);
    }
    P.dzL[b * nw + k] = dzl;
    P.dzU[b * nw + k] = dzu;
  }
  rp = wave_min(rp);
  rz = wave_min(rz);
  gd = wave_sum(gd);
  if (lane == 0) {
    P.a_max[b] = fmin(rp, 1.0);
    P.a_z[b] = fmin(rz, 1.0);
    P.gd_out[b] = gd;
    P.switch_ok[b] = ls_switch_flags(P.theta[b], P.theta_min[b], gd);
    if (P.active[b]) P.dwl[b] = P.delta_w[b];
  }
  // the line-search setup: no output above is among its inputs except alpha_max and gd (registers)
  if (ls.act) ls_setup_wave(b, nw, ls, fmin(rp, 1.0), gd);
}

// The solve loop's per-iteration unpack after the optimality test, fused into that kernel's tail
// (cpl_ipm.hip; was a launch of its own): X = unpack(w) (free columns from w, fixed ones from
// Xbase), tau = max(0.99, 1 - mu) and the iteration's snapshot act = active && !in_resto.
struct IpmUnpack {
  int32_t n;
  const int32_t* freepos;
  const double* Xbase;
  const uint8_t* in_resto;
  double* X;
  double* tau;
  uint8_t* act;
  // IPOPT's backup acceptable point (BacktrackingLineSearch::StoreAcceptablePoint): a regular
  // iterate at the acceptable level is copied here (acc_w == NULL: not kept)
  double* acc_w;
  double* acc_y;
  double* acc_zL;
  double* acc_zU;
  uint8_t* has_acc;
  uint8_t* any_reset;  // (the solve loop's fused search) flags to clear, or NULL
  // IPOPT's BacktrackingLineSearch::Reset on a barrier change (MonotoneMuUpdate): the soft restoration
  // phase ends (in_soft cleared where mu changed; NULL: not kept)
  uint8_t* in_soft;
};

// one entry e of A = dc/dw = [J_free | -P] (batch-major [B][m][nw]) from the CSR Jacobian values:
// amap[r * nf + k] = CSR position of (row r, free column k), -1 (structural zero) or -2 (a
// structural 1 the folded layout skips); NaN -> 0 (a cone at zero tangential force); the slack
// block is -1 at (r, nf + row_slack[r]).  Shared by cpl_ipm_dense_a and the solver's fused launch.
__device__ __forceinline__ void dense_a_entry(int64_t e, int m, int nw, int nf, int nnz,
                                              const int32_t* __restrict__ amap,
                                              const int32_t* __restrict__ row_slack,
                                              const double* __restrict__ jac, double* __restrict__ A,
                                              const uint8_t* __restrict__ active) {
  const int per = m * nw;
  const int64_t b = e / per;
  if (active && !active[b]) return;
  const int rc = (int)(e - b * per);
  const int r = rc / nw, k = rc - r * nw;
  double v = 0.0;
  if (k < nf) {
    const int q = amap[r * nf + k];
    if (q >= 0) {
      v = jac[b * nnz + q];
      v = v == v ? v : 0.0;
    } else if (q == -2) {
      v = 1.0;
    }
  } else if (row_slack[r] == k - nf) {
    v = -1.0;
  }
  A[e] = v;
}

}  // namespace cpl
