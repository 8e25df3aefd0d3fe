// cpl_ipm.hip — fused per-instance vector work of the solve loop's filter line search
// (centroidalplanner_amd/batch_ipm.py): the trial point and the acceptance test of IPOPT's filter
// line search (Waechter & Biegler 2006, §2.3-2.4) for every instance in one launch each, instead of
// ~50 elementwise tensor launches per trial.  One wave per instance: lanes run over the instance's
// primal-slack vector (nw <= 128) and constraint rows, sums by xor shuffles.  Every quantity is
// float64; the decisions are the ones batch_ipm.py's host (torch) path takes, with sums reduced in
// a different order (last-bit differences only).
#include <hip/hip_runtime.h>

#include <cfloat>

#include <cmath>
#include <cstdint>
#include <string>

#include "cpl_status.hpp"
#include "cpl_accept.hpp"
#include "cpl_wave.hpp"

namespace cpl {

constexpr int IPM_WAVES = 4;  // instances per 256-thread workgroup
constexpr int IPM_MU_ROUNDS = 6;  // barrier decreases per iteration (0.1 -> the floor at tol 1e-8 takes 6)

__device__ __forceinline__ double ipm_wave_sum(double v) { return wave_sum(v); }

// wt = w + alpha d;  X[b, free[k]] = (mask ? wt : w_keep)[k],  X[b, fixed[j]] = Xbase[b, fixed[j]]
__global__ __launch_bounds__(256) void cpl_ipm_trial_point_kernel(
    int64_t batch, int n, int nf, int nw, const int64_t* __restrict__ free_idx, const int64_t* __restrict__ fixed_idx,
    const double* __restrict__ Xbase, const double* __restrict__ w, const double* __restrict__ d,
    const double* __restrict__ alpha, const uint8_t* __restrict__ mask, const double* __restrict__ w_keep,
    double* __restrict__ wt, double* __restrict__ X) {
  const int64_t b = (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch) return;
  const int lane = threadIdx.x & 63;
  const double a = alpha[b];
  const bool m = mask[b] != 0;
  for (int k = lane; k < nw; k += 64) {
    const double v = w[b * nw + k] + a * d[b * nw + k];
    wt[b * nw + k] = v;
    if (k < nf) X[b * n + free_idx[k]] = m ? v : w_keep[b * nw + k];
  }
  for (int j = lane; j < n - nf; j += 64) X[b * n + fixed_idx[j]] = Xbase[b * n + fixed_idx[j]];
}

// IPOPT's acceptance test of one trial point per instance, and the take() of batch_ipm.py:
//   theta = sum |c(w_t)|, phi = f_t - mu (sum log(w_t - wl) + sum log(wu - w_t)),
//   ok = finite & theta <= theta_max & filter-acceptable & (f-type ? Armijo : sufficient decrease)
// for instances with searching & (extra_mask or 1); accepted ones copy (f, g, w_t, alpha, aug) into
// the line-search state and stop searching.  th_out / ok_out: theta and ok of every instance.
__global__ __launch_bounds__(256) void cpl_ipm_judge_take_kernel(
    int64_t batch, int nw, int m, int nf, int nfilt, const int32_t* __restrict__ row_slack,
    const double* __restrict__ gl, const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU,
    const double* __restrict__ wl0, const double* __restrict__ wu0, const double* __restrict__ wt,
    const double* __restrict__ f_t, const double* __restrict__ g_t, const double* __restrict__ alpha,
    const double* __restrict__ mu, const double* __restrict__ theta_k, const double* __restrict__ phi_k,
    const double* __restrict__ gd, const uint8_t* __restrict__ switch_ok, const double* __restrict__ theta_max,
    const double* __restrict__ filt_t, const double* __restrict__ filt_p, const uint8_t* __restrict__ extra_mask,
    uint8_t* __restrict__ searching, double* __restrict__ st_f, double* __restrict__ st_g, double* __restrict__ st_w,
    double* __restrict__ st_alpha, uint8_t* __restrict__ st_aug, double* __restrict__ th_out,
    uint8_t* __restrict__ ok_out, int mode) {
  const int64_t b = (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch) return;
  const int lane = threadIdx.x & 63;
  const double* wb = wt + b * nw;
  const double* gb = g_t + b * m;
  double th = 0.0;
  for (int r = lane; r < m; r += 64) {
    const int s = row_slack[r];
    th += fabs(s < 0 ? gb[r] - gl[r] : gb[r] - wb[nf + s]);
  }
  double lg = 0.0;
  for (int k = lane; k < nw; k += 64) {
    if (hasL[k]) lg += log(wb[k] - wl0[k]);
    if (hasU[k]) lg += log(wu0[k] - wb[k]);
  }
  th = ipm_wave_sum(th);
  lg = ipm_wave_sum(lg);
  const double ph = f_t[b] - mu[b] * lg;
  const double al = alpha[b];
  bool aug = false;
  const bool ok = ls_acceptable_wave(th, ph, theta_k[b], phi_k[b], gd[b], al, switch_ok[b], theta_max[b],
                                     filt_t + b * nfilt, filt_p + b * nfilt, nfilt, &aug);
  const bool take = ok && searching[b] && (extra_mask == nullptr || extra_mask[b]);
  if (take) {
    for (int r = lane; r < m; r += 64) st_g[b * m + r] = gb[r];
    for (int k = lane; k < nw; k += 64) st_w[b * nw + k] = wb[k];
  }
  if (lane == 0) {
    th_out[b] = th;
    ok_out[b] = ok ? 1 : 0;
    if (take) {
      st_f[b] = f_t[b];
      st_alpha[b] = al;
      st_aug[b] = aug ? 1 : 0;
      searching[b] = 0;
    }
  }
}

// IPOPT's scaled optimality error at the current iterate (s_max = 100), the convergence test and
// the monotone barrier update of one iteration (batch_ipm.py errors / check / err_mu):
//   dual = grad_w + A^T y - zL + zU,  comp = (w - wl) zL, (wu - w) zU,
//   err0 = max(|dual|max / s_d, |c|max, comp_max / s_c)  -> optimal (tol) / acceptable (tol_acc for
//   acc_iter consecutive iterations) / still active;
//   two rounds of mu <- max(min(0.2 mu, mu^1.5), tol/10) while err_mu <= 10 mu and mu > tol/10, each
//   resetting the instance's filter.  Writes status/acc/active/d_inf in place; mu, filter -> *_out.
__global__ __launch_bounds__(256) void cpl_ipm_optimality_kernel(
    int64_t batch, int nw, int m, int nfilt, int nbounds, double tol, double acc_tol, int acc_iter,
    const double* __restrict__ A, const double* __restrict__ gw, const double* __restrict__ c,
    const double* __restrict__ w, const double* __restrict__ y, const double* __restrict__ zL,
    const double* __restrict__ zU, const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU,
    const double* __restrict__ wl0, const double* __restrict__ wu0, const double* __restrict__ mu_in,
    const double* __restrict__ filt_t, const double* __restrict__ filt_p, const int64_t* __restrict__ fcount,
    uint8_t* __restrict__ active, int64_t* __restrict__ status, int64_t* __restrict__ acc,
    double* __restrict__ d_inf_out, double* __restrict__ err0_out, double* __restrict__ base_out,
    double* __restrict__ mu_out, double* __restrict__ filt_t_out, double* __restrict__ filt_p_out,
    int64_t* __restrict__ fcount_out, int mu_rounds, double mu_min, const uint8_t* __restrict__ tiny_flag,
    const uint8_t* __restrict__ skip, const IpmUnpack up) {
  const int64_t b = (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch) return;
  const int lane = threadIdx.x & 63;
  // (the fused line search's flags cleared here, one launch before the search sets them)
  if (b == 0 && lane == 0 && up.any_reset) up.any_reset[0] = up.any_reset[1] = 0;
  // the solve loop's unpack (IpmUnpack) at the iteration's barrier parameter and active flag
  auto unpack = [&](double mu_v, bool act_v) {
    if (!up.X) return;
    for (int j = lane; j < up.n; j += 64) {
      const int k = up.freepos[j];
      up.X[b * up.n + j] = k >= 0 ? w[b * nw + k] : up.Xbase[b * up.n + j];
    }
    if (lane == 0) {
      up.tau[b] = fmax(1.0 - mu_v, 0.99);
      up.act[b] = act_v && !up.in_resto[b];
    }
  };
  if (skip && skip[b]) {  // (an instance in the restoration phase: its own test and barrier update)
    for (int k = lane; k < nfilt; k += 64) {
      filt_t_out[b * nfilt + k] = filt_t[b * nfilt + k];
      filt_p_out[b * nfilt + k] = filt_p[b * nfilt + k];
    }
    if (lane == 0) {
      mu_out[b] = mu_in[b];
      fcount_out[b] = fcount[b];
    }
    unpack(mu_in[b], active[b] != 0);
    return;
  }
  const double* Ab = A + b * (int64_t)m * nw;
  const double* yb = y + b * m;
  // lanes own w entries k = lane, lane + 64 (nw <= 128)
  double cl[2] = {0.0, 0.0}, cu[2] = {0.0, 0.0};
  double dmax = 0.0, zs = 0.0, clmax = 0.0, cumax = 0.0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = lane + 64 * h;
    if (k < nw) {
      double dual = gw[b * nw + k];
      dual = seq_dot_acc(dual, Ab + k, nw, yb, m);
      const double zl = zL[b * nw + k], zu = zU[b * nw + k], wk = w[b * nw + k];
      dual = dual - zl + zu;
      dmax = fmax(dmax, fabs(dual));
      zs += fabs(zl) + fabs(zu);
      cl[h] = hasL[k] ? (wk - wl0[k]) * zl : 0.0;
      cu[h] = hasU[k] ? (wu0[k] - wk) * zu : 0.0;
      clmax = fmax(clmax, cl[h]);
      cumax = fmax(cumax, cu[h]);
    }
  }
  double ys = 0.0, cmax = 0.0;
  for (int r = lane; r < m; r += 64) {
    ys += fabs(yb[r]);
    cmax = fmax(cmax, fabs(c[b * m + r]));
  }
  // wave reductions (DPP, cpl_wave.hpp; all lanes end with the totals)
  dmax = wave_max(dmax);
  clmax = wave_max(clmax);
  cumax = wave_max(cumax);
  cmax = wave_max(cmax);
  zs = ipm_wave_sum(zs);
  ys = ipm_wave_sum(ys);
  const double s_max = 100.0;
  const double sd = fmax((ys + zs) / (double)max(m + nbounds, 1), s_max) / s_max;
  const double sc = fmax(zs / (double)max(nbounds, 1), s_max) / s_max;
  const double base = fmax(dmax / sd, cmax);
  const double err0 = fmax(base, fmax(clmax, cumax) / sc);
  // convergence test
  bool act = active[b] != 0;
  const bool done_now = act && err0 <= tol;
  const int64_t acc_new = (act && err0 <= acc_tol) ? acc[b] + 1 : 0;
  const bool acc_now = act && !done_now && acc_new >= acc_iter;
  act = act && !done_now && !acc_now;
  if (up.acc_w && act && err0 <= acc_tol) {  // the backup acceptable point (CurrentIsAcceptable)
    for (int k = lane; k < nw; k += 64) {
      up.acc_w[b * nw + k] = w[b * nw + k];
      up.acc_zL[b * nw + k] = zL[b * nw + k];
      up.acc_zU[b * nw + k] = zU[b * nw + k];
    }
    for (int r = lane; r < m; r += 64) up.acc_y[b * m + r] = yb[r];
    if (lane == 0) up.has_acc[b] = 1;
  }
  // barrier update (IPOPT MonotoneMuUpdate, mu_allow_fast_monotone_decrease): while the barrier
  // problem is solved to kappa_eps mu (or once after two tiny steps), at most mu_rounds times
  double mu = mu_in[b];
  bool reset = false;
  const bool force = tiny_flag && tiny_flag[b];
  for (int round = 0; round < mu_rounds; ++round) {
    double em = 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = lane + 64 * h;
      if (k < nw) {
        em = fmax(em, fabs(cl[h] - (hasL[k] ? mu : 0.0)));
        em = fmax(em, fabs(cu[h] - (hasU[k] ? mu : 0.0)));
      }
    }
    em = wave_max(em);
    const double err_mu = fmax(base, em / sc);
    if (act && (err_mu <= 10.0 * mu || (force && round == 0)) && mu > mu_min) {
      mu = fmax(fmin(0.2 * mu, pow(mu, 1.5)), mu_min);
      reset = true;
    }
  }
  for (int k = lane; k < nfilt; k += 64) {
    filt_t_out[b * nfilt + k] = reset ? INFINITY : filt_t[b * nfilt + k];
    filt_p_out[b * nfilt + k] = reset ? INFINITY : filt_p[b * nfilt + k];
  }
  if (lane == 0) {
    acc[b] = acc_new;
    if (done_now) status[b] = 0;
    else if (acc_now) status[b] = 1;
    active[b] = act ? 1 : 0;
    d_inf_out[b] = dmax;
    err0_out[b] = err0;
    base_out[b] = base;
    mu_out[b] = mu;
    fcount_out[b] = reset ? 0 : fcount[b];
    if (reset && up.in_soft) up.in_soft[b] = 0;  // (the line search's Reset: the soft restoration phase ends)
  }
  unpack(mu, act);
}

// Fraction-to-the-boundary step (batch_ipm.py max_step, both sides): the largest alpha <= 1 with
//   primal (v2 == NULL): -tau (v - lo) / d over hasL & d < 0 and
//                        -tau (up - v) / -d over hasU & d > 0;
//   dual (v2 != NULL):   multipliers zL = v (hasL), zU = v2 (hasU) kept >= 0: -tau v / d over
//                        hasL & d < 0 and -tau v2 / d2 over hasU & d2 < 0.
__global__ __launch_bounds__(256) void cpl_ipm_max_step_kernel(int64_t batch, int nw, const double* __restrict__ v,
                                                               const double* __restrict__ d,
                                                               const double* __restrict__ v2,
                                                               const double* __restrict__ d2,
                                                               const uint8_t* __restrict__ hasL,
                                                               const uint8_t* __restrict__ hasU,
                                                               const double* __restrict__ lo,
                                                               const double* __restrict__ up,
                                                               const double* __restrict__ tau,
                                                               double* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch) return;
  const int lane = threadIdx.x & 63;
  const double t = tau[b];
  double r = INFINITY;
  for (int k = lane; k < nw; k += 64) {
    const double vk = v[b * nw + k], dk = d[b * nw + k];
    if (v2 == nullptr) {
      if (hasL[k] && dk < 0.0) r = fmin(r, -t * (vk - lo[k]) / dk);
      if (hasU[k] && dk > 0.0) r = fmin(r, -t * (up[k] - vk) / -dk);
    } else {
      if (hasL[k] && dk < 0.0) r = fmin(r, -t * vk / dk);
      const double v2k = v2[b * nw + k], d2k = d2[b * nw + k];
      if (hasU[k] && d2k < 0.0) r = fmin(r, -t * v2k / d2k);
    }
  }
  r = wave_min(r);
  if (lane == 0) out[b] = fmin(r, 1.0);
}

// The Newton system's right-hand side and matrix (batch_ipm.py step, "setup"):
//   Sigma = zL/(w - wl) + zU/(wu - w), grad_phi = grad_w - mu/(w - wl) + mu/(wu - w),
//   r1 = -(grad_phi + A^T y), r2 = -c, M = diag(Sigma) + [H 0; 0 0] (H: nf x nf, may be NULL),
//   theta = sum |c|, phi = f - mu (sum log(w - wl) + sum log(wu - w)),
//   Mr_diag = Sigma + sqrt(mu) / max(1, |w|)^2 (the feasibility step's diagonal).
// LM: the Hessian block comes as the compact limited-memory model of the native engine's k_lbfgs
// (per instance [sigma, nv, U (lm_pairs x nf), W (lm_pairs x nf)]): H = sigma I + sum_{i < nv}
// (-u_i u_i' + w_i w_i'), each entry evaluated here in the order the dense build used, staged per wave
// in dynamic LDS — the dense nf x nf model never goes through memory.
// WIDE (small batches): one instance per workgroup — wave 0 does the per-variable and per-row work
// exactly as the one-wave form, the M entries are spread over the four waves (every entry the same
// operations in the same order: bitwise the one-wave result); at B = 1 one wave filled 47 x 47
// entries alone.
constexpr int LM_REG_PAIRS = 8;  // the column build's largest limited-memory history
template <bool LM, bool WIDE = false>
__global__ __launch_bounds__(256) void cpl_ipm_newton_setup_kernel(
    int64_t batch, int nw, int m, int nf, const double* __restrict__ w, const double* __restrict__ zL,
    const double* __restrict__ zU, const double* __restrict__ gw, const double* __restrict__ A,
    const double* __restrict__ y, const double* __restrict__ c, const double* __restrict__ f,
    const double* __restrict__ mu, const uint8_t* __restrict__ hasL, const uint8_t* __restrict__ hasU,
    const double* __restrict__ wl0, const double* __restrict__ wu0, const double* __restrict__ H, int h_sym,
    double* __restrict__ M, double* __restrict__ r1, double* __restrict__ r2, double* __restrict__ gphi,
    double* __restrict__ mr_diag, double* __restrict__ theta, double* __restrict__ phi,
    const uint8_t* __restrict__ active, const double* __restrict__ Hc, int lm_pairs) {
  const int64_t b = WIDE ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch || (active && !active[b])) return;  // converged: its Newton system is never read
  const int lane = threadIdx.x & 63;
  const bool w0 = !WIDE || threadIdx.x < 64;  // the wave doing the per-variable / per-row work
  const int et = WIDE ? (int)threadIdx.x : lane, es = WIDE ? 256 : 64;  // the M entries' thread / stride
  const double mub = mu[b];
  const double* Ab = A + b * (int64_t)m * nw;
  const double* yb = y + b * m;
  double* Mb = M + b * (int64_t)nw * nw;
  __shared__ double sig_s[IPM_WAVES][128];
  double* sg = sig_s[WIDE ? 0 : threadIdx.x >> 6];
  double lg = 0.0;
  for (int k = lane; w0 && k < nw; k += 64) {
    const double wk = w[b * nw + k];
    double sig = 0.0, gp = gw[b * nw + k];
    if (hasL[k]) {
      const double dl = wk - wl0[k];
      sig += zL[b * nw + k] / dl;
      gp -= mub / dl;
      lg += log(dl);
    }
    if (hasU[k]) {
      const double du = wu0[k] - wk;
      sig += zU[b * nw + k] / du;
      gp += mub / du;
      lg += log(du);
    }
    double aty = 0.0;
    aty = seq_dot_acc(aty, Ab + k, nw, yb, m);
    gphi[b * nw + k] = gp;
    r1[b * nw + k] = -(gp + aty);
    const double aw = fmax(fabs(wk), 1.0);
    mr_diag[b * nw + k] = sig + sqrt(mub) / (aw * aw);
    sg[k] = sig;
  }
  // M = diag(Sigma) + [H 0; 0 0], written row by row with the lanes along the row (coalesced);
  // the wave's own LDS row of Sigma needs no workgroup barrier, only the wave's LDS ordering
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores have landed
  __builtin_amdgcn_wave_barrier();
  if (WIDE) __syncthreads();  // Sigma from wave 0 to every wave
  if (LM) {
    extern __shared__ __align__(16) double lm_dyn[];
    const int per = 2 * lm_pairs * nf;
    double* UW = lm_dyn + (WIDE ? 0 : (threadIdx.x >> 6) * per);  // this wave's (workgroup's) U | W
    const double* hc = Hc + b * (int64_t)(2 + per);
    const double sigma = hc[0];
    const int nv = (int)hc[1];
    for (int e = et; e < nv * nf; e += es) {
      UW[e] = hc[2 + e];
      UW[lm_pairs * nf + e] = hc[2 + lm_pairs * nf + e];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (WIDE) __syncthreads();
    const double* U = UW;
    const double* W = UW + lm_pairs * nf;
    if (nw <= 64 && lm_pairs <= LM_REG_PAIRS) {
      // lane j builds column j: its pair entries u_i[j], w_i[j] in registers, the row's u_i[k], w_i[k]
      // LDS broadcasts (one address per wave), four rows in flight; each entry the same operations in
      // the same order as the entry loop below (bitwise its M)
      const int jj = lane;
      const bool cj = jj < nf;
      double Uj[LM_REG_PAIRS], Wj[LM_REG_PAIRS];
#pragma unroll
      for (int i = 0; i < LM_REG_PAIRS; ++i) {
        Uj[i] = (cj && i < nv) ? U[i * nf + jj] : 0.0;
        Wj[i] = (cj && i < nv) ? W[i * nf + jj] : 0.0;
      }
      const int r0 = WIDE ? (int)(threadIdx.x >> 6) : 0, rs = WIDE ? IPM_WAVES : 1;
      constexpr int RU = 4;
      for (int k0 = r0; k0 < nw; k0 += rs * RU) {
        double h[RU];
        int kr[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          kr[u] = k0 + rs * u;
          h[u] = jj == kr[u] ? sigma : 0.0;
        }
#pragma unroll
        for (int i = 0; i < LM_REG_PAIRS; ++i) {
          if (i >= nv) break;
#pragma unroll
          for (int u = 0; u < RU; ++u) {
            const int kk = kr[u] < nf ? kr[u] : 0;
            h[u] = (h[u] - U[i * nf + kk] * Uj[i]) + W[i * nf + kk] * Wj[i];
          }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int kk = kr[u];
          if (kk < nw && jj < nw) {
            double v = (jj == kk) ? sg[kk] : 0.0;
            if (kk < nf && cj) v += h[u];
            Mb[kk * nw + jj] = v;
          }
        }
      }
    } else {
    // four entries per lane at a time (independent chains: their LDS reads overlap), each entry's
    // operations in the order of the one-entry loop
    constexpr int EU = 4;
    for (int e0 = et; e0 < nw * nw; e0 += es * EU) {
      int kk[EU], jj[EU];
      bool in[EU];
      double h[EU];
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int e = e0 + es * u;
        kk[u] = e / nw;
        jj[u] = e - kk[u] * nw;
        in[u] = e < nw * nw && kk[u] < nf && jj[u] < nf;
        h[u] = jj[u] == kk[u] ? sigma : 0.0;
      }
      for (int i = 0; i < nv; ++i) {
#pragma unroll
        for (int u = 0; u < EU; ++u)
          if (in[u])
            h[u] = (h[u] - U[i * nf + kk[u]] * U[i * nf + jj[u]]) + W[i * nf + kk[u]] * W[i * nf + jj[u]];
      }
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int e = e0 + es * u;
        if (e < nw * nw) {
          double v = (jj[u] == kk[u]) ? sg[kk[u]] : 0.0;
          if (in[u]) v += h[u];
          Mb[e] = v;
        }
      }
    }
    }  // (nw > 64)
  } else {
    const double* Hb = H ? H + b * (int64_t)nf * nf : nullptr;
    // h_sym: H is the raw central-difference matrix (cpl_ipm_fd_hessian_raw), symmetrised here as
    // batch_ipm.py's fd_hessian does: 0.5 (H + H^T) (unrolled: four entries' loads in flight)
#pragma unroll 4
    for (int e = et; e < nw * nw; e += es) {
      const int k = e / nw, j = e - k * nw;
      double v = (j == k) ? sg[k] : 0.0;
      if (Hb && k < nf && j < nf) v += h_sym ? 0.5 * (Hb[k * nf + j] + Hb[j * nf + k]) : Hb[k * nf + j];
      Mb[e] = v;
    }
  }
  if (!w0) return;
  double th = 0.0;
  for (int r = lane; r < m; r += 64) {
    const double cr = c[b * m + r];
    r2[b * m + r] = -cr;
    th += fabs(cr);
  }
  th = ipm_wave_sum(th);
  lg = ipm_wave_sum(lg);
  if (lane == 0) {
    theta[b] = th;
    phi[b] = f[b] - mub * lg;
  }
}

// batches up to this size run the Newton setup one instance per workgroup (WIDE)
constexpr int64_t NEWTON_WIDE_MAX = 1024;

// After the Newton step (batch_ipm.py step): bound-multiplier steps dzL = mu/dl - zL - zL/dl dw,
// dzU = mu/du - zU + zU/du dw, their fraction-to-the-boundary step a_z, the primal one a_max,
// gd = grad_phi . dw, switch_ok = ls_switch_flags (gd < 0, theta <= theta_min), and delta_w_last <- delta_w on the
// active instances.
__global__ __launch_bounds__(256) void cpl_ipm_post_step_kernel(int64_t batch, const PostStepArgs P,
                                                                const LsSetupArgs ls) {
  const int64_t b = (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch) return;
  ipm_post_step_one(P, b, ls);
}

// Acceptance (batch_ipm.py step, "accept" + state write-back, in place): filter augmentation after
// h-type steps (ring slot fcount mod nfilt), filter reset of failed searches, y += alpha dy,
// z += a_z dz with the kappa_Sigma = 1e10 safeguard at the new point, w <- w_new, mu, iters.
// a_z is taken as 0 where rest (the feasibility step keeps the multipliers).  failed / rest may be
// NULL (no filter resets / no multiplier-keeping rows: the solve engine's restoration phase).
__global__ __launch_bounds__(256) void cpl_ipm_accept_kernel(const IpmAcceptArgs a, int64_t batch) {
  const int64_t b = (int64_t)blockIdx.x * IPM_WAVES + (threadIdx.x >> 6);
  if (b >= batch) return;
  ipm_accept_one(a, b, threadIdx.x & 63);
}

// dst[b] = src[b] for the rows with mask[b] (row length len doubles), 16-byte accesses when aligned.
__global__ __launch_bounds__(256) void cpl_ipm_masked_rows_kernel(int64_t total, int64_t len,
                                                                  const uint8_t* __restrict__ mask,
                                                                  const double* __restrict__ src,
                                                                  double* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  if (mask[e / len]) dst[e] = src[e];
}

// A = dc/dw = [J_free | -P] of every instance, dense [m, nw], straight from the CSR Jacobian values:
// amap[r * nf + k] = CSR position of (row r, free column k) or -1 (structural zero), NaN -> 0
// (a cone at zero tangential force); the slack block is -1 at (r, nf + row_slack[r]).
__global__ __launch_bounds__(256) void cpl_ipm_dense_a_kernel(int64_t total, int m, int nw, int nf, int nnz,
                                                              const int32_t* __restrict__ amap,
                                                              const int32_t* __restrict__ row_slack,
                                                              const double* __restrict__ jac,
                                                              double* __restrict__ A,
                                                              const uint8_t* __restrict__ active) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  dense_a_entry(e, m, nw, nf, nnz, amap, row_slack, jac, A, active);
}

// Central-difference points of the solve loop's Hessian (batch_ipm.py fd_hessian): for instance b
// and free variable k, h = fd_step max(|x_free k|, 1); point p < nf is x + h e_{free p}, point
// nf + p is x - h e_{free p}.  Xp [batch, 2 nf, n], h_out [batch, nf].  freepos[col] = k or -1.
__global__ __launch_bounds__(256) void cpl_ipm_fd_points_kernel(int64_t total, int n, int nf, double fd_step,
                                                                const int32_t* __restrict__ freepos,
                                                                const double* __restrict__ X,
                                                                double* __restrict__ Xp, double* __restrict__ h_out,
                                                                const uint8_t* __restrict__ active) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int per = 2 * nf * n;
  const int64_t b = e / per;
  if (active && !active[b]) return;
  const int pc = (int)(e - b * per);
  const int p = pc / n, col = pc - p * n;
  const double xv = X[b * n + col];
  const int k = freepos[col];
  double v = xv;
  if (k >= 0 && (p == k || p == nf + k)) {
    const double h = fd_step * fmax(fabs(xv), 1.0);
    v = p == k ? xv + h : xv - h;
    if (p == k) h_out[b * nf + k] = h;
  }
  Xp[e] = v;
}

// Raw central-difference Hessian of the Lagrangian over the free variables (batch_ipm.py
// fd_hessian): H[b, k, j] = (gL[b, k, free j] - gL[b, nf + k, free j]) / (2 h[b, k]); thread per
// entry, rows of gL read contiguously.  Symmetrised by the Newton setup.
__global__ __launch_bounds__(256) void cpl_ipm_fd_hessian_raw_kernel(int64_t total, int n, int nf,
                                                                     const int64_t* __restrict__ free_idx,
                                                                     const double* __restrict__ gL,
                                                                     const double* __restrict__ h,
                                                                     double* __restrict__ H,
                                                                     const uint8_t* __restrict__ active) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int per = nf * nf;
  const int64_t b = e / per;
  if (active && !active[b]) return;
  const int kj = (int)(e - b * per);
  const int k = kj / nf, j = kj - k * nf;
  const double* gb = gL + b * (int64_t)2 * nf * n;
  const int64_t c = free_idx[j];
  H[e] = (gb[(int64_t)k * n + c] - gb[(int64_t)(nf + k) * n + c]) / (2.0 * h[b * nf + k]);
}


// the barrier parameter's floor of IPOPT's MonotoneMuUpdate: min(tol, compl_inf_tol = 1e-4) /
// (barrier_tol_factor + 1)
double ipm_mu_min(double tol) { return fmin(tol, 1e-4) / 11.0; }

#define IPM_LAUNCH(kernel, name, ...)                                                                   \
  do {                                                                                                 \
    const int64_t blocks_ = (batch + IPM_WAVES - 1) / IPM_WAVES;                                       \
    if (blocks_ > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, name ": batch too large");       \
    hipLaunchKernelGGL(kernel, dim3((unsigned)blocks_), dim3(64 * IPM_WAVES), 0, (hipStream_t)stream,   \
                       __VA_ARGS__);                                                                   \
    hipError_t e_ = hipGetLastError();                                                                 \
    if (e_ != hipSuccess) return fail(CPL_ERR_HIP, std::string(name " launch: ") + hipGetErrorString(e_)); \
    return CPL_OK;                                                                                     \
  } while (0)


// cpl_ipm_post_step with the solve loop's line-search setup fused in (ls != NULL: LsSetupArgs)
int32_t ipm_post_step_ex(int64_t batch, int32_t nw, const double* d_w, const double* d_dw, const double* d_zL,
                         const double* d_zU, const double* d_gphi, const double* d_mu, const double* d_tau,
                         const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                         const double* d_theta, const double* d_theta_min, const uint8_t* d_active,
                         const double* d_delta_w, double* d_dwl, double* d_dzL, double* d_dzU, double* d_a_max,
                         double* d_a_z, double* d_gd, uint8_t* d_switch_ok, const LsSetupArgs* ls, void* stream) {
  LsSetupArgs L{};
  if (ls) L = *ls;
  const PostStepArgs P{(int32_t)nw, d_w, d_dw, d_zL, d_zU, d_gphi, d_mu, d_tau, d_hasL, d_hasU, d_wl0, d_wu0,
                       d_theta, d_theta_min, d_active, d_delta_w, d_dwl, d_dzL, d_dzU, d_a_max, d_a_z, d_gd,
                       d_switch_ok};
  IPM_LAUNCH(cpl_ipm_post_step_kernel, "cpl_ipm_post_step", batch, P, L);
}

// cpl_ipm_optimality with the engine's extras: mu_rounds barrier decreases at most, the floor
// mu_min, tiny_flag (a forced first decrease after two tiny steps) and skip (instances in the
// restoration phase, left untouched: their own test and barrier update run in its kernels)
int32_t ipm_optimality_ex(int64_t batch, int32_t nw, int32_t m, int32_t nfilt, int32_t nbounds, double tol,
                          double acc_tol, int32_t acc_iter, const double* d_A, const double* d_gw, const double* d_c,
                          const double* d_w, const double* d_y, const double* d_zL, const double* d_zU,
                          const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                          const double* d_mu, const double* d_filt_t, const double* d_filt_p, const int64_t* d_fcount,
                          uint8_t* d_active, int64_t* d_status, int64_t* d_acc, double* d_d_inf, double* d_err0,
                          double* d_base, double* d_mu_out, double* d_filt_t_out, double* d_filt_p_out,
                          int64_t* d_fcount_out, int32_t mu_rounds, double mu_min, const uint8_t* d_tiny_flag,
                          const uint8_t* d_skip, const IpmUnpack* unpack, void* stream) {
  const int64_t blocks = (batch + IPM_WAVES - 1) / IPM_WAVES;
  IpmUnpack up{};
  if (unpack) up = *unpack;
  if (batch == 0) return CPL_OK;
  hipLaunchKernelGGL(cpl_ipm_optimality_kernel, dim3((unsigned)blocks), dim3(64 * IPM_WAVES), 0, (hipStream_t)stream,
                     batch, (int)nw, (int)m, (int)nfilt, (int)nbounds, tol, acc_tol, (int)acc_iter, d_A, d_gw, d_c, d_w,
                     d_y, d_zL, d_zU, d_hasL, d_hasU, d_wl0, d_wu0, d_mu, d_filt_t, d_filt_p, d_fcount, d_active,
                     d_status, d_acc, d_d_inf, d_err0, d_base, d_mu_out, d_filt_t_out, d_filt_p_out, d_fcount_out,
                     (int)mu_rounds, mu_min, d_tiny_flag, d_skip, up);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_optimality launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

}  // namespace cpl

using namespace cpl;

extern "C" {

int32_t cpl_ipm_trial_point(int64_t batch, int32_t n, int32_t nf, int32_t nw, const int64_t* d_free_idx,
                            const int64_t* d_fixed_idx, const double* d_Xbase, const double* d_w, const double* d_dir,
                            const double* d_alpha, const uint8_t* d_mask, const double* d_w_keep, double* d_wt,
                            double* d_X, void* stream) {
  if (batch < 0 || n <= 0 || nf < 0 || nf > n || nw < nf)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_trial_point: bad sizes");
  if (batch == 0) return CPL_OK;
  if (!d_free_idx || (n > nf && !d_fixed_idx) || !d_Xbase || !d_w || !d_dir || !d_alpha || !d_mask || !d_w_keep ||
      !d_wt || !d_X)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_trial_point: missing buffer");
  const int64_t blocks = (batch + IPM_WAVES - 1) / IPM_WAVES;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_trial_point: batch too large");
  hipLaunchKernelGGL(cpl_ipm_trial_point_kernel, dim3((unsigned)blocks), dim3(64 * IPM_WAVES), 0, (hipStream_t)stream,
                     batch, (int)n, (int)nf, (int)nw, d_free_idx, d_fixed_idx, d_Xbase, d_w, d_dir, d_alpha, d_mask,
                     d_w_keep, d_wt, d_X);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_trial_point launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

int32_t cpl_ipm_judge_take(int64_t batch, int32_t nw, int32_t m, int32_t nf, int32_t nfilt, const int32_t* d_row_slack,
                           const double* d_gl, const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0,
                           const double* d_wu0, const double* d_wt, const double* d_f_t, const double* d_g_t,
                           const double* d_alpha, const double* d_mu, const double* d_theta_k, const double* d_phi_k,
                           const double* d_gd, const uint8_t* d_switch_ok, const double* d_theta_max,
                           const double* d_filt_t, const double* d_filt_p, const uint8_t* d_extra_mask,
                           uint8_t* d_searching, double* d_st_f, double* d_st_g, double* d_st_w, double* d_st_alpha,
                           uint8_t* d_st_aug, double* d_th_out, uint8_t* d_ok_out, int32_t mode, void* stream) {
  if (batch < 0 || nw <= 0 || m < 0 || nf < 0 || nf > nw || nfilt < 0 || mode != 0)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_judge_take: bad sizes (mode must be 0)");
  if (batch == 0) return CPL_OK;
  if ((m > 0 && (!d_row_slack || !d_gl || !d_g_t || !d_st_g)) || !d_hasL || !d_hasU || !d_wl0 || !d_wu0 || !d_wt ||
      !d_f_t || !d_alpha || !d_mu || !d_theta_k || !d_phi_k || !d_gd || !d_switch_ok || !d_theta_max ||
      (nfilt > 0 && (!d_filt_t || !d_filt_p)) || !d_searching || !d_st_f || !d_st_w || !d_st_alpha || !d_st_aug ||
      !d_th_out || !d_ok_out)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_judge_take: missing buffer");
  const int64_t blocks = (batch + IPM_WAVES - 1) / IPM_WAVES;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_judge_take: batch too large");
  hipLaunchKernelGGL(cpl_ipm_judge_take_kernel, dim3((unsigned)blocks), dim3(64 * IPM_WAVES), 0, (hipStream_t)stream,
                     batch, (int)nw, (int)m, (int)nf, (int)nfilt, d_row_slack, d_gl, d_hasL, d_hasU, d_wl0, d_wu0, d_wt,
                     d_f_t, d_g_t, d_alpha, d_mu, d_theta_k, d_phi_k, d_gd, d_switch_ok, d_theta_max, d_filt_t,
                     d_filt_p, d_extra_mask, d_searching, d_st_f, d_st_g, d_st_w, d_st_alpha, d_st_aug, d_th_out,
                     d_ok_out, (int)mode);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_judge_take launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

int32_t cpl_ipm_optimality(int64_t batch, int32_t nw, int32_t m, int32_t nfilt, int32_t nbounds, double tol,
                           double acc_tol, int32_t acc_iter, const double* d_A, const double* d_gw, const double* d_c,
                           const double* d_w, const double* d_y, const double* d_zL, const double* d_zU,
                           const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                           const double* d_mu, const double* d_filt_t, const double* d_filt_p,
                           const int64_t* d_fcount, uint8_t* d_active, int64_t* d_status, int64_t* d_acc,
                           double* d_d_inf, double* d_err0, double* d_base, double* d_mu_out, double* d_filt_t_out,
                           double* d_filt_p_out, int64_t* d_fcount_out, void* stream) {
  if (batch < 0 || nw <= 0 || nw > 128 || m < 0 || nfilt < 0 || nbounds < 0)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_optimality: need 0 < nw <= 128, m >= 0");
  if (batch == 0) return CPL_OK;
  if ((m > 0 && (!d_A || !d_c || !d_y)) || !d_gw || !d_w || !d_zL || !d_zU || !d_hasL || !d_hasU || !d_wl0 ||
      !d_wu0 || !d_mu || (nfilt > 0 && (!d_filt_t || !d_filt_p || !d_filt_t_out || !d_filt_p_out)) || !d_fcount ||
      !d_active || !d_status || !d_acc || !d_d_inf || !d_err0 || !d_base || !d_mu_out || !d_fcount_out)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_optimality: missing buffer");
  const int64_t blocks = (batch + IPM_WAVES - 1) / IPM_WAVES;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_optimality: batch too large");
  return ipm_optimality_ex(batch, nw, m, nfilt, nbounds, tol, acc_tol, acc_iter, d_A, d_gw, d_c, d_w, d_y, d_zL, d_zU,
                           d_hasL, d_hasU, d_wl0, d_wu0, d_mu, d_filt_t, d_filt_p, d_fcount, d_active, d_status, d_acc,
                           d_d_inf, d_err0, d_base, d_mu_out, d_filt_t_out, d_filt_p_out, d_fcount_out, IPM_MU_ROUNDS,
                           ipm_mu_min(tol), nullptr, nullptr, nullptr, stream);
}

int32_t cpl_ipm_max_step(int64_t batch, int32_t nw, const double* d_v, const double* d_dir, const double* d_v2,
                         const double* d_dir2, const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_lo,
                         const double* d_up, const double* d_tau, double* d_out, void* stream) {
  if (batch < 0 || nw <= 0) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_max_step: bad sizes");
  if (batch == 0) return CPL_OK;
  if (!d_v || !d_dir || !d_hasL || !d_hasU || (d_v2 ? !d_dir2 : (!d_lo || !d_up)) || !d_tau || !d_out)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_max_step: missing buffer");
  const int64_t blocks = (batch + IPM_WAVES - 1) / IPM_WAVES;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_max_step: batch too large");
  hipLaunchKernelGGL(cpl_ipm_max_step_kernel, dim3((unsigned)blocks), dim3(64 * IPM_WAVES), 0, (hipStream_t)stream,
                     batch, (int)nw, d_v, d_dir, d_v2, d_dir2, d_hasL, d_hasU, d_lo, d_up, d_tau, d_out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_max_step launch: ") + hipGetErrorString(e));
  return CPL_OK;
}


int32_t cpl_ipm_newton_setup(int64_t batch, int32_t nw, int32_t m, int32_t nf, const double* d_w, const double* d_zL,
                             const double* d_zU, const double* d_gw, const double* d_A, const double* d_y,
                             const double* d_c, const double* d_f, const double* d_mu, const uint8_t* d_hasL,
                             const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0, const double* d_H,
                             int32_t h_sym, double* d_M, double* d_r1, double* d_r2, double* d_gphi, double* d_mr_diag,
                             double* d_theta, double* d_phi, const uint8_t* d_active, void* stream) {
  if (batch < 0 || nw <= 0 || m < 0 || nf < 0 || nf > nw) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_newton_setup: bad sizes");
  // Sigma is staged per wave in sig_s[IPM_WAVES][128] (same limit as cpl_ipm_optimality / cpl_kkt_solve)
  if (nw > 128) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_newton_setup: nw > 128 is not supported");
  if (batch == 0) return CPL_OK;
  if (!d_w || !d_zL || !d_zU || !d_gw || (m > 0 && (!d_A || !d_y || !d_c || !d_r2)) || !d_f || !d_mu || !d_hasL ||
      !d_hasU || !d_wl0 || !d_wu0 || !d_M || !d_r1 || !d_gphi || !d_mr_diag || !d_theta || !d_phi)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_newton_setup: missing buffer");
  if (batch <= NEWTON_WIDE_MAX) {  // one instance per workgroup
    hipLaunchKernelGGL((cpl_ipm_newton_setup_kernel<false, true>), dim3((unsigned)batch), dim3(64 * IPM_WAVES), 0,
                       (hipStream_t)stream, batch, (int)nw, (int)m, (int)nf, d_w, d_zL,
             d_zU, d_gw, d_A, d_y, d_c, d_f, d_mu, d_hasL, d_hasU, d_wl0, d_wu0, d_H, (int)h_sym, d_M, d_r1, d_r2,
             d_gphi, d_mr_diag, d_theta, d_phi, d_active, nullptr, 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_newton_setup launch: ") + hipGetErrorString(e));
    return CPL_OK;
  }
  IPM_LAUNCH(cpl_ipm_newton_setup_kernel<false>, "cpl_ipm_newton_setup", batch, (int)nw, (int)m, (int)nf, d_w, d_zL,
             d_zU, d_gw, d_A, d_y, d_c, d_f, d_mu, d_hasL, d_hasU, d_wl0, d_wu0, d_H, (int)h_sym, d_M, d_r1, d_r2,
             d_gphi, d_mr_diag, d_theta, d_phi, d_active, nullptr, 0);
}


int32_t cpl_ipm_post_step(int64_t batch, int32_t nw, const double* d_w, const double* d_dw, const double* d_zL,
                          const double* d_zU, const double* d_gphi, const double* d_mu, const double* d_tau,
                          const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                          const double* d_theta, const double* d_theta_min, const uint8_t* d_active,
                          const double* d_delta_w, double* d_dwl, double* d_dzL, double* d_dzU, double* d_a_max,
                          double* d_a_z, double* d_gd, uint8_t* d_switch_ok, void* stream) {
  if (batch < 0 || nw <= 0) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_post_step: bad sizes");
  if (batch == 0) return CPL_OK;
  if (!d_w || !d_dw || !d_zL || !d_zU || !d_gphi || !d_mu || !d_tau || !d_hasL || !d_hasU || !d_wl0 || !d_wu0 ||
      !d_theta || !d_theta_min || !d_active || !d_delta_w || !d_dwl || !d_dzL || !d_dzU || !d_a_max || !d_a_z ||
      !d_gd || !d_switch_ok)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_post_step: missing buffer");
  return ipm_post_step_ex(batch, nw, d_w, d_dw, d_zL, d_zU, d_gphi, d_mu, d_tau, d_hasL, d_hasU, d_wl0, d_wu0, d_theta,
                          d_theta_min, d_active, d_delta_w, d_dwl, d_dzL, d_dzU, d_a_max, d_a_z, d_gd, d_switch_ok,
                          nullptr, stream);
}

int32_t cpl_ipm_accept(int64_t batch, int32_t nw, int32_t m, int32_t nfilt, const uint8_t* d_active,
                       const uint8_t* d_aug, const uint8_t* d_failed, const uint8_t* d_rest, const double* d_alpha,
                       const double* d_a_z, const double* d_theta, const double* d_phi, const double* d_filt_t_in,
                       const double* d_filt_p_in, const int64_t* d_fcount_in, const double* d_w_new,
                       const double* d_dy, const double* d_dzL, const double* d_dzU, const double* d_mu,
                       const uint8_t* d_hasL, const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0,
                       double* d_w, double* d_y, double* d_zL, double* d_zU, double* d_mu_state, int64_t* d_iters,
                       double* d_filt_t, double* d_filt_p, int64_t* d_fcount, void* stream) {
  if (batch < 0 || nw <= 0 || m < 0 || nfilt <= 0) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_accept: bad sizes");
  if (batch == 0) return CPL_OK;
  if (!d_active || !d_aug || !d_alpha || !d_a_z || !d_theta || !d_phi || !d_filt_t_in ||
      !d_filt_p_in || !d_fcount_in || !d_w_new || (m > 0 && (!d_dy || !d_y)) || !d_dzL || !d_dzU || !d_mu ||
      !d_hasL || !d_hasU || !d_wl0 || !d_wu0 || !d_w || !d_zL || !d_zU || !d_mu_state || !d_iters || !d_filt_t ||
      !d_filt_p || !d_fcount)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_accept: missing buffer");
  const IpmAcceptArgs a{(int)nw, (int)m, (int)nfilt, d_active, d_aug, d_failed, d_rest, d_alpha, d_a_z, d_theta,
                        d_phi, d_filt_t_in, d_filt_p_in, d_fcount_in, d_w_new, d_dy, d_dzL, d_dzU, d_mu, d_hasL,
                        d_hasU, d_wl0, d_wu0, d_w, d_y, d_zL, d_zU, d_mu_state, d_iters, d_filt_t, d_filt_p,
                        d_fcount};
  IPM_LAUNCH(cpl_ipm_accept_kernel, "cpl_ipm_accept", a, batch);
}

int32_t cpl_ipm_masked_rows(int64_t batch, int64_t row_len, const uint8_t* d_mask, const double* d_src, double* d_dst,
                            void* stream) {
  if (batch < 0 || row_len < 0) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_masked_rows: bad sizes");
  if (batch == 0 || row_len == 0) return CPL_OK;
  if (!d_mask || !d_src || !d_dst) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_masked_rows: missing buffer");
  const int64_t total = batch * row_len;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_masked_rows: batch too large");
  hipLaunchKernelGGL(cpl_ipm_masked_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, total,
                     row_len, d_mask, d_src, d_dst);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_masked_rows launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

int32_t cpl_ipm_dense_a(int64_t batch, int32_t m, int32_t nw, int32_t nf, int32_t nnz, const int32_t* d_amap,
                        const int32_t* d_row_slack, const double* d_jac, double* d_A, const uint8_t* d_active,
                        void* stream) {
  if (batch < 0 || m < 0 || nw <= 0 || nf < 0 || nf > nw || nnz < 0)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_dense_a: bad sizes");
  if (batch == 0 || m == 0) return CPL_OK;
  if (!d_amap || !d_row_slack || (nnz > 0 && !d_jac) || !d_A)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_dense_a: missing buffer");
  const int64_t total = batch * (int64_t)m * nw;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_dense_a: batch too large");
  hipLaunchKernelGGL(cpl_ipm_dense_a_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, total, (int)m,
                     (int)nw, (int)nf, (int)nnz, d_amap, d_row_slack, d_jac, d_A, d_active);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_dense_a launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

int32_t cpl_ipm_fd_points(int64_t batch, int32_t n, int32_t nf, double fd_step, const int32_t* d_freepos,
                          const double* d_X, double* d_Xp, double* d_h, const uint8_t* d_active, void* stream) {
  if (batch < 0 || n <= 0 || nf < 0 || nf > n) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_fd_points: bad sizes");
  if (batch == 0 || nf == 0) return CPL_OK;
  if (!d_freepos || !d_X || !d_Xp || !d_h) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_fd_points: missing buffer");
  const int64_t total = batch * 2 * (int64_t)nf * n;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_fd_points: batch too large");
  hipLaunchKernelGGL(cpl_ipm_fd_points_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, total,
                     (int)n, (int)nf, fd_step, d_freepos, d_X, d_Xp, d_h, d_active);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_fd_points launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

int32_t cpl_ipm_fd_hessian_raw(int64_t batch, int32_t n, int32_t nf, const int64_t* d_free_idx, const double* d_gL,
                               const double* d_h, double* d_H, const uint8_t* d_active, void* stream) {
  if (batch < 0 || n <= 0 || nf < 0 || nf > n) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_fd_hessian_raw: bad sizes");
  if (batch == 0 || nf == 0) return CPL_OK;
  if (!d_free_idx || !d_gL || !d_h || !d_H) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_fd_hessian_raw: missing buffer");
  const int64_t total = batch * (int64_t)nf * nf;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_ipm_fd_hessian_raw: batch too large");
  hipLaunchKernelGGL(cpl_ipm_fd_hessian_raw_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, total,
                     (int)n, (int)nf, d_free_idx, d_gL, d_h, d_H, d_active);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_ipm_fd_hessian_raw launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

}  // extern "C"

namespace cpl {
// The native engine's Newton setup over its compact limited-memory model (see the LM kernel above);
// the arguments otherwise as cpl_ipm_newton_setup.
int32_t ipm_newton_setup_lm(int64_t batch, int32_t nw, int32_t m, int32_t nf, const double* d_w, const double* d_zL,
                            const double* d_zU, const double* d_gw, const double* d_A, const double* d_y,
                            const double* d_c, const double* d_f, const double* d_mu, const uint8_t* d_hasL,
                            const uint8_t* d_hasU, const double* d_wl0, const double* d_wu0, const double* d_Hc,
                            int32_t lm_pairs, double* d_M, double* d_r1, double* d_r2, double* d_gphi,
                            double* d_mr_diag, double* d_theta, double* d_phi, const uint8_t* d_active, void* stream) {
  if (batch < 0 || nw <= 0 || nw > 128 || m < 0 || nf < 0 || nf > nw || lm_pairs <= 0 || !d_Hc)
    return fail(CPL_ERR_INVALID_ARGUMENT, "ipm_newton_setup_lm: bad arguments");
  if (batch == 0) return CPL_OK;
  const int64_t blocks = (batch + IPM_WAVES - 1) / IPM_WAVES;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "ipm_newton_setup_lm: batch too large");
  const bool wide = batch <= NEWTON_WIDE_MAX;  // one instance per workgroup
  const size_t lds = sizeof(double) * (wide ? 1 : IPM_WAVES) * 2 * (size_t)lm_pairs * nf;
  hipLaunchKernelGGL((wide ? cpl_ipm_newton_setup_kernel<true, true> : cpl_ipm_newton_setup_kernel<true, false>),
                     dim3((unsigned)(wide ? batch : blocks)), dim3(64 * IPM_WAVES), lds, (hipStream_t)stream, batch, (int)nw, (int)m, (int)nf, d_w, d_zL, d_zU, d_gw, d_A, d_y, d_c, d_f,
                     d_mu, d_hasL, d_hasU, d_wl0, d_wu0, nullptr, 0, d_M, d_r1, d_r2, d_gphi, d_mr_diag, d_theta, d_phi,
                     d_active, d_Hc, (int)lm_pairs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("ipm_newton_setup_lm launch: ") + hipGetErrorString(e));
  return CPL_OK;
}
}  // namespace cpl
