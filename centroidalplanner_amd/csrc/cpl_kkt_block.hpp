// cpl_kkt_block.hpp — the workgroup KKT kernel's solve with kept factors (cpl_kkt.hip kkt_block), shared
// with the solve engine's fused line-search kernel (cpl_kernels.hip cpl_ls_backtrack_kernel), which
// re-solves IPOPT's regularised (augmented) systems for its second-order corrections on one wave with
// the same arithmetic: the helpers are templated on the threads that take part (NT: the workgroup's 256
// or one wave's 64) — a row's dot product is computed by the same four lanes' partial sums in the same
// order either way, so both give the same bits.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "cpl_kkt_qd.hpp"
#include "cpl_kkt_wave.hpp"
#include "cpl_wave.hpp"

namespace cpl {

constexpr int KKT_THREADS = 256;
constexpr int KKT_MAX_NW = 128;

// Dot products of n strided vectors with one shared operand, G lanes per vector (G | 64): lane
// `part` of a group sums k = part, part + G, ... and the group reduces with log2(G) xor shuffles;
// fin(r, dot) runs on the group's first lane.  Every thread of the workgroup must call it (the
// shuffles run on all lanes; groups never straddle a wave).  Row r of A starts at A + r * sr, its
// k-th element at stride sk.
template <int G, int NT = KKT_THREADS, class F>
__device__ __forceinline__ void group_dots(int n, int len, const double* A, int sr, int sk, const double* x, int sx,
                                           F fin) {
  const int part = threadIdx.x % G;
  for (int base = 0; base < n * G; base += NT) {
    const int r = (base + (int)threadIdx.x) / G;
    const bool act = r < n;
    double s0 = 0.0, s1 = 0.0;
    if (act) {
      const double* a = A + (int64_t)r * sr;
      int k = part;
      for (; k + G < len; k += 2 * G) {
        const double p0 = a[k * sk], p1 = a[(k + G) * sk];
        s0 += p0 * x[k * sx];
        s1 += p1 * x[(k + G) * sx];
      }
      if (k < len) s0 += a[k * sk] * x[k * sx];
    }
    double s = s0 + s1;
    if constexpr (G == 4) {
      s = group4_sum(s);
    } else if constexpr (G == 8) {
      s = group8_sum(s);
    } else {
#pragma unroll
      for (int o = 1; o < G; o <<= 1) s += __shfl_xor(s, o);
    }
    if (act && part == 0) fin(r, s);
  }
}


// Solve with the factors in LDS: Q [nw][nw] (row-major: Q[r*nw + c]), QR array (row j = column j of
// A^T after the reflections; R[i][j] = QR[j*nw + i] for i < j, R[j][j] = QR[j*nw + j]), L [nz][nz] the
// Cholesky of the reduced Hessian, M [nw][nw] (plus delta_w on the diagonal, applied here).
// Vectors in LDS: q1 [nw], q2 [m] -> dw [nw], dy [m].  tmp: >= 2*nw doubles.  delta_w acts on the
// first nw0 unknowns (nw0 = nw but for the augmented system of a regularised Jacobian: its W block).
template <int NT = KKT_THREADS>
__device__ __forceinline__ void kkt_solve_lds(int nw, int m, int nw0, const double* Q, const double* QR,
                              const double* L, const double* M, double dW, const double* q1, const double* q2,
                              double* dw, double* dy, double* tmp) {
  const int tid = threadIdx.x;
  const int nz = nw - m;
  double* py = tmp;          // [m]
  double* t = tmp + nw;      // [nw]
  // R^T p_y = q2 (forward substitution; (R^T)[i][k] = R[k][i] = QR[i*nw + k])
  for (int i = tid; i < m; i += NT) py[i] = q2[i];
  __syncthreads();
  if (tid < 64) wave_trsv(m, true, QR, nw, 1, QR, nw + 1, py);
  __syncthreads();
  // dw <- Y p_y
  group_dots<4, NT>(nw, m, Q, nw, 1, py, 1, [&](int r, double d) { dw[r] = d; });
  __syncthreads();
  // t = q1 - (M + dW I) Y p_y
  group_dots<4, NT>(nw, nw, M, nw, 1, dw, 1, [&](int r, double d) { t[r] = q1[r] - (r < nw0 ? dW * dw[r] : 0.0) - d; });
  __syncthreads();
  if (nz > 0) {
    // rz = Z^T t into tmp[m .. m+nz) (py still needed) -> p_z by the two triangular solves
    double* rz = tmp + m;
    group_dots<4, NT>(nz, nw, Q + m, 1, nw, t, 1, [&](int c, double d) { rz[c] = d; });
    __syncthreads();
    if (tid < 64) {
      wave_trsv(nz, true, L, nz, 1, L, nz + 1, rz);    // L y = rz
      wave_trsv(nz, false, L, 1, nz, L, nz + 1, rz);   // L^T z = y
    }
    __syncthreads();
    // dw += Z p_z
    group_dots<4, NT>(nw, nz, Q + m, nw, 1, rz, 1, [&](int r, double d) { dw[r] += d; });
    __syncthreads();
  }
  // u = q1 - (M + dW I) dw  -> s = Y^T u -> R dy = s
  group_dots<4, NT>(nw, nw, M, nw, 1, dw, 1, [&](int r, double d) { t[r] = q1[r] - (r < nw0 ? dW * dw[r] : 0.0) - d; });
  __syncthreads();
  group_dots<4, NT>(m, nw, Q, 1, nw, t, 1, [&](int k, double d) { dy[k] = d; });
  __syncthreads();
  // R dy = s (backward substitution; R[i][k] = QR[k*nw + i])
  if (tid < 64) wave_trsv(m, false, QR, 1, nw, QR, nw + 1, dy);
  __syncthreads();
}


// One step of iterative refinement of a re-solve (dw, dy in LDS or global scratch, from kkt_solve_lds
// with the kept factors): the residual of the full system [[M + dW I_nw0, A^T], [A, 0]] into rscr, the
// correction when the residual exceeds 1e-13 of the right-hand side, added in place.  *flag: a
// workgroup-shared int (NT > 64), unused on one wave.  The restatements refine every full-rank re-solve.
template <int NT = KKT_THREADS>
__device__ __forceinline__ void kkt_resolve_refine(int nw, int m, int nw0, const double* Q, const double* QR,
                                                   const double* L, const double* M, const double* Ab, double dW,
                                                   const double* q1, const double* q2, double* dw, double* dy,
                                                   double* tmp, double* rscr, int* flag) {
  const int tid = threadIdx.x;
  double* f1 = rscr;
  double* f2 = f1 + nw;
  double* h1 = f2 + m;
  double* h2 = h1 + nw;
  group_dots<4, NT>(nw, m, Ab, 1, nw, dy, 1, [&](int r, double d) { f1[r] = q1[r] - (r < nw0 ? dW * dw[r] : 0.0) - d; });
  group_dots<4, NT>(nw, nw, M, nw, 1, dw, 1, [&](int r, double d) { f1[r] -= d; });
  group_dots<4, NT>(m, nw, Ab, nw, 1, dw, 1, [&](int k, double d) { f2[k] = q2[k] - d; });
  __syncthreads();
  bool need = false;
  if (tid < 64) {
    double rmax = 0.0, qmax = 0.0;
    for (int r = tid; r < nw; r += 64) { rmax = fmax(rmax, fabs(f1[r])); qmax = fmax(qmax, fabs(q1[r])); }
    for (int k = tid; k < m; k += 64) { rmax = fmax(rmax, fabs(f2[k])); qmax = fmax(qmax, fabs(q2[k])); }
    rmax = wave_max(rmax);
    qmax = wave_max(qmax);
    need = !(rmax <= 1e-13 * qmax);
    if (NT > 64 && tid == 0) *flag = need ? 1 : 0;
  }
  if constexpr (NT > 64) {
    __syncthreads();
    need = *flag != 0;
  }
  if (need) {
    kkt_solve_lds<NT>(nw, m, nw0, Q, QR, L, M, dW, f1, f2, h1, h2, tmp);
    for (int r = tid; r < nw; r += NT) dw[r] += h1[r];
    for (int k = tid; k < m; k += NT) dy[k] += h2[k];
    __syncthreads();
  }
}

// The augmented workspace of one system (cpl_kkt.hip cpl_kkt_aug_kernel, IPOPT's Jacobian regularisation;
// na = nw + m unknowns): the factors as the workgroup kernel keeps them (kkt_ws_per(na, m): Q | QR | L,
// then delta_w ...) | W~ [na][na] | A~ [m][na] | [q1; 0] [na] | Pz [nw][nw] | the stepwise re-solve's
// refinement scratch [2 (na + m)] | the one-wave re-solve's scratch: q2 [m], dw [na], dy [m],
// tmp [max(2 na, 3 m)], refinement [2 (na + m)].
struct KktAugLayout {
  int64_t Ma, Aa, q1a, Pz, rscr, wq2, wdw, wdy, wtmp, wrscr, per;
  __host__ __device__ KktAugLayout(int nw, int m) {
    const int64_t na = nw + m;
    Ma = kkt_ws_per((int)na, m);
    Aa = Ma + na * na;
    q1a = Aa + (int64_t)m * na;
    Pz = q1a + na;
    rscr = Pz + (int64_t)nw * nw;
    wq2 = rscr + 2 * (na + m);
    wdw = wq2 + m;
    wdy = wdw + na;
    wtmp = wdy + m;
    wrscr = wtmp + (2 * na > 3 * (int64_t)m ? 2 * na : 3 * (int64_t)m);
    per = wrscr + 2 * (na + m);
  }
};
__host__ __device__ inline int64_t kkt_aug_ws_per(int nw, int m) { return KktAugLayout(nw, m).per; }

struct Dd {
  double a, b;
};

// The second-order correction's re-solve of an augmented (regularised) system on ONE wave (the fused
// line-search kernel, a workgroup of one wave): the same arithmetic as cpl_kkt_aug_kernel's mode 1 —
// kkt_solve_lds and one refinement step over the kept factors, W~, A~ and [q1; 0] of the system's
// workspace wsb (global: the vectors go through its scratch), the right-hand side q2 = -c_soc given per
// lane (lanes < m) — so the same bits as the stepwise search's re-solve.  Returns (dw, dy) of the lane
// (lanes < nw, < m).  Not inlined: the search kernel keeps its own registers (the branch is taken by
// regularised systems only).
static __device__ __noinline__ Dd kkt_aug_resolve_wave(int nw, int m, double* wsb, double q2v) {
  const int lane = threadIdx.x & 63;
  const int na = nw + m;
  const KktAugLayout Lo(nw, m);
  const int64_t per = kkt_ws_per(na, m);
  const double* Q = wsb;
  const double* QR = Q + (int64_t)na * na;
  const double* L = QR + (int64_t)m * na;
  const double dW = wsb[per - 4];
  double* q2 = wsb + Lo.wq2;
  if (lane < m) q2[lane] = q2v;
  __syncthreads();
  double* dw = wsb + Lo.wdw;
  double* dy = wsb + Lo.wdy;
  kkt_solve_lds<64>(na, m, nw, Q, QR, L, wsb + Lo.Ma, dW, wsb + Lo.q1a, q2, dw, dy, wsb + Lo.wtmp);
  kkt_resolve_refine<64>(na, m, nw, Q, QR, L, wsb + Lo.Ma, wsb + Lo.Aa, dW, wsb + Lo.q1a, q2, dw, dy, wsb + Lo.wtmp,
                         wsb + Lo.wrscr, nullptr);
  return Dd{lane < nw ? dw[lane] : 0.0, lane < m ? dy[lane] : 0.0};
}

}  // namespace cpl
