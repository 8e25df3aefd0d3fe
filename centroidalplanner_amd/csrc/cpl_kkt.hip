// cpl_kkt.hip — batched primal-dual Newton step of the solve loop (centroidalplanner_amd/batch_ipm.py)
// on gfx950: one workgroup per solver instance, every matrix of the step resident in LDS.
//
// Per instance (IPOPT's KKT system, Waechter & Biegler 2006, eq. 13 with the bound terms folded in):
//     [ M    A^T ] [dw]   [r1]        M  = W + Sigma   (nw x nw, symmetric)
//     [ A     0  ] [dy] = [r2]        A  = [J_free | -P] (m x nw)
// solved by the null-space method on a Householder QR of A^T = Q [R; 0], Q = [Y Z]:
//     R^T p_y = r2,   (Z^T (M + dW I) Z) p_z = Z^T (r1 - (M + dW I) Y p_y),   dw = Y p_y + Z p_z,
//     R dy = Y^T (r1 - (M + dW I) dw),
// with IPOPT's inertia correction inside the kernel: the KKT matrix has inertia (nw+, m-, 0) iff A
// has full row rank and the reduced Hessian Z^T M Z is positive definite, so the Cholesky of the
// reduced Hessian is the inertia test (pivots at the rounding level eps max|M_ii| count as zero) and dW follows IPOPT's schedule (first trial 1e-4, or
// dW_last / 3; growth x100 without history, x8 with) until it succeeds; a rank-deficient A (|R_jj|
// tiny) gets dC = 1e-8 mu^(1/4) |R|max on R's diagonal — or, opt-in (cpl_kkt_aug_kernel below), IPOPT's
// own (2,2)-block regularisation with jacobian_regularization_value 1e-8 mu^(1/4).
// One step of iterative refinement against the unregularised system follows when dC = 0.
// The factors are kept in a per-instance workspace so second-order corrections re-solve with
// another r2 without refactorising (mode 1).
//
// No library calls: the per-instance data-dependent retry loops run on the device, so the host
// never synchronises on them.  Sizes: nw <= KKT_MAX_NW (=128), m <= nw.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>

#include "cpl_status.hpp"
#include "cpl_wave.hpp"
#include "cpl_kkt_wave.hpp"
#include "cpl_kkt_qd.hpp"
#include "cpl_kkt_block.hpp"

namespace cpl {

// Phase timestamps for scripts/kkt_probe.hip (compiled with -DCPL_KKT_PROFILE only).
#ifdef CPL_KKT_PROFILE
__device__ long long* g_kkt_prof;
#define KKT_MARK(i)                                                            \
  do {                                                                         \
    if (threadIdx.x == 0) g_kkt_prof[(int64_t)blockIdx.x * 8 + (i)] = clock64(); \
  } while (0)
#else
#define KKT_MARK(i) \
  do {              \
  } while (0)
#endif



struct KktShared {
  int flag;
  int rank_def;
  double delta_w, delta_c;
};

// Dot product of two strided LDS vectors with four independent accumulators (latency, not order,
// bounds these short loops; the solver is not a parity-critical path).
__device__ __forceinline__ double lds_dot(const double* a, int sa, const double* b, int sb, int len) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int k = 0;
  for (; k + 3 < len; k += 4) {
    s0 += a[k * sa] * b[k * sb];
    s1 += a[(k + 1) * sa] * b[(k + 1) * sb];
    s2 += a[(k + 2) * sa] * b[(k + 2) * sb];
    s3 += a[(k + 3) * sa] * b[(k + 3) * sb];
  }
  for (; k < len; ++k) s0 += a[k * sa] * b[k * sb];
  return (s0 + s1) + (s2 + s3);
}

// The same with one operand in global memory (L2-resident): eight loads in flight per thread.
__device__ __forceinline__ double glb_dot(const double* a, int sa, const double* b, int sb, int len) {
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int k = 0;
  for (; k + 7 < len; k += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += a[(k + u) * sa] * b[(k + u) * sb];
  }
  for (; k < len; ++k) s[0] += a[k * sa] * b[k * sb];
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// LDS layout (doubles): Q | QR | L | dw | dy | tmp(max(2 nw, 3 m)).  M, the right-hand sides and the
// refinement's residual / correction stay in global memory (L2-resident while the workgroup runs):
// the image is 32.6 KiB at nw = 47, m = 30 — five workgroups per CU.
__host__ __device__ inline int kkt_lds_doubles(int nw, int m) {
  const int nz = nw - m;
  return nw * nw + m * nw + nz * nz + nw + m + (2 * nw > 3 * m ? 2 * nw : 3 * m);
}

// The factorisation (mode 0) also stages M Z [nw][nz] in LDS, right after tmp, when the larger
// image still fits: the reduced Hessian's Z^T (M Z) then reads it from LDS instead of 24 dependent
// rounds of L2 loads (at nw = 47, m = 30: 38.2 KiB, four workgroups per CU — measured as fast as
// five for this kernel).  Otherwise M Z goes to the global workspace.
__host__ __device__ inline bool kkt_mz_in_lds(int nw, int m) {
  return (int64_t)(kkt_lds_doubles(nw, m) + nw * (nw - m) + 8) * 8 <= 160 * 1024;
}
__host__ __device__ inline int kkt_launch_lds_doubles(int nw, int m, int mode) {
  return kkt_lds_doubles(nw, m) + (mode == 0 && kkt_mz_in_lds(nw, m) ? nw * (nw - m) : 0) + 8;
}

// One system on one workgroup (the body of cpl_kkt_kernel and cpl_kkt_aug_kernel): M [nw][nw], A
// [m][nw], the right-hand sides q1 [nw], q2 [m] in global memory; *mub (mode 0: the barrier parameter),
// *lastb (the previous delta_w, or none); the outputs dwo [nw0], dyo [m], *dWo, *dCo, *infob; wsb the
// system's workspace (the factors kept for mode 1).  nw0 = nw but for an augmented system (Pzg set):
// delta_w then acts on its first nw0 unknowns only — on the reduced Hessian as dW Pz, Pz = Z[:nw0]^T
// Z[:nw0] (global scratch Pzg [nz][nz]) — and dw is its first nw0 entries.
// NW, MM > 0: specialised for one system size (nw = NW, m = MM; the arguments are ignored) — every
// stride, trip count and index division becomes a compile-time constant, which the
// instruction-issue-bound kernel needs (SQ counters: ~75 % of wave cycles parked, the SIMDs' issue
// near saturation from 4 workgroups per CU); NW = 0: any size.
template <int NW, int MM>
__device__ __forceinline__ void kkt_block(int mode, int nw_arg, int m_arg, int nw0, const double* __restrict__ M,
                                          const double* __restrict__ Ab, const double* __restrict__ q1,
                                          const double* __restrict__ q2, const double* mub, const double* lastb,
                                          double* __restrict__ dwo, double* __restrict__ dyo, double* dWo,
                                          double* dCo, int32_t* infob, double* __restrict__ wsb, double* Pzg,
                                          double* rscr, double* sm, KktShared& sh) {
  const int nw = NW > 0 ? NW : nw_arg;
  const int m = NW > 0 ? MM : m_arg;
  const int tid = threadIdx.x;
  const int nz = nw - m;
  double* Q = sm;
  double* QR = Q + nw * nw;
  double* L = QR + m * nw;
  double* dw = L + nz * nz;
  double* dy = dw + nw;
  double* tmp = dy + m;  // max(2 nw, 3 m)
  // refinement residual and correction: global scratch past M Z in the workspace (overwritten by
  // the factors at the end)
  double* e1 = wsb + nw * nz;
  double* e2 = e1 + nw;
  double* c1 = e2 + m;
  double* c2 = c1 + nw;

  if (mode == 1) {  // re-solve with the kept factors
    const int64_t per = kkt_ws_per(nw, m);
    for (int64_t i = tid; i < per - 4; i += KKT_THREADS) sm[i] = wsb[i];
    if (tid == 0) { sh.delta_w = wsb[per - 4]; sh.delta_c = wsb[per - 3]; }
    __syncthreads();
    kkt_solve_lds(nw, m, nw0, Q, QR, L, M, sh.delta_w, q1, q2, dw, dy, tmp);
    if (rscr)  // (the augmented system) one step of iterative refinement, as its factorisation's, with
               // the residual and correction in rscr: wsb holds the kept factors
      kkt_resolve_refine(nw, m, nw0, Q, QR, L, M, Ab, sh.delta_w, q1, q2, dw, dy, tmp, rscr, &sh.flag);
    for (int i = tid; i < nw0; i += KKT_THREADS) dwo[i] = dw[i];
    for (int i = tid; i < m; i += KKT_THREADS) dyo[i] = dy[i];
    return;
  }

  // ---- Householder QR of A^T: row j of QR = column j of A^T
  for (int i = tid; i < m * nw; i += KKT_THREADS) QR[i] = Ab[i];
  __syncthreads();
  KKT_MARK(0);
  // Householder QR two columns at a time.  Wave 0 forms the reflector pair (j, j+1) — v in place
  // (v_j = 1 implicit), beta, R_jj on the diagonal, H_j applied to column j+1 in between — and
  // c_j = v_{j+1}^T v_j; then all waves take both dots of every later column in one pass
  //   s0 = beta_j (y_j + v_j^T y),  s1 = beta_{j+1} (y_{j+1} + v_{j+1}^T y - s0 c_j)
  // (8 lanes per column) and the update y -= s0 v_j + s1 v_{j+1}: wave 0 updates columns j+2, j+3
  // and goes straight on to the next pair — two workgroup barriers per pair of columns.
  double* beta = tmp;        // [m]
  double* s0v = tmp + m;     // [m]
  double* s1v = tmp + 2 * m; // [m] (tmp holds max(2 nw, 3 m) doubles)
  double* cpair = dw;        // [m / 2 + 1]: c_j of the pair starting at j (dw is free until the solve)
  const int wid = tid >> 6, lane = tid & 63;
  const int nwaves = KKT_THREADS >> 6;
  auto house = [&](int j) {
    double* x = QR + j * nw;
    const int i0 = j + 1 + lane, i1 = i0 + 64;
    const double x0 = i0 < nw ? x[i0] : 0.0, x1 = i1 < nw ? x[i1] : 0.0;
    const double sig = wave_sum(x0 * x0 + x1 * x1);
    const double alpha = x[j];
    if (sig == 0.0) {
      if (lane == 0) beta[j] = 0.0;  // R_jj = alpha stays on the diagonal
    } else {
      const double nrm = sqrt(alpha * alpha + sig);
      const double v0 = alpha <= 0.0 ? alpha - nrm : -sig / (alpha + nrm);
      const double rv0 = 1.0 / v0;
      if (i0 < nw) x[i0] = x0 * rv0;
      if (i1 < nw) x[i1] = x1 * rv0;
      if (lane == 0) { beta[j] = 2.0 * v0 * v0 / (sig + v0 * v0); x[j] = nrm; }  // R_jj on the diagonal
    }
  };
  auto house2 = [&](int j) {  // wave 0: reflectors j and j+1, c_j
    house(j);
    if (j + 1 >= m) return;
    const double* v = QR + j * nw;
    double* y = QR + (j + 1) * nw;
    const int i0 = j + 1 + lane, i1 = i0 + 64;
    const double p = wave_sum((i0 < nw ? v[i0] * y[i0] : 0.0) + (i1 < nw ? v[i1] * y[i1] : 0.0));
    const double sj = beta[j] * (y[j] + p);
    if (lane == 0) y[j] -= sj;
    if (i0 < nw) y[i0] -= sj * v[i0];
    if (i1 < nw) y[i1] -= sj * v[i1];
    house(j + 1);
    const double* v2 = QR + (j + 1) * nw;
    const int k0 = j + 2 + lane, k1 = k0 + 64;
    const double q = wave_sum((k0 < nw ? v[k0] * v2[k0] : 0.0) + (k1 < nw ? v[k1] * v2[k1] : 0.0));
    if (lane == 0) cpair[j >> 1] = v[j + 1] + q;
  };
  if (m > 0 && wid == 0) house2(0);
  __syncthreads();
  #pragma unroll 1
  for (int j = 0; j + 2 < m; j += 2) {
    const double b0 = beta[j], b1 = beta[j + 1], cj = cpair[j >> 1];
    const double* v0 = QR + j * nw;
    const double* v1 = QR + (j + 1) * nw;
    {  // both dots of columns k >= j+2, 8 lanes per column
      const int part = tid & 7;
      const int ncol = m - j - 2;
      for (int base = 0; base < ncol * 8; base += KKT_THREADS) {
        const int kk = (base + tid) >> 3;
        const bool act = kk < ncol;
        double a0 = 0.0, a1 = 0.0;
        const double* y = QR + (j + 2 + kk) * nw;
        if (act)
          for (int i = j + 2 + part; i < nw; i += 8) {
            const double yi = y[i];
            a0 += v0[i] * yi;
            a1 += v1[i] * yi;
          }
        a0 = group8_sum(a0);
        a1 = group8_sum(a1);
        if (act && part == 0) {
          const double yj = y[j], yj1 = y[j + 1];
          const double s0 = b0 * (yj + v0[j + 1] * yj1 + a0);
          s0v[j + 2 + kk] = s0;
          s1v[j + 2 + kk] = b1 * (yj1 + a1 - s0 * cj);
        }
      }
    }
    __syncthreads();
    // update rows i >= j of every later column: y_i -= s0 v0'_i + s1 v1'_i
    auto upd = [&](int k) {
      double* y = QR + k * nw;
      const double s0 = s0v[k], s1 = s1v[k];
      for (int i = j + lane; i < nw; i += 64) {
        const double w0 = i == j ? 1.0 : v0[i];
        const double w1 = i == j ? 0.0 : (i == j + 1 ? 1.0 : v1[i]);
        y[i] -= s0 * w0 + s1 * w1;
      }
    };
    if (wid == 0) {
      upd(j + 2);
      if (j + 3 < m) upd(j + 3);
      house2(j + 2);
    } else {
      // the other waves: column pairs j+2+2 wid, then every 2 (nwaves-1) columns — four columns
      // per pass with their loads issued together (the reflector weights of the lane's rows held
      // in registers), the same arithmetic as upd()
      const int i0 = j + lane, i1 = i0 + 64;
      const double w00 = i0 == j ? 1.0 : (i0 < nw ? v0[i0] : 0.0);
      const double w01 = i0 == j ? 0.0 : (i0 == j + 1 ? 1.0 : (i0 < nw ? v1[i0] : 0.0));
      const double w10 = i1 < nw ? v0[i1] : 0.0;
      const double w11 = i1 < nw ? v1[i1] : 0.0;
      const int step = 2 * (nwaves - 1);
#pragma unroll 1
      for (int kb = j + 2 + 2 * wid; kb < m; kb += 2 * step) {
        const int ks[4] = {kb, kb + 1, kb + step, kb + step + 1};
        double y0[4], y1[4], s0[4], s1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = ks[u] < m;
          const double* y = QR + ks[u] * nw;
          y0[u] = ok && i0 < nw ? y[i0] : 0.0;
          y1[u] = ok && i1 < nw ? y[i1] : 0.0;
          s0[u] = ok ? s0v[ks[u]] : 0.0;
          s1[u] = ok ? s1v[ks[u]] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (ks[u] < m) {
            double* y = QR + ks[u] * nw;
            if (i0 < nw) y[i0] = y0[u] - (s0[u] * w00 + s1[u] * w01);
            if (i1 < nw) y[i1] = y1[u] - (s0[u] * w10 + s1[u] * w11);
          }
        }
      }
    }
    __syncthreads();
  }
  KKT_MARK(1);
  // ---- Q = H_0 ... H_{m-1} I, backward, a pair of reflectors per pass (the QR's pairs): per
  // column q of Q, s1 = beta_{j+1} (q_{j+1} + v_{j+1}^T q), s0 = beta_j (q_j + v_j^T q - s1 c_j),
  // q -= s1 v_{j+1} + s0 v_j; 4 lanes per column; a lone last reflector (m odd) goes first.
  for (int i = tid; i < nw * nw; i += KKT_THREADS) Q[i] = (i / nw == i % nw) ? 1.0 : 0.0;
  __syncthreads();
  {
    const int part = tid & 3;
    int jtop = (m & 1) ? m - 1 : m;  // pairs (j, j+1) with j even below jtop
    if (m & 1) {
      const int j = m - 1;
      const double bj = beta[j];
      const double* v = QR + j * nw;
      for (int base = 0; base < (nw - j) * 4; base += KKT_THREADS) {
        const int c = j + ((base + tid) >> 2);  // columns c < j are still e_c: H_j leaves them
        const bool act = c < nw;
        double sv = 0.0;
        if (act) {
          if (part == 0) sv = Q[j * nw + c];
          for (int r = j + 1 + part; r < nw; r += 4) sv += v[r] * Q[r * nw + c];
        }
        sv = group4_sum(sv);
        sv *= bj;
        if (act) {
          if (part == 0) Q[j * nw + c] -= sv;
          for (int r = j + 1 + part; r < nw; r += 4) Q[r * nw + c] -= sv * v[r];
        }
      }
      __syncthreads();
    }
    #pragma unroll 1
    for (int j = jtop - 2; j >= 0; j -= 2) {
      const double b0 = beta[j], b1 = beta[j + 1], cj = cpair[j >> 1];
      const double* v0 = QR + j * nw;
      const double* v1 = QR + (j + 1) * nw;
      for (int base = 0; base < (nw - j) * 4; base += KKT_THREADS) {
        // columns c < j are still e_c (every reflector applied so far, and H_j, H_{j+1}, are zero
        // above their own row): only columns j .. nw-1 change
        const int c = j + ((base + tid) >> 2);
        const bool act = c < nw;
        double a0 = 0.0, a1 = 0.0;
        if (act)
          for (int r = j + 2 + part; r < nw; r += 4) {
            const double qr = Q[r * nw + c];
            a0 += v0[r] * qr;
            a1 += v1[r] * qr;
          }
        a0 = group4_sum(a0);
        a1 = group4_sum(a1);
        if (act) {
          const double qj = Q[j * nw + c], qj1 = Q[(j + 1) * nw + c];
          const double s1 = b1 * (qj1 + a1);
          const double s0 = b0 * (qj + v0[j + 1] * qj1 + a0 - s1 * cj);
          if (part == 0) {
            Q[j * nw + c] = qj - s0;
            Q[(j + 1) * nw + c] = qj1 - s1 - s0 * v0[j + 1];
          }
          for (int r = j + 2 + part; r < nw; r += 4) Q[r * nw + c] -= s1 * v1[r] + s0 * v0[r];
        }
      }
      __syncthreads();
    }
  }
  KKT_MARK(2);
  // ---- rank deficiency: delta_c on R's diagonal
  if (tid == 0) {
    double rmax = 0.0;
    for (int j = 0; j < m; ++j) rmax = fabs(QR[j * nw + j]) > rmax ? fabs(QR[j * nw + j]) : rmax;
    const double dc = 1e-8 * pow(*mub, 0.25) * (rmax > 0.0 ? rmax : 1.0);
    int def = 0;
    for (int j = 0; j < m; ++j)
      if (!(fabs(QR[j * nw + j]) >= 1e-10 * rmax) || rmax == 0.0) {
        double& rjj = QR[j * nw + j];
        rjj = rjj < 0.0 ? rjj - dc : rjj + dc;
        def = 1;
      }
    sh.rank_def = def;
    sh.delta_c = def ? dc : 0.0;
  }
  if (Pzg && nz > 0) {  // the augmented system: delta_w's shift of the reduced Hessian, Z[:nw0]^T Z[:nw0]
    for (int e = tid; e < nz * nz; e += KKT_THREADS) {
      const int a = e / nz, c = e - a * nz;
      Pzg[e] = lds_dot(Q + m + a, nw, Q + m + c, nw, nw0);
    }
  }
  __syncthreads();
  // ---- reduced Hessian Hr = Z^T (M Z), M Z staged in LDS or the global workspace
  double* Hr0 = L;  // keep the unshifted reduced Hessian in the workspace slot of L first
  if (nz > 0) {
    // LDS after tmp when it fits (kkt_mz_in_lds), else global scratch (the workspace; overwritten
    // at the end)
    double* MZ = kkt_mz_in_lds(nw, m) ? tmp + (2 * nw > 3 * m ? 2 * nw : 3 * m) : wsb;
    // MZ = M Z: a thread per (row r, 4 columns), M[r][k] from global once per k, Z[k][c..c+3] from
    // LDS (reads past Z's last column land inside the LDS image and are discarded)
    const int nb = (nz + 3) >> 2;
    #pragma unroll 1
    for (int t = tid; t < nw * nb; t += KKT_THREADS) {
      const int r = t / nb, cb = (t - r * nb) * 4;
      const double* mr = M + r * nw;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      #pragma unroll 1
      for (int k0 = 0; k0 < nw; k0 += 8) {  // eight global loads in flight, then the FMAs
        double mv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) mv[u] = k0 + u < nw ? mr[k0 + u] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (k0 + u < nw) {
            const double* zk = Q + (k0 + u) * nw + m + cb;
            a0 += mv[u] * zk[0];
            a1 += mv[u] * zk[1];
            a2 += mv[u] * zk[2];
            a3 += mv[u] * zk[3];
          }
        }
      }
      double* o = MZ + r * nz + cb;
      o[0] = a0;
      if (cb + 1 < nz) o[1] = a1;
      if (cb + 2 < nz) o[2] = a2;
      if (cb + 3 < nz) o[3] = a3;
    }
    __syncthreads();
    // Hr = Z^T (M Z): a thread per (row a, 4 columns), Z[r][a] from LDS, MZ[r][c..c+3] from global
    #pragma unroll 1
    for (int t = tid; t < nz * nb; t += KKT_THREADS) {
      const int ar = t / nb, cb = (t - ar * nb) * 4;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      const int w1 = cb + 1 < nz, w2 = cb + 2 < nz, w3 = cb + 3 < nz;
      #pragma unroll 1
      for (int r0 = 0; r0 < nw; r0 += 2) {  // eight global loads in flight, then the FMAs
        double mz[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const double* p = MZ + (r0 + u) * nz + cb;
          const bool ok = r0 + u < nw;
          mz[u][0] = ok ? p[0] : 0.0;
          mz[u][1] = ok && w1 ? p[1] : 0.0;
          mz[u][2] = ok && w2 ? p[2] : 0.0;
          mz[u][3] = ok && w3 ? p[3] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (r0 + u < nw) {
            const double zv = Q[(r0 + u) * nw + m + ar];
            a0 += zv * mz[u][0];
            a1 += zv * mz[u][1];
            a2 += zv * mz[u][2];
            a3 += zv * mz[u][3];
          }
        }
      }
      double* o = Hr0 + ar * nz + cb;
      o[0] = a0;
      if (cb + 1 < nz) o[1] = a1;
      if (cb + 2 < nz) o[2] = a2;
      if (cb + 3 < nz) o[3] = a3;
    }
    __syncthreads();
    // symmetrise, keep a copy in dw.. region (nz*nz may exceed it: use the global scratch again)
    double* Hsave = MZ;
    for (int e = tid; e < nz * nz; e += KKT_THREADS) {
      const int a = e / nz, c = e % nz;
      Hsave[e] = 0.5 * (Hr0[a * nz + c] + Hr0[c * nz + a]);
    }
    __syncthreads();
    KKT_MARK(3);
    // ---- inertia correction: Cholesky of Hr + delta_w I, IPOPT's delta_w schedule — wave 0 alone
    // (no workgroup barriers inside the retry loop; the other waves wait at the next barrier)
    if (tid < 64) {
      const double last = lastb ? *lastb : 0.0;
      double dW = 0.0;
      int32_t inf = 0;
      // a pivot at or below DBL_EPSILON max|M_ii| — the rounding level of Z^T M Z's entries, M
      // carrying barrier terms up to ~1e12 — counts as a zero eigenvalue (wrong inertia, as IPOPT
      // counts zero eigenvalues): numerically flat directions get delta_w, not an unbounded step
      double mmax = 0.0;
      for (int a = tid; a < nw; a += 64) mmax = fmax(mmax, fabs(M[a * nw + a]));
      mmax = wave_max(mmax);
      const double pivot_min = 2.220446049250313e-16 * mmax;
      #pragma unroll 1
      for (int attempt = 0; attempt < 64; ++attempt) {
        for (int e = tid; e < nz * nz; e += 64)
          L[e] = Hsave[e] + (Pzg ? dW * Pzg[e] : ((e / nz == e % nz) ? dW : 0.0));
        if (wave_cholesky(L, nz, pivot_min)) break;
        if (dW == 0.0) dW = last == 0.0 ? 1e-4 : fmax(1e-20, last / 3.0);
        else dW *= last == 0.0 ? 100.0 : 8.0;
        if (dW > 1e40) { inf = 1; break; }
      }
      if (tid == 0) {
        sh.delta_w = dW;
        if (infob) *infob = inf;
      }
    }
    __syncthreads();
  } else {
    if (tid == 0) { sh.delta_w = 0.0; if (infob) *infob = 0; }
    __syncthreads();
  }
  const double dW = sh.delta_w;
  KKT_MARK(4);
  // ---- solve, then one step of iterative refinement on the unregularised system
  kkt_solve_lds(nw, m, nw0, Q, QR, L, M, dW, q1, q2, dw, dy, tmp);
  KKT_MARK(5);
  if (!sh.rank_def) {
    // e1[r] is written and then updated by the same lane (group assignment depends on r only)
    group_dots<4>(nw, m, Ab, 1, nw, dy, 1, [&](int r, double d) { e1[r] = q1[r] - (r < nw0 ? dW * dw[r] : 0.0) - d; });
    group_dots<4>(nw, nw, M, nw, 1, dw, 1, [&](int r, double d) { e1[r] -= d; });
    group_dots<4>(m, nw, Ab, nw, 1, dw, 1, [&](int k, double d) { e2[k] = q2[k] - d; });
    __syncthreads();
    // refine only when the residual is above 1e-13 of the right-hand side (wave 0 decides)
    if (tid < 64) {
      double rmax = 0.0, qmax = 0.0;
      for (int r = tid; r < nw; r += 64) { rmax = fmax(rmax, fabs(e1[r])); qmax = fmax(qmax, fabs(q1[r])); }
      for (int k = tid; k < m; k += 64) { rmax = fmax(rmax, fabs(e2[k])); qmax = fmax(qmax, fabs(q2[k])); }
      rmax = wave_max(rmax);
      qmax = wave_max(qmax);
      if (tid == 0) sh.flag = !(rmax <= 1e-13 * qmax);
    }
    __syncthreads();
    if (sh.flag) {
      // the correction (e1, e2) -> (c1, c2), global scratch
      kkt_solve_lds(nw, m, nw0, Q, QR, L, M, dW, e1, e2, c1, c2, tmp);
      for (int r = tid; r < nw; r += KKT_THREADS) dw[r] += c1[r];
      for (int k = tid; k < m; k += KKT_THREADS) dy[k] += c2[k];
      __syncthreads();
    }
  }
  KKT_MARK(6);
  for (int i = tid; i < nw0; i += KKT_THREADS) dwo[i] = dw[i];
  for (int i = tid; i < m; i += KKT_THREADS) dyo[i] = dy[i];
  if (tid == 0) { *dWo = dW; *dCo = sh.delta_c; }
  // keep the factors for mode 1 (the global scratch use above is finished: barrier first)
  __syncthreads();
  const int64_t per = kkt_ws_per(nw, m);
  for (int64_t i = tid; i < per - 4; i += KKT_THREADS) wsb[i] = sm[i];
  if (tid == 0) { wsb[per - 4] = dW; wsb[per - 3] = sh.delta_c; wsb[per - 2] = 0.0; wsb[per - 1] = 0.0; }
  KKT_MARK(7);
}

template <int NW, int MM>
__global__ __launch_bounds__(KKT_THREADS) __attribute__((amdgpu_waves_per_eu(5, 8))) void cpl_kkt_kernel(
    int mode, int64_t batch, int nw_arg, int m_arg, const double* __restrict__ Mg, const double* __restrict__ Ag,
    const double* __restrict__ r1g, const double* __restrict__ r2g, const double* __restrict__ mug,
    const double* __restrict__ dw_last, const uint8_t* __restrict__ active, double* __restrict__ dwg,
    double* __restrict__ dyg, double* __restrict__ dWg, double* __restrict__ dCg, int32_t* __restrict__ info,
    double* __restrict__ ws) {
  extern __shared__ __align__(16) double sm[];
  __shared__ KktShared sh;
  const int nw = NW > 0 ? NW : nw_arg;
  const int m = NW > 0 ? MM : m_arg;
  const int64_t b = blockIdx.x;
  if (b >= batch) return;
  const int tid = threadIdx.x;
  if (active && !active[b]) {
    for (int i = tid; i < nw; i += KKT_THREADS) dwg[b * nw + i] = 0.0;
    for (int i = tid; i < m; i += KKT_THREADS) dyg[b * m + i] = 0.0;
    if (tid == 0 && mode == 0) { dWg[b] = 0.0; dCg[b] = 0.0; info[b] = 0; }
    return;
  }
  kkt_block<NW, MM>(mode, nw, m, nw, Mg + b * nw * nw, Ag + b * m * nw, r1g + b * nw, r2g + b * m,
                    mug ? mug + b : nullptr, dw_last ? dw_last + b : nullptr, dwg + b * nw, dyg + b * m,
                    dWg ? dWg + b : nullptr, dCg ? dCg + b : nullptr, info ? info + b : nullptr,
                    ws + b * kkt_ws_per(nw, m), nullptr, nullptr, sm, sh);
}

// IPOPT's regularisation of a rank-deficient Jacobian (cpl_solve_options.jacobian_regularization;
// IpPDPerturbationHandler: delta_c = jacobian_regularization_value 1e-8 * mu^jacobian_regularization_
// exponent 0.25 on the (2,2) block): [[W + dW I, A^T], [A, -delta_c I]] solved by the same null-space
// method as the augmented system in (dw, s), W~ = diag(W, I), A~ = [A, -sqrt(delta_c) I] (full row
// rank), whose KKT conditions are exactly the regularised system's (s = sqrt(delta_c) dy) — the
// restatements' form (oracle/cpl_solve_host.c kkt_factor with cplo_set_jac_reg, batch_ipm.py kkt_host).
// Launched after the factorisation kernel of the same call (either kernel marks a rank-deficient
// system by its delta_c != 0, its R-pivot treatment): the marked systems only, mode 0 re-factorising
// them in the augmented form and overwriting dw, dy, delta_w (delta_c := IPOPT's), mode 1 re-solving
// with the augmented factors (and, like the factorisation, one step of iterative refinement — the
// restatements refine every full-rank re-solve).  Workspace per system: KktAugLayout (cpl_kkt_block.hpp;
// the fused search kernel re-solves there on one wave, kkt_aug_resolve_wave).

__global__ __launch_bounds__(KKT_THREADS) void cpl_kkt_aug_kernel(
    int mode, int64_t batch, int nw, int m, const double* __restrict__ Mg, const double* __restrict__ Ag,
    const double* __restrict__ r1g, const double* __restrict__ r2g, const double* __restrict__ mug,
    const double* __restrict__ dw_last, const uint8_t* __restrict__ active, double* __restrict__ dwg,
    double* __restrict__ dyg, double* __restrict__ dWg, double* __restrict__ dCg, int32_t* __restrict__ info,
    double* __restrict__ wsa) {
  extern __shared__ __align__(16) double sm[];
  __shared__ KktShared sh;
  const int64_t b = blockIdx.x;
  if (b >= batch || (active && !active[b]) || dCg[b] == 0.0) return;
  const int na = nw + m, tid = threadIdx.x;
  const KktAugLayout Lo(nw, m);
  double* wsb = wsa + b * Lo.per;
  double* Ma = wsb + Lo.Ma;
  double* Aa = wsb + Lo.Aa;
  double* q1a = wsb + Lo.q1a;
  double* Pz = wsb + Lo.Pz;
  double* rscr = wsb + Lo.rscr;
  if (mode == 0) {
    const double* M = Mg + b * nw * nw;
    const double* A = Ag + b * m * nw;
    const double sdc = sqrt(1e-8 * pow(mug[b], 0.25));
    for (int e = tid; e < na * na; e += KKT_THREADS) {
      const int r = e / na, c = e - r * na;
      Ma[e] = (r < nw && c < nw) ? M[r * nw + c] : (r == c ? 1.0 : 0.0);
    }
    for (int e = tid; e < m * na; e += KKT_THREADS) {
      const int r = e / na, c = e - r * na;
      Aa[e] = c < nw ? A[r * nw + c] : (c - nw == r ? -sdc : 0.0);
    }
  }
  for (int i = tid; i < na; i += KKT_THREADS) q1a[i] = i < nw ? r1g[b * nw + i] : 0.0;
  __syncthreads();
  kkt_block<0, 0>(mode, na, m, nw, Ma, Aa, q1a, r2g + b * m, mug ? mug + b : nullptr,
                  dw_last ? dw_last + b : nullptr, dwg + b * nw, dyg + b * m, dWg ? dWg + b : nullptr, dCg + b,
                  info ? info + b : nullptr, wsb, Pz, mode == 1 ? rscr : nullptr, sm, sh);
  if (mode == 0 && tid == 0) dCg[b] = 1e-8 * pow(mug[b], 0.25);  // (stays != 0: the mark for mode 1)
}

// grad f + J^T y per instance from the CSR values (the Lagrangian gradient the solve loop
// differentiates for its Hessian): one thread per (instance, column), the column's entries through
// a host-built CSC index of the fixed structure.  Instance b takes the multipliers of instance
// b / y_repeat (the 2 n_free finite-difference points of one iterate share its y).  A NaN Jacobian
// value (a cone at zero tangential force, 0/0) counts as 0.
__global__ __launch_bounds__(256) void cpl_lagrangian_grad_kernel(int64_t total, int n, int m, int nnz,
                                                                  const int32_t* __restrict__ col_ptr,
                                                                  const int32_t* __restrict__ csc_k,
                                                                  const int32_t* __restrict__ csc_row,
                                                                  const double* __restrict__ grad,
                                                                  const double* __restrict__ jac,
                                                                  const double* __restrict__ y, int y_repeat,
                                                                  double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int64_t b = e / n;
  const int j = (int)(e - b * n);
  const double* jb = jac + b * nnz;
  const double* yb = y + (b / y_repeat) * m;
  double s = grad[e];
  for (int q = col_ptr[j]; q < col_ptr[j + 1]; ++q) {
    double v = jb[csc_k[q]];
    v = v == v ? v : 0.0;
    s += v * yb[csc_row[q]];
  }
  out[e] = s;
}


// sum_{k < K} a[k * stride] * v[k] (a in global memory, v in LDS): the loads issued 16 at a time
// before their FMAs (one L2 round trip per 16 terms, 32 VGPRs in flight)
template <int K>
__device__ __forceinline__ double col_dot_u(const double* a, int stride, const double* v, int vstride = 1) {
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  #pragma unroll 1
  for (int k0 = 0; k0 < K; k0 += 16) {
    double av[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) av[u] = k0 + u < K ? a[(k0 + u) * stride] : 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (k0 + u < K) s[u & 3] += av[u] * v[(k0 + u) * vstride];
  }
  return (s[0] + s[1]) + (s[2] + s[3]);
}




// W4: Z's accumulation and the reflector pairs' c_p on the workgroup's four waves (small batches: the
// GPU is idle but for the few systems) — Z's 16 register-resident columns on wave 0, its 17th (a full
// wave sum per reflector on the one-wave kernel's critical path) on wave 1, the c_p on waves 2 and 3;
// the QR before and everything after on wave 0, as the one-wave kernel: the same factors and steps bit
// for bit (scripts/r6_kkt_w4_probe.sh: one system 63 -> 60 us, Z 28k -> 20k cycles).
template <int NW, int MM, bool W4 = false>
__global__ __launch_bounds__(W4 ? 256 : 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void cpl_kkt_wave_kernel(
    int mode, int64_t batch, const double* __restrict__ Mg, const double* __restrict__ Ag,
    const double* __restrict__ r1g, const double* __restrict__ r2g, const double* __restrict__ mug,
    const double* __restrict__ dw_last, const uint8_t* __restrict__ active, double* __restrict__ dwg,
    double* __restrict__ dyg, double* __restrict__ dWg, double* __restrict__ dCg, int32_t* __restrict__ info,
    double* __restrict__ ws) {
  using W = KktWave<NW, MM>;
  constexpr int NZ = W::NZ, ZS = W::ZS, NP = W::NP, NFAC = W::NFAC;
  extern __shared__ __align__(16) double sm[];
  const int lane = threadIdx.x & 63;
  const int wid = W4 ? (int)(threadIdx.x >> 6) : 0;
  const int64_t b = blockIdx.x;
  if (b >= batch) return;
  double* QR = sm;                 // [MM][NW]
  double* Z = QR + MM * NW;        // [NW][ZS]
  double* L = Z + NW * ZS;         // [NLP]: the lower triangle packed by rows
  double* beta = L + W::NLP;       // [MM]
  double* cp = beta + MM;          // [NP + 1]
  double* s1 = sm + NFAC;          // [NW] scratch
  double* s2 = s1 + NW;            // [NW] scratch
  // the refinement's broadcast copies of dw and dy share the scratch slots (dy is read before the M dw
  // product writes s1, dw is not written by it)
  double* dwl = s2;                // [NW] dw (broadcast copy)
  double* dyl = s1;                // [MM] dy (broadcast copy)
  const double* M = Mg + b * NW * NW;
  const double* Ab = Ag + b * MM * NW;
  double* wsb = ws + b * kkt_ws_per(NW, MM);
  const bool rw = lane < NW;
  const int lc = rw ? lane : 0;
  const double q1v = rw ? r1g[b * NW + lane] : 0.0;
  const double q2v = lane < MM ? r2g[b * MM + lane] : 0.0;

  if (active && !active[b]) {
    if (wid != 0) return;
    if (rw) dwg[b * NW + lane] = 0.0;
    if (lane < MM) dyg[b * MM + lane] = 0.0;
    if (lane == 0 && mode == 0) { dWg[b] = 0.0; dCg[b] = 0.0; info[b] = 0; }
    return;
  }
  if (mode == 1) {  // re-solve with the kept factors
    if (wid != 0) return;
    double dwv, dyv;
    kkt_wave_resolve<NW, MM>(M, wsb, q1v, q2v, sm, &dwv, &dyv);
    if (rw) dwg[b * NW + lane] = dwv;
    if (lane < MM) dyg[b * MM + lane] = dyv;
    return;
  }

  // ---- Householder QR of A^T with the matrix register-resident: lane (g = lane >> 3, part =
  // lane & 7) holds A^T[i][k] for the rows i = part + 8t and the columns k = g + 8q.  Per column j
  // the 8 lanes of group j & 7 form the reflector (a group sum, two broadcasts) and publish its
  // entries through a 47-double LDS buffer; every trailing column's dot is a group sum and its
  // update stays in registers — 2 x 6 LDS operations per column instead of ~50.
  if (!W4 || wid == 0) {  // (W4: the QR on wave 0 — its column blocks on four waves measured no faster,
                          // the reflectors' scalar chain is its critical path)
    constexpr int RT = (NW + 7) / 8;  // row blocks per lane
    constexpr int CQ = (MM + 7) / 8;  // column blocks per lane
    const int g = lane >> 3, part = lane & 7;
    double a[CQ][RT];
#pragma unroll
    for (int q = 0; q < CQ; ++q)
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const int k = g + 8 * q, i = part + 8 * t;
        a[q][t] = (k < MM && i < NW) ? Ab[k * NW + i] : 0.0;
      }
    double* vbuf = s1;  // [NW] the current reflector's entries
    KKT_MARK(0);
    // column j = 8 QB + jj: its entries sit in block QB of group jj (rows block QB holds row j, at
    // lane 9 jj), and the blocks q < QB (finished columns) and t < QB (rows above j) are skipped —
    // compile-time per QB
    auto step = [&](auto qbc, int jj) {
      constexpr int QB = decltype(qbc)::value;
      const int j = 8 * QB + jj;
      const double* c = a[QB];
      // sigma = sum_{i > j} x_i^2 (a group sum), alpha = x_j (lane 9 jj)
      double ps = 0.0;
#pragma unroll
      for (int t = QB; t < RT; ++t) {
        const int i = part + 8 * t;
        if (i > j && i < NW) ps += c[t] * c[t];
      }
      ps = group8_sum(ps);
      const double sig = wave_bcast(ps, 9 * jj);
      const double alpha = wave_bcast(c[QB], 9 * jj);
      // the reflector (LAPACK's dlarfg form): nrm = sqrt(alpha^2 + sigma), v0 = alpha - nrm
      // (cancellation-free when alpha > 0), beta = 2 v0^2 / (sigma + v0^2)
      double bj = 0.0, rv0 = 0.0, nrm = alpha;
      if (sig != 0.0) {
        nrm = sqrt(alpha * alpha + sig);
        const double v0 = alpha <= 0.0 ? alpha - nrm : -sig / (alpha + nrm);
        rv0 = 1.0 / v0;
        bj = 2.0 * v0 * v0 / (sig + v0 * v0);
      }
      if (lane == 0) beta[j] = bj;
      if (g == jj) {  // R_jj and the scaled reflector entries (zero when sigma = 0), kept and published
#pragma unroll
        for (int t = QB; t < RT; ++t) {
          const int i = part + 8 * t;
          if (i < NW && i >= j) {
            const double nv = i == j ? nrm : (sig != 0.0 ? a[QB][t] * rv0 : a[QB][t]);
            if (i > j) vbuf[i] = nv;
            a[QB][t] = nv;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (bj != 0.0 && j + 1 < MM) {
        double vl[RT];
#pragma unroll
        for (int t = QB; t < RT; ++t) {
          const int i = part + 8 * t;
          vl[t] = (i > j && i < NW) ? vbuf[i] : (i == j ? 1.0 : 0.0);
        }
        double d[CQ];
#pragma unroll
        for (int q = QB; q < CQ; ++q) {
          d[q] = 0.0;
#pragma unroll
          for (int t = QB; t < RT; ++t) d[q] += vl[t] * a[q][t];
        }
#pragma unroll
        for (int q = QB; q < CQ; ++q) {
          const int k = g + 8 * q;
          const double sk = bj * group8_sum(d[q]);
          if (k > j && k < MM) {
#pragma unroll
            for (int t = QB; t < RT; ++t) a[q][t] -= sk * vl[t];
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    };
    static_assert(CQ <= 4, "nw 47, m <= 32");
    #pragma unroll 1
    for (int jj = 0; jj < 8; ++jj) step(std::integral_constant<int, 0>(), jj);
    if constexpr (CQ > 1) {
      #pragma unroll 1
      for (int jj = 0; jj < 8 && 8 + jj < MM; ++jj) step(std::integral_constant<int, 1>(), jj);
    }
    if constexpr (CQ > 2) {
      #pragma unroll 1
      for (int jj = 0; jj < 8 && 16 + jj < MM; ++jj) step(std::integral_constant<int, 2>(), jj);
    }
    if constexpr (CQ > 3) {
      #pragma unroll 1
      for (int jj = 0; jj < 8 && 24 + jj < MM; ++jj) step(std::integral_constant<int, 3>(), jj);
    }
    // the factored matrix into the LDS image (row k of QR = column k of A^T after the reflections)
#pragma unroll
    for (int q = 0; q < CQ; ++q)
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const int k = g + 8 * q, i = part + 8 * t;
        if (k < MM && i < NW) QR[k * NW + i] = a[q][t];
      }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (W4) __syncthreads();
  KKT_MARK(1);
  // c_p = v_{2p}^T v_{2p+1} for the paired chains (lane p keeps c_p; W4: waves 2 and 3, beside Z)
  if constexpr (W4) {
    if (wid >= 2) {
      #pragma unroll 1
      for (int p = wid - 2; p < NP; p += 2) {
        const double c = wave_sum(refl_entry<NW>(QR, 2 * p) * refl_entry<NW>(QR, 2 * p + 1));
        if (lane == 0) cp[p] = c;
      }
    }
  } else {
    double cl = 0.0;
    #pragma unroll 1
    for (int p = 0; p < NP; ++p) {
      const double c = wave_sum(refl_entry<NW>(QR, 2 * p) * refl_entry<NW>(QR, 2 * p + 1));
      if (lane == p) cl = c;
    }
    if (lane < NP) cp[lane] = cl;
  }
  // ---- Z = H_0 ... H_{m-1} [0; I], register-resident: lane (c = lane >> 2, part = lane & 3) holds
  // Z[i][c] for the rows i = part + 4t of column c < 16, the columns past 16 a row per lane; per
  // reflector (backward) a group-of-4 sum per column, the next reflector's entries loaded one step
  // ahead.  Rows < j of Z are still zero at step j.  (W4: wave 0 the 16 columns, wave 1 the rest.)
  if (!W4 || wid < 2) {
    const bool zmain = !W4 || wid == 0, zextra = !W4 || wid == 1;
    constexpr int ZT = (NW + 3) / 4;
    constexpr int NZX = NZ > 16 ? NZ - 16 : 0;
    const int c16 = lane >> 2, part = lane & 3;
    double z[ZT];
#pragma unroll
    for (int t = 0; t < ZT; ++t) {
      const int i = part + 4 * t;
      z[t] = (c16 < NZ && i == MM + c16) ? 1.0 : 0.0;
    }
    double zx[NZX > 0 ? NZX : 1];
#pragma unroll
    for (int c = 0; c < NZX; ++c) zx[c] = lane == MM + 16 + c ? 1.0 : 0.0;
    auto load_refl = [&](int j, double (&vl)[ZT], double& vx) {
#pragma unroll
      for (int t = 0; t < ZT; ++t) {
        const int i = part + 4 * t;
        vl[t] = (i > j && i < NW) ? QR[j * NW + i] : (i == j ? 1.0 : 0.0);
      }
      vx = NZX > 0 ? refl_entry<NW>(QR, j) : 0.0;
    };
    double vl[ZT], vx;
    load_refl(MM - 1, vl, vx);
    double bj = beta[MM - 1];
    // reflector j = 4 JB + jj (backward): rows below 4 JB are still zero, so the row blocks t < JB
    // are skipped — compile-time per JB
    auto zstep = [&](auto jbc, int j) {
      constexpr int JB = decltype(jbc)::value;
      double nl[ZT], nx = 0.0, nb = 0.0;
      if (j > 0) {
        load_refl(j - 1, nl, nx);
        nb = beta[j - 1];
      }
      if (bj != 0.0) {
        if (zmain) {
          double d0 = 0.0, d1 = 0.0;
#pragma unroll
          for (int t = JB; t < ZT; t += 2) {
            d0 += vl[t] * z[t];
            if (t + 1 < ZT) d1 += vl[t + 1] * z[t + 1];
          }
          const double sc = bj * group4_sum(d0 + d1);
          if (c16 < NZ) {
#pragma unroll
            for (int t = JB; t < ZT; ++t) z[t] -= sc * vl[t];
          }
        }
        if (zextra) {
#pragma unroll
          for (int c = 0; c < NZX; ++c) zx[c] -= bj * wave_sum(vx * zx[c]) * vx;
        }
      }
#pragma unroll
      for (int t = 0; t < ZT; ++t) vl[t] = j > 0 ? nl[t] : 0.0;
      vx = nx;
      bj = nb;
    };
    static_assert((MM + 3) / 4 <= 8, "m <= 32");
    auto zblock = [&](auto jbc) {
      constexpr int JB = decltype(jbc)::value;
      if constexpr (4 * JB < MM) {
        #pragma unroll 1
        for (int j = (4 * JB + 3 < MM ? 4 * JB + 3 : MM - 1); j >= 4 * JB; --j) zstep(jbc, j);
      }
    };
    zblock(std::integral_constant<int, 7>());
    zblock(std::integral_constant<int, 6>());
    zblock(std::integral_constant<int, 5>());
    zblock(std::integral_constant<int, 4>());
    zblock(std::integral_constant<int, 3>());
    zblock(std::integral_constant<int, 2>());
    zblock(std::integral_constant<int, 1>());
    zblock(std::integral_constant<int, 0>());
    if (zmain && c16 < NZ && c16 < 16) {
#pragma unroll
      for (int t = 0; t < ZT; ++t) {
        const int i = part + 4 * t;
        if (i < NW) Z[i * ZS + c16] = z[t];
      }
    }
    if (zextra && lane < NW) {
#pragma unroll
      for (int c = 0; c < NZX; ++c) Z[lane * ZS + 16 + c] = zx[c];
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (W4) {  // Z and c_p complete; wave 0 goes on alone
    __syncthreads();
    if (wid != 0) return;
  }
  KKT_MARK(2);
  // ---- rank deficiency: delta_c on R's diagonal
  double dC = 0.0;
  bool rank_def = false;
  {
    const double rjj = lane < MM ? QR[lane * NW + lane] : 0.0;
    const double rmax = wave_max(fabs(rjj));
    const bool defl = lane < MM && (!(fabs(rjj) >= 1e-10 * rmax) || rmax == 0.0);
    rank_def = __ballot(defl) != 0ull;
    if (rank_def) {
      const double dc = 1e-8 * pow(mug[b], 0.25) * (rmax > 0.0 ? rmax : 1.0);
      if (defl) QR[lane * NW + lane] = rjj < 0.0 ? rjj - dc : rjj + dc;
      dC = dc;
    }
    __builtin_amdgcn_wave_barrier();
  }
  // ---- reduced Hessian Hr = Z^T (M Z): M Z a lane per row through the global workspace (L2),
  // Hr's upper triangle a lane per entry, into L's packed lower triangle; the Cholesky keeps the unshifted rows in
  // registers for its delta_w retries
  double dW = 0.0;
  int32_t inf = 0;
  double Mf[MFrag<NW>::RB][MFrag<NW>::KB];  // M's MFMA fragments: Z^T M Z here, every M product later
  load_m_frags<NW>(M, Mf);
  if constexpr (NZ > 0) {
    // W = M Z and Hr = Z^T W on the FP64 matrix cores (v_mfma_f64_16x16x4f64: A lane l = A[l & 15]
    // [k = l >> 4], B lane l = B[k = l >> 4][l & 15], D lane l reg q = D[(l >> 4) + 4q][l & 15]),
    // padded to 16-row / 16-column tiles and 4-deep k-steps.  W's accumulator register q of row
    // block kb / 4 is exactly Hr's B fragment of k-step kb, so W never leaves the registers; Z^T's
    // A fragment of k-step kb is Z's B fragment.  Hr's upper triangle goes to L's packed lower triangle.
    static_assert(NW <= 48 && NZ <= 32, "MFMA tiling of Z^T M Z: nw <= 48, nz <= 32");
    constexpr int KB = (NW + 3) / 4;    // k-steps
    constexpr int RB = (NW + 15) / 16;  // row blocks of W
    constexpr int CB = (NZ + 15) / 16;  // column blocks of W / Hr
    typedef double f64x4 __attribute__((ext_vector_type(4)));
    const int li = lane & 15, lk = lane >> 4;
    double Zf[KB][CB];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int k = 4 * kb + lk, c = 16 * cb + li;
        Zf[kb][cb] = (k < NW && c < NZ) ? Z[k * ZS + c] : 0.0;
      }
    f64x4 W[RB][CB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Mf[rb][kb], Zf[kb][cb], acc, 0, 0, 0);
        W[rb][cb] = acc;
      }
    }
#pragma unroll
    for (int ab = 0; ab < CB; ++ab)
#pragma unroll
      for (int cb = ab; cb < CB; ++cb) {
        f64x4 h = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) h = __builtin_amdgcn_mfma_f64_16x16x4f64(Zf[kb][ab], W[kb / 4][cb][kb % 4], h, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ar = 16 * ab + lk + 4 * q, c = 16 * cb + li;
          if (ar < NZ && c < NZ && ar <= c) L[c * (c + 1) / 2 + ar] = h[q];  // Hr(c, ar), c >= ar
        }
      }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    KKT_MARK(3);
    // ---- inertia correction: Cholesky of Hr + delta_w I, IPOPT's delta_w schedule (as the
    // workgroup kernel: pivots at or below DBL_EPSILON max|M_ii| count as zero)
    const double last = dw_last ? dw_last[b] : 0.0;
    const double mmax = wave_max(rw ? fabs(M[lane * NW + lane]) : 0.0);
    const double pivot_min = 2.220446049250313e-16 * mmax;
    // the lane's row of Hr in registers (from the L image just written), the factor in place
    const int lr = lane < NZ ? lane : 0;
    double hs[NZ], a[NZ];
#pragma unroll
    for (int c = 0; c < NZ; ++c) hs[c] = c <= lr ? L[lr * (lr + 1) / 2 + c] : L[c * (c + 1) / 2 + lr];
    #pragma unroll 1
    for (int attempt = 0; attempt < 64; ++attempt) {
#pragma unroll
      for (int c = 0; c < NZ; ++c) a[c] = lane < NZ ? hs[c] + (c == lane ? dW : 0.0) : 0.0;
      if (wave_cholesky_reg<NZ>(a, pivot_min)) break;
      if (dW == 0.0) dW = last == 0.0 ? 1e-4 : fmax(1e-20, last / 3.0);
      else dW *= last == 0.0 ? 100.0 : 8.0;
      if (dW > 1e40) { inf = 1; break; }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < NZ) {
#pragma unroll
      for (int c = 0; c < NZ; ++c)
        if (c <= lane) L[lane * (lane + 1) / 2 + c] = a[c];
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0 && info) info[b] = inf;
  KKT_MARK(4);
  // ---- solve, then one step of iterative refinement on the unregularised system (one inlined
  // copy of the solve: pass 1 solves for the correction of pass 0's residual)
  double dwv = 0.0, dyv = 0.0;
  double r1v = q1v, r2v = q2v;
  #pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    double c1, c2;
    wave_null_solve_t<NW, MM>(QR, Z, L, beta, cp, Mf, dW, r1v, r2v, s1, s2, &c1, &c2);
    if (pass == 0) {
      dwv = c1;
      dyv = c2;
    } else {
      dwv += c1;
      dyv += c2;
    }
    KKT_MARK(5);
    if (pass == 1 || rank_def) break;
    if (rw) dwl[lane] = dwv;
    if (lane < MM) dyl[lane] = dyv;
    __builtin_amdgcn_wave_barrier();
    // e1 = q1 - dW dw - A^T dy - M dw,  e2 = q2 - A dw
    const double aty = col_dot_u<MM>(Ab + lc, NW, dyl);
    const double mdw = mfma_matvec<NW>(Mf, dwl, s1);
    const double e1 = rw ? q1v - dW * dwv - aty - mdw : 0.0;
    const double adw = col_dot_u<NW>(Ab + (lane < MM ? lane : 0) * NW, 1, dwl);
    const double e2 = lane < MM ? q2v - adw : 0.0;
    const double rmax = wave_max(fmax(fabs(e1), fabs(e2)));
    const double qmax = wave_max(fmax(fabs(q1v), fabs(q2v)));
    if (rmax <= 1e-13 * qmax) break;  // refine only above 1e-13 of the right-hand side
    r1v = e1;
    r2v = e2;
    __builtin_amdgcn_wave_barrier();
  }
  KKT_MARK(6);
  if (rw) dwg[b * NW + lane] = dwv;
  if (lane < MM) dyg[b * MM + lane] = dyv;
  if (lane == 0) { dWg[b] = dW; dCg[b] = dC; }
  // keep the factors for mode 1 (every scratch read above is done: same wave, program order)
  __threadfence_block();
  for (int i = lane; i < NFAC; i += 64) wsb[i] = sm[i];
  if (lane == 0) { wsb[NFAC] = dW; wsb[NFAC + 1] = dC; }
  KKT_MARK(7);
}


// ---- the restoration phase's Newton system (quasi-definite): cpl_kkt_qd.hpp ----------------
__global__ __launch_bounds__(KKT_THREADS) void cpl_kkt_qd_kernel(
    int64_t batch, int nw, int m, const double* __restrict__ W, const double* __restrict__ A,
    const double* __restrict__ Dinv, const double* __restrict__ r1, const double* __restrict__ r2,
    const uint8_t* __restrict__ active, double* __restrict__ dwl, double* __restrict__ dw_out,
    double* __restrict__ dy_out, double* __restrict__ delta_w_out, double* __restrict__ Kws) {
  const int64_t b = blockIdx.x;
  if (b >= batch || (active && !active[b])) return;
  extern __shared__ __align__(16) double qd_lds[];
  qd_solve_block<KKT_THREADS>(b, nw, m, W, A, Dinv, r1, r2, dwl, dw_out, dy_out, delta_w_out, Kws, qd_lds);
}

}  // namespace cpl

using namespace cpl;

using KktKernel = void (*)(int, int64_t, int, int, const double*, const double*, const double*, const double*,
                          const double*, const double*, const uint8_t*, double*, double*, double*, double*, int32_t*,
                          double*);

// The size-specialised instance for the solve loop's 4-contact systems (nw 47, m 30: Ground /
// Superquadric with an environment), the generic one otherwise.
static inline KktKernel kkt_kernel_for(int nw, int m) {
  if (nw == 47 && m == 30) return cpl_kkt_kernel<47, 30>;
  return cpl_kkt_kernel<0, 0>;
}
using KktWaveKernel = void (*)(int, int64_t, const double*, const double*, const double*, const double*,
                              const double*, const double*, const uint8_t*, double*, double*, double*, double*,
                              int32_t*, double*);

// The one-wave kernel for the sizes it is specialised for (the 4-contact solve loop's nw 47, m 30),
// nullptr otherwise.  With its register-resident QR / Z and the FP64-MFMA reduced Hessian it
// factorises faster than the workgroup kernel at every batch size (scripts/kkt_ab.hip,
// profiles/r2_v7/kkt_ab/: 1 system 0.069 vs 0.099 ms, 1 024 0.080 vs 0.134, 8 192 0.42 vs 0.94);
// its re-solve is 4-7 us slower up to ~1 000 systems, less than the factorisation gains, so the
// choice depends on the system size only: every batch size, the single-instance Solve() included,
// runs the same kernel and an instance's iterates do not depend on the batch it is solved in
// (tests/test_gpu_solve_engine.py: B = 1 vs inside B = 64).  CPL_KKT_KERNEL=block or =wave forces
// one (measurement only).
// batches up to this size factorise on four waves per system (cpl_kkt_wave_kernel<.., true>): the same
// factors bit for bit, the QR's column blocks in parallel (CPL_KKT_W4=0 / 1: never / always; measurement)
constexpr int64_t KKT_W4_MAX = 256;
static bool kkt_use_w4(int64_t batch) {
  static const int forced = [] {
    const char* e = std::getenv("CPL_KKT_W4");
    return e ? (std::string(e) == "1" ? 1 : 0) + (std::string(e) == "0" ? 2 : 0) : 0;
  }();
  return forced == 1 || (forced == 0 && batch <= KKT_W4_MAX);
}
static KktWaveKernel kkt_wave_kernel_for(int nw, int m) {
  static const int forced = [] {
    const char* e = std::getenv("CPL_KKT_KERNEL");
    if (!e) return 0;
    return std::string(e) == "block" ? 1 : (std::string(e) == "wave" ? 2 : 0);
  }();
  KktWaveKernel wk = nullptr;
  if (nw == 47 && m == 30) wk = cpl_kkt_wave_kernel<47, 30>;
  if (!wk || forced == 1) return nullptr;
  return wk;
}

// the system size runs the one-wave kernel (whose factors the fused line-search kernel re-solves with)
namespace cpl {
bool kkt_wave_size(int nw, int m) { return kkt_wave_kernel_for(nw, m) != nullptr; }

// IPOPT's Jacobian regularisation (cpl_kkt_aug_kernel): its workspace doubles per system, or -1 when
// the augmented system (nw + m unknowns) exceeds the workgroup kernel (128 unknowns, one LDS image)
int64_t kkt_aug_workspace_doubles(int nw, int m) {
  const int na = nw + m;
  if (nw <= 0 || m < 0 || m > nw || na > KKT_MAX_NW) return -1;
  if (sizeof(double) * (size_t)kkt_launch_lds_doubles(na, m, 0) > 160 * 1024) return -1;
  return kkt_aug_ws_per(nw, m);
}

// the marked (delta_c != 0) systems of the cpl_kkt_solve call just issued with the same arguments,
// re-factorised (mode 0) or re-solved (mode 1) in IPOPT's regularised form
int32_t kkt_aug_solve(int mode, int64_t batch, int nw, int m, const double* d_M, const double* d_A, const double* d_r1,
                      const double* d_r2, const double* d_mu, const double* d_dwl, const uint8_t* d_active, double* d_dw,
                      double* d_dy, double* d_delta_w, double* d_delta_c, int32_t* d_info, double* d_wsa,
                      hipStream_t st) {
  if (batch == 0) return CPL_OK;
  if (kkt_aug_workspace_doubles(nw, m) < 0 || !d_delta_c || !d_wsa || (mode == 0 && (!d_mu || !d_delta_w)))
    return fail(CPL_ERR_INVALID_ARGUMENT, "kkt_aug_solve: bad arguments");
  const size_t lds = sizeof(double) * (size_t)kkt_launch_lds_doubles(nw + m, m, mode);
  hipLaunchKernelGGL(cpl_kkt_aug_kernel, dim3((unsigned)batch), dim3(KKT_THREADS), lds, st, mode, batch, nw, m, d_M,
                     d_A, d_r1, d_r2, d_mu, d_dwl, d_active, d_dw, d_dy, d_delta_w, d_delta_c, d_info, d_wsa);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_kkt_aug_kernel launch: ") + hipGetErrorString(e));
  return CPL_OK;
}
}  // namespace cpl

extern "C" {

int32_t cpl_lagrangian_grad(int64_t batch, int32_t n, int32_t m, int32_t nnz, const int32_t* d_col_ptr,
                            const int32_t* d_csc_k, const int32_t* d_csc_row, const double* d_grad,
                            const double* d_jac, const double* d_y, int32_t y_repeat, double* d_out, void* stream) {
  if (batch < 0 || n <= 0 || m < 0 || nnz < 0 || y_repeat < 1)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_lagrangian_grad: bad sizes");
  if (batch == 0) return CPL_OK;
  if (!d_col_ptr || !d_grad || !d_out || (nnz > 0 && (!d_csc_k || !d_csc_row || !d_jac)) || (m > 0 && !d_y))
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_lagrangian_grad: missing buffer");
  const int64_t total = batch * n;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_lagrangian_grad: batch too large");
  hipLaunchKernelGGL(cpl_lagrangian_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, total, (int)n,
                     (int)m, (int)nnz, d_col_ptr, d_csc_k, d_csc_row, d_grad, d_jac, d_y, (int)y_repeat, d_out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_lagrangian_grad launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

int64_t cpl_kkt_workspace_doubles(int32_t nw, int32_t m) {
  if (nw <= 0 || m < 0 || m > nw) return -1;
  return kkt_ws_per(nw, m);
}

int32_t cpl_kkt_solve(int32_t mode, int64_t batch, int32_t nw, int32_t m, const double* d_M, const double* d_A,
                      const double* d_r1, const double* d_r2, const double* d_mu, const double* d_delta_w_last,
                      const uint8_t* d_active, double* d_dw, double* d_dy, double* d_delta_w, double* d_delta_c,
                      int32_t* d_info, double* d_ws, void* stream) {
  if (mode != 0 && mode != 1) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_solve: mode must be 0 or 1");
  if (batch < 0 || nw <= 0 || m < 0 || m > nw || nw > KKT_MAX_NW)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_solve: need 0 <= m <= nw <= 128");
  if (batch == 0) return CPL_OK;
  if (!d_M || (m > 0 && !d_A) || !d_r1 || (m > 0 && !d_r2) || !d_dw || (m > 0 && !d_dy) || !d_ws)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_solve: missing buffer");
  if (mode == 0 && (!d_mu || !d_delta_w || !d_delta_c || !d_info))
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_solve: factorisation needs mu, delta_w, delta_c, info");
  if (batch > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_solve: batch too large");
  if (KktWaveKernel wk = kkt_wave_kernel_for(nw, m)) {
    const size_t lds = sizeof(double) * (size_t)kktw_lds_doubles(nw, m);
    const bool w4 = mode == 0 && kkt_use_w4(batch);
    const KktWaveKernel k = w4 ? static_cast<KktWaveKernel>(cpl_kkt_wave_kernel<47, 30, true>) : wk;
    hipLaunchKernelGGL(k, dim3((unsigned)batch), dim3(w4 ? 256 : 64), lds,
                       (hipStream_t)stream, (int)mode, batch, d_M, d_A, d_r1, d_r2, d_mu, d_delta_w_last, d_active, d_dw,
                       d_dy, d_delta_w, d_delta_c, d_info, d_ws);
  } else {
    const size_t lds = sizeof(double) * (size_t)kkt_launch_lds_doubles(nw, m, mode);
    if (lds > 160 * 1024) return fail(CPL_ERR_UNSUPPORTED, "cpl_kkt_solve: system too large for one LDS image");
    hipLaunchKernelGGL(kkt_kernel_for(nw, m), dim3((unsigned)batch), dim3(KKT_THREADS), lds, (hipStream_t)stream,
                       (int)mode, batch, (int)nw, (int)m, d_M, d_A, d_r1, d_r2, d_mu, d_delta_w_last, d_active, d_dw,
                       d_dy, d_delta_w, d_delta_c, d_info, d_ws);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_kkt_kernel launch: ") + hipGetErrorString(e));
  return CPL_OK;
}


int32_t cpl_kkt_qd_solve(int64_t batch, int32_t nw, int32_t m, const double* d_W, const double* d_A,
                         const double* d_Dinv, const double* d_r1, const double* d_r2, const uint8_t* d_active,
                         double* d_delta_w_last, double* d_dw, double* d_dy, double* d_delta_w, double* d_ws,
                         void* stream) {
  if (batch < 0 || nw <= 0 || m < 0 || nw > KKT_MAX_NW || m > nw)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_qd_solve: need 0 <= m <= nw, 0 < nw <= 128");
  // the kernel's dynamic LDS image (W + A D^-1 A^T, the right-hand side, D^-1 and y, A) must fit one
  // workgroup's 160 KiB
  const size_t lds = sizeof(double) * qd_lds_doubles(nw, m);
  if (lds > 160 * 1024)
    return fail(CPL_ERR_UNSUPPORTED, "cpl_kkt_qd_solve: system too large for one LDS image (nw^2 + nw + 2m + m nw "
                                     "doubles must fit 160 KiB)");
  if (batch == 0) return CPL_OK;
  if (!d_W || (m > 0 && (!d_A || !d_Dinv || !d_r2 || !d_dy)) || !d_r1 || !d_dw || !d_delta_w_last || !d_ws)
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_qd_solve: missing buffer");
  if (batch > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_kkt_qd_solve: batch too large");
  hipLaunchKernelGGL(cpl_kkt_qd_kernel, dim3((unsigned)batch), dim3(KKT_THREADS), lds, (hipStream_t)stream, batch,
                     (int)nw, (int)m, d_W, d_A, d_Dinv, d_r1, d_r2, d_active, d_delta_w_last, d_dw, d_dy, d_delta_w,
                     d_ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CPL_ERR_HIP, std::string("cpl_kkt_qd_kernel launch: ") + hipGetErrorString(e));
  return CPL_OK;
}

}  // extern "C"
