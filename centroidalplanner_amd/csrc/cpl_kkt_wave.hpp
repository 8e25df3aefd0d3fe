// cpl_kkt_wave.hpp — the one-wave null-space KKT solve pieces shared by the one-wave KKT kernel
// (cpl_kkt.hip cpl_kkt_wave_kernel) and the solve engine's line-search kernel (cpl_kernels.hip
// cpl_ls_backtrack_kernel: second-order corrections re-solve with the kept factors in the same launch).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "cpl_wave.hpp"

namespace cpl {

// Workspace size per instance (doubles): Q [nw*nw] | QR [m*nw] (R's diagonal on its diagonal) |
// L [nz*nz] | scalars [4] (the one-wave kernel's factor image, smaller, fits inside it)
__host__ __device__ inline int64_t kkt_ws_per(int nw, int m) {
  const int nz = nw - m;
  return (int64_t)nw * nw + (int64_t)m * nw + (int64_t)nz * nz + 4;
}

// ==========================================================================================
// One wave per system, size-specialised (NW x MM known at compile time, NW <= 64): the same
// null-space step with the same inertia correction as the workgroup kernel above, but every phase
// runs on ONE wave — no workgroup barriers (the workgroup kernel parks ~75 % of its wave cycles on
// them) — and each phase issues its memory operations in bulk before it computes, so that a step
// pays one LDS / L2 round trip instead of one per pass:
//   * nw-vectors live one element per lane;
//   * QR of A^T register-resident (lane (g, part) holds rows part + 8t of columns g + 8q): each
//     reflector from an 8-lane group sum, published through a 47-double LDS buffer, the trailing
//     columns updated in registers (8 lanes per column);
//   * Z = H_0 ... H_{m-1} [0; I] (only Z, not the whole Q), register-resident, 4 lanes per column;
//   * Y p_y = Q [p_y; 0] and Y^T u = (Q^T u)[0, m) as reflector chains, two reflectors per wave
//     sum (c_p = v_{2p}^T v_{2p+1} precomputed);
//   * W = M Z and Z^T W on the FP64 matrix cores (v_mfma_f64_16x16x4f64), W's accumulators reused
//     as Z^T W's B fragments; M's fragments stay in registers for every later M product;
//   * the inertia-correcting Cholesky and the triangular sweeps with the rows in registers.
// LDS image QR | Z | L (the lower triangle, packed by rows) | beta | cp | 2 nw vector slots: 19.5 KiB
// at nw = 47, m = 30, i.e. eight systems per CU — as many as its registers allow (21.7 KiB and seven
// with the full square L and 3 nw + m slots).  Factor workspace (mode 1): the image's factors, dW, dC.
// ==========================================================================================
template <int NW, int MM>
struct KktWave {
  static constexpr int NZ = NW - MM;
  static constexpr int ZS = NZ + (NZ & 1);          // Z row stride: even, so rows are 16-byte aligned
  static constexpr int NP = MM / 2;                 // reflector pairs (a lone last one when MM is odd)
  static constexpr int NLP = NZ * (NZ + 1) / 2;     // L's packed lower triangle: L(r, c) at r (r + 1) / 2 + c
  static constexpr int NFAC = MM * NW + NW * ZS + NLP + MM + NP + 1;
  static constexpr int LDS = ((NFAC + 2 * NW) + 1) & ~1;
  static_assert(NW <= 64 && MM <= NW, "one wave per system: nw <= 64");
};

__host__ __device__ inline int kktw_lds_doubles(int nw, int m) {
  const int nz = nw - m, zs = nz + (nz & 1);
  return ((m * nw + nw * zs + nz * (nz + 1) / 2 + m + m / 2 + 1 + 2 * nw) + 1) & ~1;
}

// two wave sums, their DPP chains interleaved (the result in every lane)
__device__ __forceinline__ void wave_sum2(double a, double b, double& A, double& B) {
  a += dpp_mov<DPP_QUAD_XOR1>(a);
  b += dpp_mov<DPP_QUAD_XOR1>(b);
  a += dpp_mov<DPP_QUAD_XOR2>(a);
  b += dpp_mov<DPP_QUAD_XOR2>(b);
  a += dpp_mov<DPP_ROW_HALF_MIRROR>(a);
  b += dpp_mov<DPP_ROW_HALF_MIRROR>(b);
  a += dpp_mov<DPP_ROW_MIRROR>(a);
  b += dpp_mov<DPP_ROW_MIRROR>(b);
  a += dpp_mov<DPP_ROW_BCAST15, 0xa>(a, 0.0);
  b += dpp_mov<DPP_ROW_BCAST15, 0xa>(b, 0.0);
  a += dpp_mov<DPP_ROW_BCAST31, 0xc>(a, 0.0);
  b += dpp_mov<DPP_ROW_BCAST31, 0xc>(b, 0.0);
  A = wave_bcast(a, 63);
  B = wave_bcast(b, 63);
}

// The lane's entry of reflector j: v_j[lane] (1 at lane j, 0 above it)
template <int NW>
__device__ __forceinline__ double refl_entry(const double* QR, int j) {
  const int lane = threadIdx.x & 63;
  return (lane > j && lane < NW) ? QR[j * NW + lane] : (lane == j ? 1.0 : 0.0);
}

// x <- Q x = H_0 H_1 ... H_{MM-1} x   (bl: beta_j in lane j, cl: c_p in lane p).  Rolled over the
// reflector pairs with the next pair's entries loaded one step ahead: two reflectors per wave-sum
// latency, a handful of VGPRs.
template <int NW, int MM>
__device__ __forceinline__ double chain_Q(double x, const double* QR, double bl, double cl) {
  if constexpr (MM & 1) {
    constexpr int j = MM - 1;
    const double v = refl_entry<NW>(QR, j);
    x -= wave_bcast(bl, j) * wave_sum(v * x) * v;
  }
  if constexpr (MM >= 2) {
    double v0 = refl_entry<NW>(QR, MM / 2 * 2 - 2), v1 = refl_entry<NW>(QR, MM / 2 * 2 - 1);
    #pragma unroll 1
    for (int p = MM / 2 - 1; p >= 0; --p) {  // H_{2p} H_{2p+1}: s1 first, s0 corrected by c_p
      const int j = 2 * p;
      const double n0 = p > 0 ? refl_entry<NW>(QR, j - 2) : 0.0, n1 = p > 0 ? refl_entry<NW>(QR, j - 1) : 0.0;
      double A0, A1;
      wave_sum2(v0 * x, v1 * x, A0, A1);
      const double s1 = wave_bcast(bl, j + 1) * A1;
      const double s0 = wave_bcast(bl, j) * (A0 - s1 * wave_bcast(cl, p));
      x -= s1 * v1 + s0 * v0;
      v0 = n0;
      v1 = n1;
    }
  }
  return x;
}

// x <- Q^T x = H_{MM-1} ... H_1 H_0 x
template <int NW, int MM>
__device__ __forceinline__ double chain_Qt(double x, const double* QR, double bl, double cl) {
  if constexpr (MM >= 2) {
    double v0 = refl_entry<NW>(QR, 0), v1 = refl_entry<NW>(QR, 1);
    #pragma unroll 1
    for (int p = 0; p < MM / 2; ++p) {  // H_{2p+1} H_{2p}: s0 first, s1 corrected by c_p
      const int j = 2 * p;
      const bool more = p + 1 < MM / 2;
      const double n0 = more ? refl_entry<NW>(QR, j + 2) : 0.0, n1 = more ? refl_entry<NW>(QR, j + 3) : 0.0;
      double A0, A1;
      wave_sum2(v0 * x, v1 * x, A0, A1);
      const double s0 = wave_bcast(bl, j) * A0;
      const double s1 = wave_bcast(bl, j + 1) * (A1 - s0 * wave_bcast(cl, p));
      x -= s0 * v0 + s1 * v1;
      v0 = n0;
      v1 = n1;
    }
  }
  if constexpr (MM & 1) {
    constexpr int j = MM - 1;
    const double v = refl_entry<NW>(QR, j);
    x -= wave_bcast(bl, j) * wave_sum(v * x) * v;
  }
  return x;
}

// Triangular solve T x = b on one wave with the lane's row of T in registers (one LDS round trip
// for the whole row instead of one per step): lane r holds x_r (b_r on entry, r < N); T(r, k) =
// T[r * si + k * sk], diagonal D[r * sd].  The same arithmetic as wave_trsv (x_i = a_i * (1 / D_i),
// a_r -= T(r, i) x_i), so the same result bit for bit.
template <int N, bool LOWER>
__device__ __forceinline__ double wave_trsv_reg(const double* T, int si, int sk, const double* D, int sd, double x) {
  const int lane = threadIdx.x & 63;
  const bool act = lane < N;
  const int lr = act ? lane : 0;
  double t[N];
#pragma unroll
  for (int k = 0; k < N; ++k) t[k] = T[lr * si + k * sk];
  const double inv = act ? 1.0 / D[lr * sd] : 0.0;
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const int i = LOWER ? s : N - 1 - s;
    const double xi = wave_bcast(x, i) * wave_bcast(inv, i);
    if (lane == i) x = xi;
    if (LOWER ? (act && lane > i) : (lane < i)) x -= t[i] * xi;
  }
  return act ? x : 0.0;
}

// wave_trsv_reg over a lower triangle packed by rows (Lp: L(r, c) at r (r + 1) / 2 + c, c <= r):
// L x = b (LOWER) or L^T x = b.  The same operands in the same order as wave_trsv_reg over the full
// square (bitwise the same x); the entries a lane loads past its row's triangle stay inside the
// array and are never used (the masked updates).
template <int N, bool LOWER>
__device__ __forceinline__ double wave_trsv_packed(const double* Lp, double x) {
  const int lane = threadIdx.x & 63;
  const bool act = lane < N;
  const int lr = act ? lane : 0;
  double t[N];
#pragma unroll
  for (int k = 0; k < N; ++k) t[k] = LOWER ? Lp[lr * (lr + 1) / 2 + k] : Lp[k * (k + 1) / 2 + lr];
  const double inv = act ? 1.0 / Lp[lr * (lr + 1) / 2 + lr] : 0.0;
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const int i = LOWER ? s : N - 1 - s;
    const double xi = wave_bcast(x, i) * wave_bcast(inv, i);
    if (lane == i) x = xi;
    if (LOWER ? (act && lane > i) : (lane < i)) x -= t[i] * xi;
  }
  return act ? x : 0.0;
}

// M as FP64-MFMA A fragments: Mf[rb][kb] = M[16 rb + (lane & 15)][4 kb + (lane >> 4)] (zero padded),
// loaded once per factorisation (M symmetric: the lanes read along a row) and kept in registers
template <int NW>
struct MFrag {
  static constexpr int KB = (NW + 3) / 4, RB = (NW + 15) / 16;
};
template <int NW>
__device__ __forceinline__ void load_m_frags(const double* M, double (&Mf)[MFrag<NW>::RB][MFrag<NW>::KB]) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int rb = 0; rb < MFrag<NW>::RB; ++rb)
#pragma unroll
    for (int kb = 0; kb < MFrag<NW>::KB; ++kb) {
      const int r = 16 * rb + li, k = 4 * kb + lk;
      Mf[rb][kb] = (r < NW && k < NW) ? M[k * NW + r] : 0.0;
    }
}

// y = M x on the matrix cores: B = [x 0 ... 0] (x in column 0, read from LDS xs), one D column per
// 16-row block; the results (lanes 0, 16, 32, 48) go through LDS ys back to one element per lane.
// ys may alias xs.  Returns y_lane (0 for lanes >= NW).
template <int NW>
__device__ __forceinline__ double mfma_matvec(const double (&Mf)[MFrag<NW>::RB][MFrag<NW>::KB], const double* xs,
                                              double* ys) {
  constexpr int KB = MFrag<NW>::KB, RB = MFrag<NW>::RB;
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  double xf[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int k = 4 * kb + lk;
    xf[kb] = (li == 0 && k < NW) ? xs[k] : 0.0;
  }
  f64x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) acc[rb] = __builtin_amdgcn_mfma_f64_16x16x4f64(Mf[rb][kb], xf[kb], acc[rb], 0, 0, 0);
  }
  __builtin_amdgcn_wave_barrier();
  if (li == 0) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * rb + lk + 4 * q;
        if (r < NW) ys[r] = acc[rb][q];
      }
  }
  __builtin_amdgcn_wave_barrier();
  return lane < NW ? ys[lane] : 0.0;
}

// mfma_matvec with M's fragments loaded from memory (L2) just before their MFMAs instead of held in
// registers: the same operands in the same order (bitwise the same y), without 72 VGPRs live across
// the caller — for kernels whose occupancy the resident fragments would cost (the line-search kernel's
// second-order corrections).
template <int NW>
__device__ __forceinline__ double mfma_matvec_g(const double* __restrict__ M, const double* xs, double* ys) {
  constexpr int KB = MFrag<NW>::KB, RB = MFrag<NW>::RB;
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  double xf[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int k = 4 * kb + lk;
    xf[kb] = (li == 0 && k < NW) ? xs[k] : 0.0;
  }
  f64x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int r = 16 * rb + li, k = 4 * kb + lk;
      const double mf = (r < NW && k < NW) ? M[k * NW + r] : 0.0;
      acc[rb] = __builtin_amdgcn_mfma_f64_16x16x4f64(mf, xf[kb], acc[rb], 0, 0, 0);
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (li == 0) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * rb + lk + 4 * q;
        if (r < NW) ys[r] = acc[rb][q];
      }
  }
  __builtin_amdgcn_wave_barrier();
  return lane < NW ? ys[lane] : 0.0;
}

// The null-space solve on one wave.  q1v (lanes < NW), q2v (lanes < MM): the right-hand sides in
// registers; returns dw in *dwv (lanes < NW) and dy in *dyv (lanes < MM).  s1, s2: LDS scratch of NW
// doubles.  M: the system's (symmetric) M in global memory, read by columns.
// the same with any M x product (mv(xs, ys): M xs through the LDS vectors, as mfma_matvec)
template <int NW, int MM, class MV>
__device__ __forceinline__ void wave_null_solve_mv(const double* QR, const double* Z, const double* L,
                                                   const double* beta, const double* cp, MV&& mv, double dW,
                                                   double q1v, double q2v, double* s1, double* s2, double* dwv,
                                                   double* dyv) {
  constexpr int NZ = NW - MM;
  constexpr int ZS = KktWave<NW, MM>::ZS;
  const int lane = threadIdx.x & 63;
  // beta and c_p for the two chains (lanes j / p)
  const double bl = lane < MM ? beta[lane] : 0.0;
  const double cl = lane < MM / 2 ? cp[lane] : 0.0;
  const bool rw = lane < NW;
  // R^T p_y = q2   ((R^T)[i][k] = QR[i * NW + k])
  const double py = wave_trsv_reg<MM, true>(QR, NW, 1, QR, NW + 1, lane < MM ? q2v : 0.0);
  // x = Y p_y = Q [p_y; 0]
  double x = chain_Q<NW, MM>(py, QR, bl, cl);
  if (rw) s2[lane] = x;
  __builtin_amdgcn_wave_barrier();
  if constexpr (NZ > 0) {
    // t = q1 - (M + dW I) Y p_y  ->  rz = Z^T t  ->  L L^T p_z = rz
    const double mx = mv(s2, s1);
    if (rw) s1[lane] = q1v - dW * x - mx;
    __builtin_amdgcn_wave_barrier();
    double rz = 0.0;
    if (lane < NZ) {
      double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 8
      for (int r = 0; r < NW; ++r) a[r & 3] += Z[r * ZS + lane] * s1[r];
      rz = (a[0] + a[1]) + (a[2] + a[3]);
    }
    const double yz = wave_trsv_packed<NZ, true>(L, rz);   // L y = rz
    const double pz = wave_trsv_packed<NZ, false>(L, yz);  // L^T p_z = y
    __builtin_amdgcn_wave_barrier();
    if (lane < NZ) s2[lane] = pz;
    __builtin_amdgcn_wave_barrier();
    // dw = Y p_y + Z p_z
    if (rw) {
      double a[2] = {0.0, 0.0};
#pragma unroll
      for (int c = 0; c < NZ; ++c) a[c & 1] += Z[lane * ZS + c] * s2[c];
      x += a[0] + a[1];
    }
    __builtin_amdgcn_wave_barrier();
    if (rw) s2[lane] = x;
    __builtin_amdgcn_wave_barrier();
  }
  *dwv = x;
  // u = q1 - (M + dW I) dw  ->  Y^T u = (Q^T u)[0, m)  ->  R dy = Y^T u
  const double mx = mv(s2, s1);
  const double u = chain_Qt<NW, MM>(rw ? q1v - dW * x - mx : 0.0, QR, bl, cl);
  *dyv = wave_trsv_reg<MM, false>(QR, 1, NW, QR, NW + 1, lane < MM ? u : 0.0);  // R[i][k] = QR[k * NW + i]
  __builtin_amdgcn_wave_barrier();
}

template <int NW, int MM>
__device__ __forceinline__ void wave_null_solve_t(const double* QR, const double* Z, const double* L,
                                                  const double* beta, const double* cp,
                                                  const double (&Mf)[MFrag<NW>::RB][MFrag<NW>::KB], double dW,
                                                  double q1v, double q2v, double* s1, double* s2, double* dwv,
                                                  double* dyv) {
  wave_null_solve_mv<NW, MM>(QR, Z, L, beta, cp, [&](const double* xs, double* ys) { return mfma_matvec<NW>(Mf, xs, ys); },
                             dW, q1v, q2v, s1, s2, dwv, dyv);
}


// Re-solve with the factors a factorisation kept (mode 1 of cpl_kkt_wave_kernel): the factor image
// (NFAC doubles) copied from the instance's workspace wsb into LDS sm (W::LDS doubles: the image
// then two NW scratch vectors), M's fragments loaded from global memory, the null-space solve.
// q1v (lanes < NW), q2v (lanes < MM): the right-hand sides; *dwv, *dyv as wave_null_solve_t.
template <int NW, int MM>
__device__ __forceinline__ void kkt_wave_resolve(const double* __restrict__ M, const double* __restrict__ wsb,
                                                 double q1v, double q2v, double* sm, double* dwv, double* dyv) {
  using W = KktWave<NW, MM>;
  constexpr int NZ = W::NZ, ZS = W::ZS, NFAC = W::NFAC;
  const int lane = threadIdx.x & 63;
  double* QR = sm;
  double* Z = QR + MM * NW;
  double* L = Z + NW * ZS;
  double* beta = L + W::NLP;
  double* cp = beta + MM;
  double* s1 = sm + NFAC;
  double* s2 = s1 + NW;
  for (int i = lane; i < NFAC; i += 64) sm[i] = wsb[i];
  const double dW = wsb[NFAC];
  __builtin_amdgcn_wave_barrier();
  double Mf[MFrag<NW>::RB][MFrag<NW>::KB];
  load_m_frags<NW>(M, Mf);
  wave_null_solve_t<NW, MM>(QR, Z, L, beta, cp, Mf, dW, q1v, q2v, s1, s2, dwv, dyv);
}

// kkt_wave_resolve with M's fragments loaded per product (mfma_matvec_g): bitwise the same step, for
// kernels that cannot keep 72 VGPRs of fragments resident (the line-search kernel)
template <int NW, int MM>
__device__ __forceinline__ void kkt_wave_resolve_g(const double* __restrict__ M, const double* __restrict__ wsb,
                                                   double q1v, double q2v, double* sm, double* dwv, double* dyv) {
  using W = KktWave<NW, MM>;
  constexpr int NZ = W::NZ, ZS = W::ZS, NFAC = W::NFAC;
  const int lane = threadIdx.x & 63;
  double* QR = sm;
  double* Z = QR + MM * NW;
  double* L = Z + NW * ZS;
  double* beta = L + W::NLP;
  double* cp = beta + MM;
  double* s1 = sm + NFAC;
  double* s2 = s1 + NW;
  for (int i = lane; i < NFAC; i += 64) sm[i] = wsb[i];
  const double dW = wsb[NFAC];
  __builtin_amdgcn_wave_barrier();
  wave_null_solve_mv<NW, MM>(QR, Z, L, beta, cp, [&](const double* xs, double* ys) { return mfma_matvec_g<NW>(M, xs, ys); },
                             dW, q1v, q2v, s1, s2, dwv, dyv);
}

// kkt_wave_resolve_g reading the factors straight from the instance's workspace (global memory, an L2
// hit after the factorisation) instead of an LDS copy: the same operations on the same values (bitwise
// the same step), with only the two NW-double scratch vectors in LDS (`scratch`) — for the line-search
// kernel at large batches, whose 22 KiB LDS image of the factors bounded its waves per CU
template <int NW, int MM>
__device__ __forceinline__ void kkt_wave_resolve_gg(const double* __restrict__ M, const double* __restrict__ wsb,
                                                    double q1v, double q2v, double* scratch, double* dwv,
                                                    double* dyv) {
  using W = KktWave<NW, MM>;
  constexpr int NZ = W::NZ, ZS = W::ZS, NFAC = W::NFAC;
  const double* QR = wsb;
  const double* Z = QR + MM * NW;
  const double* L = Z + NW * ZS;
  const double* beta = L + W::NLP;
  const double* cp = beta + MM;
  double* s1 = scratch;
  double* s2 = s1 + NW;
  const double dW = wsb[NFAC];
  wave_null_solve_mv<NW, MM>(QR, Z, L, beta, cp, [&](const double* xs, double* ys) { return mfma_matvec_g<NW>(M, xs, ys); },
                             dW, q1v, q2v, s1, s2, dwv, dyv);
}

}  // namespace cpl
