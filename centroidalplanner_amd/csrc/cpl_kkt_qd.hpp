// cpl_kkt_qd.hpp — the restoration phase's quasi-definite Newton system of one instance on one
// workgroup, and the one-wave Cholesky / triangular-solve helpers it shares with the KKT kernels.
// Used by cpl_kkt_qd_kernel (cpl_kkt.hip) and by the solve engine's small-batch tail kernel
// (cpl_solver.hip k_tail_small), which runs it right after the same instance's restoration entry.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "cpl_wave.hpp"

namespace cpl {

// Right-looking Cholesky of the n x n matrix H (row-major, stride n) in LDS, lower factor in place,
// by one wave (wave-uniform control flow, no workgroup barriers): lanes own rows; LDS accesses of
// one wave complete in order, so a lane reads the column entries other lanes scaled in the
// previous instruction.  Returns true (wave-uniform) when every pivot is above pivot_min and finite.
__device__ __forceinline__ bool wave_cholesky(double* H, int n, double pivot_min) {
  const int lane = threadIdx.x & 63;
  __builtin_amdgcn_wave_barrier();
  #pragma unroll 1
  for (int k = 0; k < n; ++k) {
    const double d = H[k * n + k];
    if (!(d > pivot_min) || !(d < INFINITY)) return false;
    const double lkk = sqrt(d);
    const double inv = 1.0 / lkk;
    for (int i = k + 1 + lane; i < n; i += 64) H[i * n + k] *= inv;
    if (lane == 0) H[k * n + k] = lkk;
    __builtin_amdgcn_wave_barrier();
    // trailing update of the lower triangle, the (i, j) entries of the trailing square spread over
    // the lanes (independent read-modify-writes, about four per lane at n = 17)
    const int sq = n - k - 1;
    // e / sq through a float reciprocal (exact: e < 128^2 and (e + 0.5) / sq sits >= 0.5 / sq from
    // an integer, far above the float error) instead of an integer division per element
    const float rsq = 1.0f / (float)(sq > 0 ? sq : 1);
    for (int e = lane; e < sq * sq; e += 64) {
      const int ii = (int)(((float)e + 0.5f) * rsq), jj = e - ii * sq;
      if (jj <= ii) {
        const int i = k + 1 + ii, j = k + 1 + jj;
        H[i * n + j] -= H[i * n + k] * H[j * n + k];
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  return true;
}

// Triangular solve T x = b in place (x holds b on entry), n <= 128, by wave 0 alone: rows live in
// lanes (lane, lane + 64); column-oriented substitution, the solved component broadcast by a
// shuffle, one LDS read + FMA per lane and step.  T(i, k) = Tm[i * si + k * sk]; diagonal
// D[i * sd].  lower: forward substitution; otherwise backward.  Callers barrier afterwards.
__device__ __forceinline__ void wave_trsv(int n, bool lower, const double* Tm, int si, int sk, const double* D, int sd, double* x) {
  const int lane = threadIdx.x & 63;
  const int r0 = lane, r1 = lane + 64;
  double a0 = r0 < n ? x[r0] : 0.0;
  double a1 = r1 < n ? x[r1] : 0.0;
  // reciprocal diagonal of the lane's rows, computed in parallel ahead of the sequential sweep
  const double v0 = r0 < n ? 1.0 / D[r0 * sd] : 0.0;
  const double v1 = r1 < n ? 1.0 / D[r1 * sd] : 0.0;
  #pragma unroll 1
  for (int t = 0; t < n; ++t) {
    const int i = lower ? t : n - 1 - t;
    const double ai = i < 64 ? wave_bcast(a0, i) : wave_bcast(a1, i - 64);
    const double xi = ai * (i < 64 ? wave_bcast(v0, i) : wave_bcast(v1, i - 64));
    if (r0 == i) a0 = xi;
    if (r1 == i) a1 = xi;
    if (lower) {
      if (r0 > i && r0 < n) a0 -= Tm[r0 * si + i * sk] * xi;
      if (r1 > i && r1 < n) a1 -= Tm[r1 * si + i * sk] * xi;
    } else {
      if (r0 < i) a0 -= Tm[r0 * si + i * sk] * xi;
      if (r1 < i) a1 -= Tm[r1 * si + i * sk] * xi;
    }
  }
  if (r0 < n) x[r0] = a0;
  if (r1 < n) x[r1] = a1;
}


// Right-looking Cholesky on one wave with lane r holding row r of the N x N matrix in a[] (the
// lower factor replaces the lower triangle; the upper triangle is left as it was).  The same
// operations in the same order as wave_cholesky (l_ik = a_ik * (1 / l_kk), a_ij -= l_ik l_jk), so
// the same factor bit for bit, with no LDS round trips.  false (wave-uniform) on a pivot at or
// below pivot_min or non-finite.
template <int N>
__device__ __forceinline__ bool wave_cholesky_reg(double (&a)[N], double pivot_min) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const double d = wave_bcast(a[k], k);
    if (!(d > pivot_min) || !(d < INFINITY)) return false;
    const double lkk = sqrt(d);
    const double inv = 1.0 / lkk;
    const double lik = lane > k ? a[k] * inv : 0.0;
    if (lane == k) a[k] = lkk;
    if (lane > k) a[k] = lik;
#pragma unroll
    for (int j = k + 1; j < N; ++j) {
      const double ljk = wave_bcast(lik, j);
      if (lane >= j) a[j] -= lik * ljk;
    }
  }
  return true;
}


// ---- the restoration phase's Newton system (quasi-definite) -------------------------------
// IPOPT's restoration problem (min rho sum(p + n) + eta/2 |D_R (x - x_R)|^2 s.t. c(w) - p + n = 0,
// p, n >= 0) with p and n eliminated, as IPOPT's AugRestoSystemSolver reduces it:
//     [ W   A^T ] [dw]   [r1]      D = 1/Sigma_p + 1/Sigma_n > 0 (diagonal, m)
//     [ A   -D  ] [dy] = [r2]
// has the right inertia iff K = W + A^T D^-1 A is positive definite, so its Cholesky is the inertia
// test and dW follows IPOPT's schedule (first 1e-4, or dW_last / 3; x100 / x8).  Then
// dw = K^-1 (r1 + A^T D^-1 r2), dy = D^-1 (A dw - r2).  One workgroup per instance: K formed once
// (lower triangle, mirrored: bitwise symmetric) into the global workspace, each attempt factorised
// by one wave in LDS (batch_ipm.py kkt_qd restates it).  Pivots at or below eps max|K_ii| count as
// zero eigenvalues.
// One factorisation attempt of the quasi-definite system's K + dW I on one wave: for the 4-contact
// size the rows live in registers (wave_cholesky_reg: bitwise the LDS factor, no LDS round trips:
// the restoration phase's factorisations took 150-350 us with the LDS version's read-modify-writes
// over the trailing square); the factor goes to L for the triangular solves.
template <int N>
__device__ __forceinline__ bool qd_factor_reg(const double* __restrict__ K, double dW, double piv, double* L) {
  const int lane = threadIdx.x & 63;
  double a[N];
#pragma unroll
  for (int k = 0; k < N; ++k) a[k] = lane < N ? K[lane * N + k] + (lane == k ? dW : 0.0) : 0.0;
  const bool ok = wave_cholesky_reg<N>(a, piv);
  if (ok && lane < N) {
#pragma unroll
    for (int k = 0; k < N; ++k) L[lane * N + k] = a[k];
  }
  return ok;
}

// the dynamic LDS image of qd_solve_block, in doubles
__host__ __device__ inline size_t qd_lds_doubles(int nw, int m) {
  return (size_t)nw * nw + nw + 2 * (size_t)(m > 0 ? m : 1) + (size_t)m * nw;
}

// The solve of instance b by the NT threads of one workgroup (qd_lds: the dynamic LDS image,
// nw^2 + nw + 2m + m nw doubles).  Every thread of the workgroup calls it (workgroup barriers inside).
template <int NT>
__device__ __forceinline__ void qd_solve_block(int64_t b, int nw, int m, const double* __restrict__ W,
                                               const double* __restrict__ A, const double* __restrict__ Dinv,
                                               const double* __restrict__ r1, const double* __restrict__ r2,
                                               double* __restrict__ dwl, double* __restrict__ dw_out,
                                               double* __restrict__ dy_out, double* __restrict__ delta_w_out,
                                               double* __restrict__ Kws, double* qd_lds) {
  double* L = qd_lds;              // [nw][nw]
  double* v = L + nw * nw;         // [nw]: rhs -> solution
  double* t = v + nw;              // [m]: D^-1 r2
  __shared__ double s_red[NT / 64];
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  const double* Wb = W + b * (int64_t)nw * nw;
  double* As = t + m;             // [m][nw]: A staged in LDS
  double* Ds = As + m * nw;       // [m]: D^-1
  for (int e = tid; e < m * nw; e += NT) As[e] = A[b * (int64_t)m * nw + e];
  for (int r = tid; r < m; r += NT) Ds[r] = Dinv[b * m + r];
  __syncthreads();
  const double* Ab = As;
  const double* Db = Ds;
  double* Kb = Kws + b * (int64_t)nw * nw;
  // K = W + A^T D^-1 A, lower triangle (i >= j) summed over the rows in order, mirrored
  double dmax = 0.0;
  for (int e = tid; e < nw * nw; e += NT) {
    const int i = e / nw, j = e - i * nw;
    if (j > i) continue;
    double s = 0.0;
    for (int r = 0; r < m; ++r) s += (Ab[r * nw + i] * Db[r]) * Ab[r * nw + j];
    const double k = Wb[i * nw + j] + s;
    Kb[i * nw + j] = k;
    Kb[j * nw + i] = k;
    if (i == j) dmax = fmax(dmax, fabs(k));
  }
  for (int r = tid; r < m; r += NT) t[r] = Db[r] * r2[b * m + r];
  dmax = wave_max(dmax);
  if ((tid & 63) == 0) s_red[tid >> 6] = dmax;
  __syncthreads();  // (also orders the global K stores before the copies below)
  double kmax = 0.0;
  for (int q = 0; q < NT / 64; ++q) kmax = fmax(kmax, s_red[q]);
  const double piv_tol = 2.220446049250313e-16 * kmax;
  const double last = dwl[b];
  double dW = 0.0;
  for (int attempt = 0; attempt < 64; ++attempt) {
    if (nw == 47) {  // (K's global copy was written by this workgroup before the barrier above)
      if (tid < 64) {
        const bool ok = qd_factor_reg<47>(Kb, dW, piv_tol, L);
        if (tid == 0) s_ok = ok ? 1 : 0;
      }
    } else {
      for (int e = tid; e < nw * nw; e += NT) {
        const int i = e / nw, j = e - i * nw;
        L[e] = Kb[e] + (i == j ? dW : 0.0);
      }
      __syncthreads();
      if (tid < 64) {
        const bool ok = wave_cholesky(L, nw, piv_tol);
        if (tid == 0) s_ok = ok ? 1 : 0;
      }
    }
    __syncthreads();
    if (s_ok) break;
    dW = dW == 0.0 ? (last == 0.0 ? 1e-4 : fmax(last / 3.0, 1e-20)) : dW * (last == 0.0 ? 100.0 : 8.0);
    __syncthreads();
  }
  // rhs = r1 + A^T (D^-1 r2)
  for (int k = tid; k < nw; k += NT) {
    double s = 0.0;
    for (int r = 0; r < m; ++r) s += Ab[r * nw + k] * t[r];
    v[k] = r1[b * nw + k] + s;
  }
  __syncthreads();
  if (tid < 64) {
    wave_trsv(nw, true, L, nw, 1, L, nw + 1, v);   // L u = rhs
    wave_trsv(nw, false, L, 1, nw, L, nw + 1, v);  // L^T dw = u
  }
  __syncthreads();
  for (int k = tid; k < nw; k += NT) dw_out[b * nw + k] = v[k];
  for (int r = tid; r < m; r += NT) {
    double s = 0.0;
    for (int k = 0; k < nw; ++k) s += Ab[r * nw + k] * v[k];
    dy_out[b * m + r] = Db[r] * (s - r2[b * m + r]);
  }
  if (tid == 0) {
    if (delta_w_out) delta_w_out[b] = dW;
    dwl[b] = dW;
  }
}

}  // namespace cpl
