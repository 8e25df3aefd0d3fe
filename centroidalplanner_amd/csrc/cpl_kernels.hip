// cpl_kernels.hip — the hot path on gfx950: batched eval_g + eval_jac_g + eval_f + eval_grad_f
// of CentroidalPlanner's IFOPT problem, one wave-lane per instance.
//
// Mapping (memory-bound pointwise work, no MFMA):
//   * one workgroup = one wave = a tile of 64 consecutive instances;
//   * the tile's decision vectors (64*n doubles, contiguous in HBM) are streamed into LDS with
//     16-byte coalesced loads; each lane then reads its own instance row from LDS;
//   * each lane evaluates its instance in IFOPT order (values / CSR Jacobian / dense gradient)
//     and "emits" every output double into a per-lane LDS row of CHUNK slots; when the chunk is
//     full the wave writes the 64 x CHUNK block back with 16-byte stores, so every store wave-
//     instruction covers 8 contiguous 128-byte runs of instance records (AoS, IFOPT layout).
// Arithmetic: IEEE binary64 with -ffp-contract=off and the reference's operation order
// (see the oracle, oracle/cpl_oracle.c, and DESIGN.md §Numerics); integer and half-integer pow
// exponents go through a double-double power (correctly rounded), instance-independent
// Superquadric factors are precomputed on the host with glibc pow (bit-identical to the
// reference).  Reference lines are cited at each block.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <string>

#include "cpl_layout.hpp"
#include "cpl_status.hpp"

namespace cpl {

constexpr int TILE = 64;          // instances per workgroup (= one wave)
constexpr int CHUNK = 16;         // doubles staged per lane before a write-back
constexpr int SROW = CHUNK + 2;   // LDS row stride in doubles (rows stay 16-B aligned)

// Kernel parameters: everything instance-independent, by value in the kernarg segment.
struct KParams {
  int32_t N, n, m, nnz;
  int32_t env_kind;
  int32_t has_env;
  int32_t x_aligned16;
  int32_t pad0;
  int8_t map_order[CPL_MAX_CONTACTS];
  double mass_default;
  double gravity[3];
  double wrench[6];
  double mu;
  double ground_z;
  double C[3], R[3], P[3];
  // instance-independent Superquadric factors, host glibc pow (same bits as the reference)
  double EJ[3];    // P/pow(R,P)                  src/Superquadric.cpp:54-56
  double Ka[3];    // P*pow(R,-P)                 leading factor of row a of GetNormalJacobian
  double Kb[3];    // (P*P)*pow(R,P*-2.0)
  double Rm2[3];   // pow(R,-(P*2.0))
  double Rp2[3];   // pow(R,P*2.0)
  double Psq[3], Pm1[3], P2[3], P2m2[3], P2m3[3];
  double F_thr[CPL_MAX_CONTACTS];
  double W_com, com_ref[3];
  double W_p[CPL_MAX_CONTACTS], W_F[CPL_MAX_CONTACTS];
  double p_ref[CPL_MAX_CONTACTS][3], F_ref[CPL_MAX_CONTACTS][3];
};
static_assert(sizeof(KParams) < 4096, "kernel parameters must fit the kernarg segment");

// ------------------------------------------------------------------------------------------
// double-double helpers for exact-exponent pow
// ------------------------------------------------------------------------------------------
struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd fast_two_sum(double a, double b) {
  double s = a + b;
  double e = b - (s - a);
  return {s, e};
}
__device__ __forceinline__ dd dd_mul(dd a, dd b) {
  double p = a.hi * b.hi;
  double e = __builtin_fma(a.hi, b.hi, -p);
  e = __builtin_fma(a.hi, b.lo, e);
  e = __builtin_fma(a.lo, b.hi, e);
  return fast_two_sum(p, e);
}
__device__ __forceinline__ dd dd_sqr(dd a) {
  double p = a.hi * a.hi;
  double e = __builtin_fma(a.hi, a.hi, -p);
  e = __builtin_fma(a.hi + a.hi, a.lo, e);
  return fast_two_sum(p, e);
}
__device__ __forceinline__ dd dd_recip(dd a) {
  double q = 1.0 / a.hi;
  double r = __builtin_fma(-a.hi, q, 1.0);
  r = __builtin_fma(-a.lo, q, r);
  return fast_two_sum(q, q * r);
}
__device__ __forceinline__ dd dd_ipow(double x, unsigned k) {
  dd r = {1.0, 0.0};
  dd b = {x, 0.0};
  bool first = true;
  while (k) {
    if (k & 1u) {
      r = first ? b : dd_mul(r, b);
      first = false;
    }
    k >>= 1;
    if (k) b = dd_sqr(b);
  }
  return r;
}

// pow with the semantics of C pow: exact-exponent fast paths (integer, half-integer) computed in
// double-double and rounded once (correctly rounded except in ~2^-47-probability ties); every
// other case (non-finite or zero base, overflow, general exponents) goes to OCML pow.
// The exponent is always instance-independent here, so the branch is wave-uniform.
__device__ double cpow(double x, double e) {
  if (fabs(e) <= 1024.0) {
    const bool finite_nz = (x != 0.0) && (fabs(x) <= 1.7976931348623157e308);
    if (e == rint(e)) {
      if (finite_nz) {
        int k = (int)e;
        dd r = dd_ipow(x, (unsigned)(k < 0 ? -k : k));
        if (k < 0) r = dd_recip(r);
        if (fabs(r.hi) <= 1.7976931348623157e308 && r.hi != 0.0 && fabs(r.hi) >= 2.2250738585072014e-308) return r.hi;
      }
      return pow(x, e);
    }
    const double e2 = e + e;
    if (e2 == rint(e2)) {
      if (finite_nz && x > 0.0) {
        const double kf = floor(e);
        const int k = (int)kf;
        const double s = sqrt(x);
        const double rs = __builtin_fma(-s, s, x);
        dd sq = fast_two_sum(s, rs / (s + s));
        dd r = dd_ipow(x, (unsigned)(k < 0 ? -k : k));
        if (k < 0) r = dd_recip(r);
        r = dd_mul(r, sq);
        if (fabs(r.hi) <= 1.7976931348623157e308 && r.hi != 0.0 && fabs(r.hi) >= 2.2250738585072014e-308) return r.hi;
      }
      return pow(x, e);
    }
  }
  return pow(x, e);
}

// Eigen 3.3 Vector3d reductions as the reference sees them (SSE2 packet reduction):
// dot / squaredNorm = (a0*b0 + a1*b1) + a2*b2.
__device__ __forceinline__ double dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
  return (a0 * b0 + a1 * b1) + a2 * b2;
}

// ------------------------------------------------------------------------------------------
// LDS-staged coalesced writer of one output array
// ------------------------------------------------------------------------------------------
struct Stage {
  double* lds;      // [TILE][SROW]
  double* out;      // first record of this tile (nullptr: output not requested)
  int64_t stride;   // record length in doubles
  int valid;        // instances of this tile (rows to write)
  int k0;           // record offset of the staged chunk
  int j;            // slots filled in the staged chunk (wave-uniform)
};

__device__ __forceinline__ void stage_flush(Stage& s, int lane) {
  __syncthreads();
  const int cnt = s.j;
  if (cnt > 0) {
    if (((s.stride | (int64_t)s.k0 | (int64_t)cnt) & 1) == 0 && (reinterpret_cast<uintptr_t>(s.out) & 15) == 0) {
      const int half = cnt >> 1;
      const int total = s.valid * half;
      if (cnt == CHUNK) {
        for (int e = lane; e < total; e += TILE) {
          const int r = e / (CHUNK / 2), q = e % (CHUNK / 2);
          const double2 v = *reinterpret_cast<const double2*>(s.lds + r * SROW + 2 * q);
          *reinterpret_cast<double2*>(s.out + (int64_t)r * s.stride + s.k0 + 2 * q) = v;
        }
      } else {
        for (int e = lane; e < total; e += TILE) {
          const int r = e / half, q = e - r * half;
          const double2 v = *reinterpret_cast<const double2*>(s.lds + r * SROW + 2 * q);
          *reinterpret_cast<double2*>(s.out + (int64_t)r * s.stride + s.k0 + 2 * q) = v;
        }
      }
    } else {
      const int total = s.valid * cnt;
      for (int e = lane; e < total; e += TILE) {
        const int r = e / cnt, q = e - r * cnt;
        s.out[(int64_t)r * s.stride + s.k0 + q] = s.lds[r * SROW + q];
      }
    }
  }
  __syncthreads();
  s.k0 += cnt;
  s.j = 0;
}

__device__ __forceinline__ void emit(Stage& s, int lane, double v) {
  if (!s.out) return;  // wave-uniform
  s.lds[lane * SROW + s.j] = v;
  if (++s.j == CHUNK) stage_flush(s, lane);
}
__device__ __forceinline__ void finish(Stage& s, int lane) {
  if (s.out && s.j > 0) stage_flush(s, lane);
}

// ------------------------------------------------------------------------------------------
// Superquadric per-contact quantities, src/Superquadric.cpp:40-209, with common subexpressions
// shared across the 9 normal-Jacobian entries; every entry keeps the reference's operation
// order (see DESIGN.md for the term-by-term correspondence).
// ------------------------------------------------------------------------------------------
struct SQContact {
  double val;        // GetEnvironmentValue (+= from 0, then -= 1)
  double ej[3];      // GetEnvironmentJacobian
  double en[3];      // GetNormalValue
  double nj[3][3];   // GetNormalJacobian
};

__device__ __forceinline__ void superquadric_contact(const KParams& K, double p0, double p1, double p2,
                                                     bool want_nj, SQContact& o) {
  const double p[3] = {p0, p1, p2};
  double d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) d[a] = -K.C[a] + p[a];

  // src/Superquadric.cpp:40-49: value += pow((p-C)/R, P) over the axes, then -= 1
  double v = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) v += cpow((p[a] - K.C[a]) / K.R[a], K.P[a]);
  v -= 1.0;
  o.val = v;

  // src/Superquadric.cpp:51-57 and 60-69
  double pm1[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    pm1[a] = cpow(p[a] - K.C[a], K.Pm1[a]);
    o.ej[a] = K.EJ[a] * pm1[a];
  }
  const double nrm = sqrt((o.ej[0] * o.ej[0] + o.ej[1] * o.ej[1]) + o.ej[2] * o.ej[2]);
#pragma unroll
  for (int a = 0; a < 3; ++a) o.en[a] = -o.ej[a] / nrm;

  if (!want_nj) return;

  // src/Superquadric.cpp:72-209
  double inv[3], pP[3], p2P[3], p2Pm2[3], p2Pm3[3], T[3], Dg[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double t = K.C[a] - p[a];
    inv[a] = 1.0 / (t * t);
    pP[a] = cpow(d[a], K.P[a]);
    p2P[a] = cpow(d[a], K.P2[a]);
    p2Pm2[a] = cpow(d[a], K.P2m2[a]);
    p2Pm3[a] = cpow(d[a], K.P2m3[a]);
    T[a] = ((K.Rm2[a] * inv[a]) * K.Psq[a]) * p2P[a];
    Dg[a] = (K.Kb[a] * p2P[a]) * inv[a];
  }
  // diagonal entries (a, a); b < c are the other two axes
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int b = a == 0 ? 1 : 0;
    const int c = a == 2 ? 1 : 2;
    double lead = K.Ka[a];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lead = lead * (k == a ? pP[a] : K.Rm2[k]);
      lead = lead * inv[k];
    }
    lead = lead * K.Pm1[a];
    lead = lead * 1.0;
    const double S = (T[b] + T[c]) + Dg[a];
    const double E = (((((((K.C[b] * K.C[b]) * K.Psq[c]) * p2P[c]) * K.Rp2[b] +
                         (((K.C[c] * K.C[c]) * K.Psq[b]) * p2P[b]) * K.Rp2[c]) +
                        (((p[b] * p[b]) * K.Psq[c]) * p2P[c]) * K.Rp2[b]) +
                       (((p[c] * p[c]) * K.Psq[b]) * p2P[b]) * K.Rp2[c]) -
                      ((((K.C[b] * p[b]) * K.Psq[c]) * p2P[c]) * K.Rp2[b]) * 2.0) -
                     ((((K.C[c] * p[c]) * K.Psq[b]) * p2P[b]) * K.Rp2[c]) * 2.0;
    o.nj[a][a] = lead / cpow(S, 3.0 / 2.0) * E;
  }
  // off-diagonal entries (a, b), o = remaining axis
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      if (a == b) continue;
      const int oo = 3 - a - b;
      double lead = K.Ka[a];
      if (a < b) {  // src/Superquadric.cpp:109, 119, 163
        lead = lead * pm1[a];
        lead = lead * K.Psq[b];
        lead = lead * p2Pm3[b];
        lead = lead * K.P2m2[b];
      } else {      // src/Superquadric.cpp:129, 173, 183
        lead = lead * K.Psq[b];
        lead = lead * p2Pm3[b];
        lead = lead * K.P2m2[b];
        lead = lead * pm1[a];
      }
      lead = lead * K.Rm2[b];
      lead = lead * 1.0;
      const double S = (K.Kb[oo] * p2Pm2[oo] + K.Kb[a] * p2Pm2[a]) + (K.Psq[b] * p2Pm2[b]) * K.Rm2[b];
      o.nj[a][b] = lead / cpow(S, 3.0 / 2.0) * (-1.0 / 2.0);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The evaluation kernel
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TILE) void cpl_eval_kernel(const KParams K, int64_t batch,
                                                         const double* __restrict__ x,
                                                         const double* __restrict__ mass,
                                                         const uint8_t* __restrict__ env_tag,
                                                         double* __restrict__ g_out,
                                                         double* __restrict__ jac_out,
                                                         double* __restrict__ f_out,
                                                         double* __restrict__ grad_out) {
  extern __shared__ __align__(16) double smem[];
  const int lane = threadIdx.x;
  const int n = K.n;
  const int N = K.N;
  const int64_t b0 = (int64_t)blockIdx.x * TILE;
  const int valid = (int)((batch - b0) < TILE ? (batch - b0) : TILE);

  double* X = smem;                     // [TILE][n]
  double* SG = X + TILE * n;            // g / grad staging [TILE][SROW]
  double* SJ = SG + TILE * SROW;        // jac staging      [TILE][SROW]

  // ---- stream the tile's x (valid*n contiguous doubles) into LDS, 16 B per lane-access
  {
    const double* xt = x + b0 * n;
    const int total = valid * n;
    if (K.x_aligned16) {
      const int pairs = total >> 1;
      const double2* src = reinterpret_cast<const double2*>(xt);
      double2* dst = reinterpret_cast<double2*>(X);
      for (int e = lane; e < pairs; e += TILE) dst[e] = src[e];
      if ((total & 1) && lane == 0) X[total - 1] = xt[total - 1];
    } else {
      for (int e = lane; e < total; e += TILE) X[e] = xt[e];
    }
  }
  __syncthreads();

  const int row = lane < valid ? lane : valid - 1;
  const double* xr = X + row * n;
  const int64_t b = b0 + row;
  const double m_i = mass ? mass[b] : K.mass_default;
  const int kind_i = K.env_kind == CPL_ENV_MIXED
                         ? (env_tag[b] == CPL_ENV_SUPERQUADRIC ? CPL_ENV_SUPERQUADRIC : CPL_ENV_GROUND)
                         : K.env_kind;

  const double c0 = xr[0], c1 = xr[1], c2 = xr[2];

  Stage G = {SG, g_out ? g_out + b0 * K.m : nullptr, K.m, valid, 0, 0};
  Stage J = {SJ, jac_out ? jac_out + b0 * K.nnz : nullptr, K.nnz, valid, 0, 0};

  if (G.out || J.out) {
    // ---- CentroidalStatics::GetValues, src/Constraints/CentroidalStatics.cpp:37-61
    if (G.out) {
      double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, v5 = 0.0;
      for (int k = 0; k < N; ++k) {
        const double* q = xr + 3 + 9 * K.map_order[k];
        const double F0 = q[0], F1 = q[1], F2 = q[2];
        const double d0 = q[3] - c0, d1 = q[4] - c1, d2 = q[5] - c2;
        v0 += F0; v1 += F1; v2 += F2;
        v3 += d1 * F2 - d2 * F1;
        v4 += d2 * F0 - d0 * F2;
        v5 += d0 * F1 - d1 * F0;
      }
      v0 -= K.wrench[0]; v1 -= K.wrench[1]; v2 -= K.wrench[2];
      v3 -= K.wrench[3]; v4 -= K.wrench[4]; v5 -= K.wrench[5];
      v0 += m_i * K.gravity[0]; v1 += m_i * K.gravity[1]; v2 += m_i * K.gravity[2];
      emit(G, lane, v0); emit(G, lane, v1); emit(G, lane, v2);
      emit(G, lane, v3); emit(G, lane, v4); emit(G, lane, v5);
    }
    // ---- CentroidalStatics::FillJacobianBlock, src/Constraints/CentroidalStatics.cpp:75-137
    if (J.out) {
      for (int r = 0; r < 3; ++r)  // I3 of every F_i (:93-95)
        for (int i = 0; i < N; ++i) emit(J, lane, 1.0);
      // CoM block: -= over contacts in map order (:119-136)
      double a31 = 0.0, a32 = 0.0, a40 = 0.0, a42 = 0.0, a50 = 0.0, a51 = 0.0;
      for (int k = 0; k < N; ++k) {
        const double* q = xr + 3 + 9 * K.map_order[k];
        a31 -= q[2]; a32 -= -q[1];
        a40 -= -q[2]; a42 -= q[0];
        a50 -= q[1]; a51 -= -q[0];
      }
      // row 3: CoM(1,2), then per contact (column order) F(1,2) (:96-97), p(1,2) (:108-109)
      emit(J, lane, a31); emit(J, lane, a32);
      for (int i = 0; i < N; ++i) {
        const double* q = xr + 3 + 9 * i;
        emit(J, lane, -(q[5] - c2)); emit(J, lane, q[4] - c1);
        emit(J, lane, q[2]); emit(J, lane, -q[1]);
      }
      // row 4: CoM(0,2), F(0,2) (:98-99), p(0,2) (:110-111)
      emit(J, lane, a40); emit(J, lane, a42);
      for (int i = 0; i < N; ++i) {
        const double* q = xr + 3 + 9 * i;
        emit(J, lane, q[5] - c2); emit(J, lane, -(q[3] - c0));
        emit(J, lane, -q[2]); emit(J, lane, q[0]);
      }
      // row 5: CoM(0,1), F(0,1) (:100-101), p(0,1) (:112-113)
      emit(J, lane, a50); emit(J, lane, a51);
      for (int i = 0; i < N; ++i) {
        const double* q = xr + 3 + 9 * i;
        emit(J, lane, -(q[4] - c1)); emit(J, lane, q[3] - c0);
        emit(J, lane, q[1]); emit(J, lane, -q[0]);
      }
    }

    // ---- per contact, std::map order (src/CplProblem.cpp:42-75)
    for (int k = 0; k < N; ++k) {
      const int i = K.map_order[k];
      const double* q = xr + 3 + 9 * i;
      const double F0 = q[0], F1 = q[1], F2 = q[2];
      const double p0 = q[3], p1 = q[4], p2 = q[5];
      const double n0 = q[6], n1 = q[7], n2 = q[8];

      if (K.has_env) {
        double gv[4];
        double ej[3];
        double nj[3][3];
        if (kind_i == CPL_ENV_GROUND) {
          // src/Ground.cpp:23-50
          gv[0] = p2 - K.ground_z;
          gv[1] = n0 - 0.0; gv[2] = n1 - 0.0; gv[3] = n2 - 1.0;
          ej[0] = 0.0; ej[1] = 0.0; ej[2] = 1.0;
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) nj[r][cc] = 0.0;
        } else {
          SQContact s;
          superquadric_contact(K, p0, p1, p2, J.out != nullptr, s);
          gv[0] = s.val;
          gv[1] = n0 - s.en[0]; gv[2] = n1 - s.en[1]; gv[3] = n2 - s.en[2];
#pragma unroll
          for (int r = 0; r < 3; ++r) {
            ej[r] = s.ej[r];
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) nj[r][cc] = J.out ? s.nj[r][cc] : 0.0;
          }
        }
        // EnvironmentConstraint::GetValues / EnvironmentNormal::GetValues
        // (src/Constraints/EnvironmentConstraint.cpp:16-28, EnvironmentNormal.cpp:16-33)
        emit(G, lane, gv[0]); emit(G, lane, gv[1]); emit(G, lane, gv[2]); emit(G, lane, gv[3]);
        // EnvironmentConstraint::FillJacobianBlock p block (:53-60)
        emit(J, lane, ej[0]); emit(J, lane, ej[1]); emit(J, lane, ej[2]);
        // EnvironmentNormal::FillJacobianBlock: row r = p block (:75-83) then n_r = 1 (:66-68)
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          emit(J, lane, nj[r][0]); emit(J, lane, nj[r][1]); emit(J, lane, nj[r][2]);
          emit(J, lane, 1.0);
        }
      }

      // ---- FrictionCone::GetValues / FillJacobianBlock, src/Constraints/FrictionCone.cpp:30-103
      const double mu = K.mu;
      const double t1 = dot3(F0, F1, F2, n0, n1, n2);
      if (G.out) {
        const double nF = dot3(n0, n1, n2, F0, F1, F2);
        const double u0 = F0 - nF * n0, u1 = F1 - nF * n1, u2 = F2 - nF * n2;
        emit(G, lane, -t1 + K.F_thr[i]);
        emit(G, lane, sqrt((u0 * u0 + u1 * u1) + u2 * u2) - mu * t1);
      }
      if (J.out) {
        const double t2 = F0 - n0 * t1;
        const double t3 = F1 - n1 * t1;
        const double t4 = F2 - n2 * t1;
        const double t5 = F0 * n0;
        const double t6 = F1 * n1;
        const double t7 = F2 * n2;
        const double s = sqrt(t2 * t2 + t3 * t3 + t4 * t4);
        // row 0: F block -n (:82-84), n block -F (:93-95)
        emit(J, lane, -n0); emit(J, lane, -n1); emit(J, lane, -n2);
        emit(J, lane, -F0); emit(J, lane, -F1); emit(J, lane, -F2);
        // row 1: F block (:85-87), n block (:97-99)
        emit(J, lane, (t2 * (n0 * n0 - 1.0) * 2.0 + n0 * n1 * t3 * 2.0 + n0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n0);
        emit(J, lane, (t3 * (n1 * n1 - 1.0) * 2.0 + n0 * n1 * t2 * 2.0 + n1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n1);
        emit(J, lane, (t4 * (n2 * n2 - 1.0) * 2.0 + n0 * n2 * t2 * 2.0 + n1 * n2 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n2);
        emit(J, lane, (t2 * (t6 + t7 + t5 * 2.0) * 2.0 + F0 * n1 * t3 * 2.0 + F0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F0);
        emit(J, lane, (t3 * (t5 + t7 + t6 * 2.0) * 2.0 + F1 * n0 * t2 * 2.0 + F1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F1);
        emit(J, lane, (t4 * (t5 + t6 + t7 * 2.0) * 2.0 + F2 * n0 * t2 * 2.0 + F2 * n1 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F2);
      }
    }
    finish(G, lane);
    finish(J, lane);
  }

  // ---- cost: MinimizeCentroidalVariables::GetCost / FillJacobianBlock
  //      src/MinimizeCentroidalVariables.cpp:124-192
  if (f_out && lane < valid) {
    double value = 0;
    for (int k = 0; k < N; ++k) {
      const int i = K.map_order[k];
      const double* q = xr + 3 + 9 * i;
      const double e0 = q[3] - K.p_ref[i][0], e1 = q[4] - K.p_ref[i][1], e2 = q[5] - K.p_ref[i][2];
      const double h0 = q[0] - K.F_ref[i][0], h1 = q[1] - K.F_ref[i][1], h2 = q[2] - K.F_ref[i][2];
      value += 0.5 * K.W_p[i] * ((e0 * e0 + e1 * e1) + e2 * e2) + 0.5 * K.W_F[i] * ((h0 * h0 + h1 * h1) + h2 * h2);
    }
    const double r0 = c0 - K.com_ref[0], r1 = c1 - K.com_ref[1], r2 = c2 - K.com_ref[2];
    value += 0.5 * K.W_com * ((r0 * r0 + r1 * r1) + r2 * r2);
    f_out[b] = value;
  }
  if (grad_out) {
    Stage D = {SG, grad_out + b0 * n, n, valid, 0, 0};
    emit(D, lane, K.W_com * (c0 - K.com_ref[0]));
    emit(D, lane, K.W_com * (c1 - K.com_ref[1]));
    emit(D, lane, K.W_com * (c2 - K.com_ref[2]));
    for (int i = 0; i < N; ++i) {
      const double* q = xr + 3 + 9 * i;
      emit(D, lane, K.W_F[i] * (q[0] - K.F_ref[i][0]));
      emit(D, lane, K.W_F[i] * (q[1] - K.F_ref[i][1]));
      emit(D, lane, K.W_F[i] * (q[2] - K.F_ref[i][2]));
      emit(D, lane, K.W_p[i] * (q[3] - K.p_ref[i][0]));
      emit(D, lane, K.W_p[i] * (q[4] - K.p_ref[i][1]));
      emit(D, lane, K.W_p[i] * (q[5] - K.p_ref[i][2]));
      emit(D, lane, 0.0); emit(D, lane, 0.0); emit(D, lane, 0.0);
    }
    finish(D, lane);
  }
}

// ------------------------------------------------------------------------------------------
// Residual norms of g against its bounds (per shard), deterministic two-stage reduction
// ------------------------------------------------------------------------------------------
constexpr int RN_BLOCK = 256;
constexpr int RN_GRID = 1024;

__device__ __forceinline__ double row_violation(double g, bool cone) {
  if (g != g) return INFINITY;
  if (cone) return g > 0.0 ? g : 0.0;  // [-1e20, 0]: lower bound never active at finite g
  return fabs(g);
}

__global__ __launch_bounds__(RN_BLOCK) void cpl_residual_partial(int64_t total, int m, int contact_rows,
                                                                 const double* __restrict__ g,
                                                                 double* __restrict__ part) {
  __shared__ double smax[RN_BLOCK];
  __shared__ double ssum[RN_BLOCK];
  double vmax = 0.0, vsum = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * RN_BLOCK + threadIdx.x; e < total; e += (int64_t)gridDim.x * RN_BLOCK) {
    const int r = (int)(e % m);
    const bool cone = r >= 6 && ((r - 6) % contact_rows) >= contact_rows - 2;
    const double v = row_violation(g[e], cone);
    vmax = v > vmax ? v : vmax;
    vsum += v * v;
  }
  smax[threadIdx.x] = vmax;
  ssum[threadIdx.x] = vsum;
  __syncthreads();
  for (int s = RN_BLOCK / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smax[threadIdx.x] = smax[threadIdx.x] > smax[threadIdx.x + s] ? smax[threadIdx.x] : smax[threadIdx.x + s];
      ssum[threadIdx.x] += ssum[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = smax[0];
    part[2 * blockIdx.x + 1] = ssum[0];
  }
}

__global__ __launch_bounds__(RN_BLOCK) void cpl_residual_final(int nparts, const double* __restrict__ part,
                                                               double* __restrict__ out) {
  __shared__ double smax[RN_BLOCK];
  __shared__ double ssum[RN_BLOCK];
  double vmax = 0.0, vsum = 0.0;
  for (int e = threadIdx.x; e < nparts; e += RN_BLOCK) {
    vmax = part[2 * e] > vmax ? part[2 * e] : vmax;
    vsum += part[2 * e + 1];
  }
  smax[threadIdx.x] = vmax;
  ssum[threadIdx.x] = vsum;
  __syncthreads();
  for (int s = RN_BLOCK / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smax[threadIdx.x] = smax[threadIdx.x] > smax[threadIdx.x + s] ? smax[threadIdx.x] : smax[threadIdx.x + s];
      ssum[threadIdx.x] += ssum[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = smax[0];
    out[1] = ssum[0];
  }
}

// ------------------------------------------------------------------------------------------
// host side of the launch
// ------------------------------------------------------------------------------------------
static int32_t hip_fail(hipError_t e, const char* what) {
  return fail(CPL_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

static void fill_params(const cpl_problem_desc* d, KParams& K, const double* d_x) {
  std::memset(&K, 0, sizeof(K));
  const Dims D = dims_of(d->n_contacts, d->env_kind);
  K.N = D.N; K.n = D.n; K.m = D.m; K.nnz = D.nnz;
  K.env_kind = d->env_kind;
  K.has_env = has_env(d->env_kind) ? 1 : 0;
  K.x_aligned16 = (reinterpret_cast<uintptr_t>(d_x) & 15) == 0 ? 1 : 0;
  for (int k = 0; k < d->n_contacts; ++k) K.map_order[k] = (int8_t)d->map_order[k];
  K.mass_default = d->mass;
  for (int j = 0; j < 3; ++j) K.gravity[j] = d->gravity[j];
  for (int j = 0; j < 6; ++j) K.wrench[j] = d->wrench[j];
  K.mu = d->mu;
  K.ground_z = d->ground_z;
  for (int a = 0; a < 3; ++a) {
    const double C = d->sq_C[a], R = d->sq_R[a], P = d->sq_P[a];
    K.C[a] = C; K.R[a] = R; K.P[a] = P;
    K.EJ[a] = P / std::pow(R, P);
    K.Ka[a] = P * std::pow(R, -P);
    K.Kb[a] = (P * P) * std::pow(R, P * -2.0);
    K.Rm2[a] = std::pow(R, -(P * 2.0));
    K.Rp2[a] = std::pow(R, P * 2.0);
    K.Psq[a] = P * P;
    K.Pm1[a] = P - 1.0;
    K.P2[a] = P * 2.0;
    K.P2m2[a] = P * 2.0 - 2.0;
    K.P2m3[a] = P * 2.0 - 3.0;
  }
  for (int i = 0; i < CPL_MAX_CONTACTS; ++i) {
    K.F_thr[i] = d->F_thr[i];
    K.W_p[i] = d->W_p[i];
    K.W_F[i] = d->W_F[i];
    for (int j = 0; j < 3; ++j) { K.p_ref[i][j] = d->p_ref[i][j]; K.F_ref[i][j] = d->F_ref[i][j]; }
  }
  K.W_com = d->W_com;
  for (int j = 0; j < 3; ++j) K.com_ref[j] = d->com_ref[j];
}

static size_t eval_lds_bytes(int n) { return sizeof(double) * (size_t)(TILE * n + 2 * TILE * SROW); }

static int32_t launch_eval(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                           const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                           hipStream_t stream) {
  int32_t st = validate_desc(d);
  if (st) return st;
  if (batch < 0) return fail(CPL_ERR_INVALID_ARGUMENT, "negative batch");
  if (batch == 0) return CPL_OK;
  if (!d_x) return fail(CPL_ERR_INVALID_ARGUMENT, "x is required");
  if (d->env_kind == CPL_ENV_MIXED && !d_env_tag)
    return fail(CPL_ERR_INVALID_ARGUMENT, "mixed environment batch needs a per-instance env tag array");
  if ((batch + TILE - 1) / TILE > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "batch too large");
  if (!d_g && !d_jac && !d_f && !d_grad) return CPL_OK;
  KParams K;
  fill_params(d, K, d_x);
  const size_t lds = eval_lds_bytes(K.n);
  if (lds > 160 * 1024) return fail(CPL_ERR_UNSUPPORTED, "problem too large for one LDS tile");
  const unsigned grid = (unsigned)((batch + TILE - 1) / TILE);
  hipLaunchKernelGGL(cpl_eval_kernel, dim3(grid), dim3(TILE), lds, stream, K, batch, d_x, d_mass, d_env_tag,
                     d_g, d_jac, d_f, d_grad);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_eval_kernel launch");
  return CPL_OK;
}

// per-device residual workspace (RN_GRID partial pairs), allocated once
static std::mutex g_ws_mutex;
static double* g_ws[64] = {nullptr};

}  // namespace cpl

using namespace cpl;

extern "C" {

int32_t cpl_eval_batch(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                       const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                       void* stream) {
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, (hipStream_t)stream);
}

int32_t cpl_residual_norms(const cpl_problem_desc* d, int64_t batch, const double* d_g, double* d_out, void* stream) {
  int32_t st = validate_desc(d);
  if (st) return st;
  if (batch < 0 || !d_out || (batch > 0 && !d_g)) return fail(CPL_ERR_INVALID_ARGUMENT, "bad residual arguments");
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev < 0 || dev >= 64) return fail(CPL_ERR_UNSUPPORTED, "device index out of range");
  double* ws;
  {
    std::lock_guard<std::mutex> lk(g_ws_mutex);
    if (!g_ws[dev]) {
      e = hipMalloc(&g_ws[dev], sizeof(double) * 2 * RN_GRID);
      if (e != hipSuccess) return hip_fail(e, "hipMalloc residual workspace");
    }
    ws = g_ws[dev];
  }
  const Dims D = dims_of(d->n_contacts, d->env_kind);
  const int64_t total = batch * D.m;
  int64_t blocks = (total + RN_BLOCK - 1) / RN_BLOCK;
  if (blocks < 1) blocks = 1;
  if (blocks > RN_GRID) blocks = RN_GRID;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cpl_residual_partial, dim3((unsigned)blocks), dim3(RN_BLOCK), 0, s, total, D.m, D.contact_rows,
                     d_g, ws);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_residual_partial launch");
  hipLaunchKernelGGL(cpl_residual_final, dim3(1), dim3(RN_BLOCK), 0, s, (int)blocks, ws, d_out);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_residual_final launch");
  return CPL_OK;
}

int32_t cpl_time_eval_batch(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                            const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                            void* stream, int32_t reps, double* ms_per_launch) {
  if (!ms_per_launch || reps < 1) return fail(CPL_ERR_INVALID_ARGUMENT, "bad timing arguments");
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t e0, e1;
  hipError_t e = hipEventCreate(&e0);
  if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
  e = hipEventCreate(&e1);
  if (e != hipSuccess) { hipEventDestroy(e0); return hip_fail(e, "hipEventCreate"); }
  int32_t st = CPL_OK;
  hipEventRecord(e0, s);
  for (int32_t r = 0; r < reps && st == CPL_OK; ++r)
    st = launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, s);
  hipEventRecord(e1, s);
  e = hipEventSynchronize(e1);
  if (st == CPL_OK && e != hipSuccess) st = hip_fail(e, "hipEventSynchronize");
  float ms = 0.0f;
  if (st == CPL_OK) {
    e = hipEventElapsedTime(&ms, e0, e1);
    if (e != hipSuccess) st = hip_fail(e, "hipEventElapsedTime");
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (st == CPL_OK) *ms_per_launch = (double)ms / reps;
  return st;
}

}  // extern "C"
