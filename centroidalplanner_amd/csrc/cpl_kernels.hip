// cpl_kernels.hip — the hot path on gfx950: batched eval_g + eval_jac_g + eval_f + eval_grad_f
// of CentroidalPlanner's IFOPT problem for many independent instances per launch.
//
// Kernels the product dispatches (memory-bound pointwise work, no MFMA):
//   * cpl_eval_pipe_kernel<ENV> — none / Ground environments (the north-star path): persistent,
//     warp-specialised workgroups walking tiles blockIdx, blockIdx + grid, ...; one loader wave DMAs
//     the NEXT tile's decision vectors into the other half of a double-buffered LDS image
//     (global_load_lds_dwordx4) while three compute waves evaluate the current tile's work items
//     (contact blocks in std::map order, statics values + force rows, torque rows, cost) into the
//     tile's AoS output image in LDS and copy it out with 16-byte non-temporal stores, so every
//     128-byte line of g / jac is written once, whole;
//   * cpl_eval_tile_kernel<ENV> — Superquadric and mixed batches: one 256-thread workgroup per tile
//     of T consecutive instances (T sized to the LDS budget), the same work items, Superquadric
//     contacts in two barrier-separated phases (per (contact, axis) double-double power ladders into
//     an LDS scratch, then per (contact, row) the normal-Jacobian entries); mixed tiles compacted by
//     environment kind with a wave ballot;
//   * cpl_eval_kernel — the first design (one wave-lane per instance, per-lane LDS rows written
//     back 64 x CHUNK at a time), kept for A/B measurements only.
// Arithmetic: IEEE binary64 with -ffp-contract=off and the reference's operation order
// (see the oracle, oracle/cpl_oracle.c, and DESIGN.md §Numerics); integer and half-integer pow
// exponents go through a double-double power (correctly rounded), instance-independent
// Superquadric factors are precomputed on the host with glibc pow (bit-identical to the
// reference).  Reference lines are cited at each block.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "cpl_accept.hpp"
#include "cpl_kkt_block.hpp"
#include "cpl_kkt_wave.hpp"
#include "cpl_layout.hpp"
#include "cpl_wave.hpp"
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
  // tile layout of the tile-stationary kernel (doubles offsets into dynamic LDS)
  int32_t T, logT;       // instances per tile (power of two)
  int32_t S;             // work-item segments per instance
  int32_t cost_seg;      // segment index of the cost item, -1 if f/grad not requested
  int32_t offG, offJ, offD, offL, offI;
  int32_t LR;            // doubles per instance in the SQ scratch (N*SQ_L + 1)
  int32_t offX1, offMB, offTB;  // pipelined kernel: second x buffer, masses, env tags
  int32_t want_g, want_j, want_f, want_grad;
  int32_t want_norms;    // fused residual norms of g (cpl_eval_batch_norms)
  int32_t contact_rows;  // constraint rows per contact: 6 (environment) or 2
  int32_t ablate;        // measurement-only ablation (cpl_set_tuning), 0 in production
  int32_t sq_ladder;     // every P_a is an integer in [2, 64]: double-double power ladders
  int32_t grid_cap;      // (entry kernel, the kind split's Ground half) the workgroups that walk the
                         // tiles while the Superquadric list is non-empty (0: every workgroup)
  int32_t cw_prio;       // (entry kernel) the compute waves' wave priority (s_setprio; 0 = default)
  int32_t list_prio;     // (tile kernel, LIST) the gather / copy-out at a raised wave priority (1 = yes)
  // fused Lagrangian gradient (cpl_eval_lagrangian_grad): grad f + J^T y of every instance from the
  // LDS tile image, through a CSC index of the fixed structure; instance b takes y[b / y_repeat]
  int32_t want_lgrad, y_repeat;
  const int32_t* col_ptr;
  const int32_t* csc_k;
  const int32_t* csc_row;
  const double* ly;
  const uint8_t* lg_active;  // optional: instance b / y_repeat inactive -> its rows are skipped
  int32_t offC;              // doubles offset of the LDS copy of the CSC index (fused gradient)
  // Jacobian output layout (cpl_eval_batch_ex): fold = FOLD_NONE (IFOPT CSR values), FOLD_COMMON /
  // FOLD_GROUND (values only: the structurally constant entries skipped, cpl_layout.hpp); jbase /
  // cstride = offset of the first contact block and length of one, in the (folded) record
  int32_t fold, jbase, cstride;
  int32_t soa;               // outputs entry-major ([m][B], [nnz][B], [n][B]) instead of instance-major
  int32_t jdirect;           // tile kernel: the Jacobian items write their entries straight to the
                             // output records instead of the LDS tile image (smaller tiles' LDS)
  int32_t offA;              // (jdirect) doubles offset of the statics CoM-pair scratch [T][6]
  int32_t offRB, offCS, offST;  // entry kernel: row bases [2][T] (int64), cone scratch, statics scratch
  // (the solve engine's NLP scaling, eval_batch_scaled; pipelined kernel only) f, grad times
  // sc_df[b], g row r times sc_dc[b, r], Jacobian entry q (row sc_row[q]) times sc_dc[b, sc_row[q]]
  const double* sc_df;
  const double* sc_dc;
  const int32_t* sc_row;
  // (the solve engine; pipelined kernel only) a device byte that, when 0, makes the launch a no-op:
  // the small-batch iteration's soft-restoration evaluation when no instance tries a soft step
  const uint8_t* gate;
};
static_assert(sizeof(KParams) < 4096, "kernel parameters must fit the kernarg segment");

// Per-block LDS copy of the parameter tables the work items index with a lane-varying contact or
// axis index.  A kernarg read with a divergent index is a vector memory load, and its vmcnt wait
// would also drain the wave's in-flight output stores; an LDS read waits on lgkmcnt only.
constexpr int CPL_MAX_ROWS = 6 + 6 * CPL_MAX_CONTACTS;
// The Superquadric per-axis factors too (the two-phase items index them with a lane-varying axis).
enum { AX_C, AX_R, AX_P, AX_EJ, AX_KA, AX_KB, AX_RM2, AX_RP2, AX_PSQ, AX_PM1, AX_P2, AX_P2M2, AX_P2M3, AX_N };
struct CTab {
  int32_t map_order[CPL_MAX_CONTACTS];
  double F_thr[CPL_MAX_CONTACTS];
  double ax[AX_N][3];          // KParams' C, R, P, EJ, Ka, Kb, Rm2, Rp2, Psq, Pm1, P2, P2m2, P2m3
  uint8_t cone[CPL_MAX_ROWS];  // row r of g is a FrictionCone row (bounds (-inf, 0]) — residual norms
};
__shared__ CTab s_ct;

// cooperative fill; the caller's next block barrier publishes it
__device__ __forceinline__ void load_ctab(const KParams& K) {
  const int t = threadIdx.x;
  if (t < CPL_MAX_CONTACTS) {
    s_ct.map_order[t] = K.map_order[t];
    s_ct.F_thr[t] = K.F_thr[t];
  }
  if (t < 3 * AX_N) {  // (no pointers into K: an address-taken kernarg struct is copied to scratch)
    const int f = t / 3, a = t - 3 * (t / 3);
    double v;
    switch (f) {
      case AX_C: v = K.C[a]; break;
      case AX_R: v = K.R[a]; break;
      case AX_P: v = K.P[a]; break;
      case AX_EJ: v = K.EJ[a]; break;
      case AX_KA: v = K.Ka[a]; break;
      case AX_KB: v = K.Kb[a]; break;
      case AX_RM2: v = K.Rm2[a]; break;
      case AX_RP2: v = K.Rp2[a]; break;
      case AX_PSQ: v = K.Psq[a]; break;
      case AX_PM1: v = K.Pm1[a]; break;
      case AX_P2: v = K.P2[a]; break;
      case AX_P2M2: v = K.P2m2[a]; break;
      default: v = K.P2m3[a]; break;
    }
    s_ct.ax[f][a] = v;
  }
  for (int r = t; r < K.m; r += blockDim.x)
    s_ct.cone[r] = r >= 6 && ((r - 6) % K.contact_rows) >= K.contact_rows - 2;
}

// ---- residual norms of g against its bounds: max violation and sum of squared violations.
// Equality rows (statics, environment, normal) have bounds [0, 0]; cone rows (-1e20, 0]
// (src/Constraints/*.cpp GetBounds).  NaN counts as an infinite violation.
__device__ __forceinline__ double row_violation(double g, bool cone) {
  if (g != g) return INFINITY;
  if (cone) return g > 0.0 ? g : 0.0;  // [-1e20, 0]: lower bound never active at finite g
  return fabs(g);
}

struct NormAcc {
  double vmax = 0.0, vsum = 0.0;
  int r = 0, rstep = 0;  // row of this thread's next element, row advance per stride
  __device__ void init(int tid, int nthreads, int m) {
    r = tid % m;
    rstep = nthreads % m;
  }
  // the g records of one tile (count = rows * instances, contiguous) from LDS
  __device__ __forceinline__ void add_tile(const double* __restrict__ Gt, int count, int tid, int nthreads, int m) {
    int rr = r;
    for (int e = tid; e < count; e += nthreads) {
      const double v = row_violation(Gt[e], s_ct.cone[rr]);
      vmax = v > vmax ? v : vmax;
      vsum += v * v;
      rr += rstep;
      if (rr >= m) rr -= m;
    }
  }
};

// LDS-only workgroup barrier: no vmcnt drain of in-flight global stores
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Block reduction of every thread's NormAcc into one partial pair per workgroup.
// Result valid in thread 0.  LDS-only barriers: the workgroup's output stores issued just before
// keep draining (a __syncthreads would wait for all of them first, on every tile).
__device__ __forceinline__ void block_norms(const NormAcc& a, double& bm, double& bs) {
  __shared__ double red_max[16], red_sum[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = (blockDim.x + 63) >> 6;
  double vmax = a.vmax, vsum = a.vsum;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double om = __shfl_xor(vmax, o);
    const double os = __shfl_xor(vsum, o);
    vmax = om > vmax ? om : vmax;
    vsum += os;
  }
  lds_barrier();  // red_* may still be read by a previous call
  if (lane == 0) { red_max[wave] = vmax; red_sum[wave] = vsum; }
  lds_barrier();
  bm = 0.0;
  bs = 0.0;
  if (tid == 0)
    for (int w = 0; w < nw; ++w) { bm = red_max[w] > bm ? red_max[w] : bm; bs += red_sum[w]; }
}

// Workspace of the fused norms: NORM_HDR doubles of header (reserved), then one partial pair per
// workgroup; the host finishes with cpl_residual_final right after the eval launch.  (A
// single-launch grid finish — last-arrival atomics at agent scope — measured 4-5 us slower at
// 65 536 x 4: its store-ack / atomic / reload round trips sit on the kernel's tail.)
constexpr int NORM_HDR = 128;


// partial pair per WAVE (tile kernel): DPP wave reductions and no barrier, so the reduction adds no
// synchronisation to a workgroup's critical path (the block reduction with its two barriers cost the
// latency-bound Superquadric tiles 14 %); pair index slot * waves + wave (slot: the tile)
__device__ __forceinline__ void partial_norms_waves(const NormAcc& a, double* __restrict__ part, int64_t slot) {
  const double bm = wave_max(a.vmax), bs = wave_sum(a.vsum);
  if ((threadIdx.x & 63) == 0) {
    const int64_t i = slot * (blockDim.x >> 6) + (threadIdx.x >> 6);
    part[2 * i] = bm;
    part[2 * i + 1] = bs;
  }
}

// partial pair per workgroup with plain stores (the kernel boundary is the coherence point)
__device__ void partial_norms(const NormAcc& a, double* __restrict__ part) {
  double bm, bs;
  block_norms(a, bm, bs);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = bm;
    part[2 * blockIdx.x + 1] = bs;
  }
}

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

// Range in which the double-double chains below stay exact-enough (error terms never underflow).
constexpr double DD_TINY = 0x1p-960;
constexpr double DD_HUGE = 0x1p+960;

__device__ __forceinline__ dd dd_mul_d(dd a, double b) {
  double p = a.hi * b;
  double e = __builtin_fma(a.hi, b, -p);
  e = __builtin_fma(a.lo, b, e);
  return fast_two_sum(p, e);
}

// pow(S, 3/2) = S*sqrt(S) in double-double, rounded once (C pow semantics outside the safe range).
// sqrt(S) only has to be close: s from v_rsq_f64 plus one Newton step (~2^-50), then the exact
// residual S - s^2 (one fma) gives the double-double correction (error ~2^-100).
__device__ __forceinline__ double pow_three_halves(double S) {
  if (S > DD_TINY && S < DD_HUGE) {
    const double r = __builtin_amdgcn_rsq(S);
    double s = S * r;
    double h = 0.5 * r;
    const double e = __builtin_fma(-h, s, 0.5);
    s = __builtin_fma(s, e, s);
    h = __builtin_fma(h, e, h);
    const double rs = __builtin_fma(-s, s, S);
    const dd sq = fast_two_sum(s, rs * h);
    return dd_mul_d(sq, S).hi;
  }
  return pow(S, 1.5);
}

// The five powers of d = p_a - C_a the normal Jacobian needs, for integer P in [2, 64]:
// B = d^(P-2) by binary powering, then exact-product chains A = B d = d^(P-1), Q = A d = d^P,
// d^(2P-3) = B A, d^(2P-2) = A^2, d^(2P) = Q^2, all in double-double and rounded once.
struct AxisPowers {
  double pm1, pP, p2Pm3, p2Pm2, p2P;
};
__device__ __forceinline__ void axis_powers(const KParams& K, int a, double d, AxisPowers& o) {
  if (K.sq_ladder) {
    const dd B = dd_ipow(d, (unsigned)K.P[a] - 2u);
    const dd A = dd_mul_d(B, d);
    const dd Q = dd_mul_d(A, d);
    const double q2 = dd_sqr(Q).hi;
    if (q2 == q2 && fabs(q2) >= DD_TINY && fabs(q2) <= DD_HUGE) {  // every chain member in range
      o.pm1 = A.hi;
      o.pP = Q.hi;
      o.p2Pm3 = dd_mul(B, A).hi;
      o.p2Pm2 = dd_sqr(A).hi;
      o.p2P = q2;
      return;
    }
  }
  o.pm1 = cpow(d, K.Pm1[a]);
  o.pP = cpow(d, K.P[a]);
  o.p2Pm3 = cpow(d, K.P2m3[a]);
  o.p2Pm2 = cpow(d, K.P2m2[a]);
  o.p2P = cpow(d, K.P2[a]);
}

// A per-axis Superquadric factor with a lane-varying axis a: from the block's LDS table (AXL) or
// from the kernel arguments (a vector load from the kernarg segment).  Mixed batches take the LDS
// table (the kernarg loads' vmcnt waits also waited for the Jacobian rows' global stores: 3.65 ->
// 3.41 ms at 1M x 16); Superquadric batches keep the kernarg loads (the LDS table raised their
// kernel from 113 to 145 VGPRs, three waves per SIMD instead of four: 0.32 -> 0.39 ms at 262k x 8).
template <bool AXL>
__device__ __forceinline__ double axv(const KParams& K, int f, int a) {
  if (AXL) return s_ct.ax[f][a];
  switch (f) {
    case AX_C: return K.C[a];
    case AX_R: return K.R[a];
    case AX_P: return K.P[a];
    case AX_EJ: return K.EJ[a];
    case AX_KA: return K.Ka[a];
    case AX_KB: return K.Kb[a];
    case AX_RM2: return K.Rm2[a];
    case AX_RP2: return K.Rp2[a];
    case AX_PSQ: return K.Psq[a];
    case AX_PM1: return K.Pm1[a];
    case AX_P2: return K.P2[a];
    case AX_P2M2: return K.P2m2[a];
    default: return K.P2m3[a];
  }
}

// axis_powers with the exponents through axv (the two-phase items: lane-varying a)
template <bool AXL>
__device__ __forceinline__ void axis_powers_ax(const KParams& K, bool ladder, int a, double d, AxisPowers& o) {
  if (ladder) {
    const dd B = dd_ipow(d, (unsigned)axv<AXL>(K, AX_P, a) - 2u);
    const dd A = dd_mul_d(B, d);
    const dd Q = dd_mul_d(A, d);
    const double q2 = dd_sqr(Q).hi;
    if (q2 == q2 && fabs(q2) >= DD_TINY && fabs(q2) <= DD_HUGE) {  // every chain member in range
      o.pm1 = A.hi;
      o.pP = Q.hi;
      o.p2Pm3 = dd_mul(B, A).hi;
      o.p2Pm2 = dd_sqr(A).hi;
      o.p2P = q2;
      return;
    }
  }
  o.pm1 = cpow(d, axv<AXL>(K, AX_PM1, a));
  o.pP = cpow(d, axv<AXL>(K, AX_P, a));
  o.p2Pm3 = cpow(d, axv<AXL>(K, AX_P2M3, a));
  o.p2Pm2 = cpow(d, axv<AXL>(K, AX_P2M2, a));
  o.p2P = cpow(d, axv<AXL>(K, AX_P2, a));
}

__device__ __forceinline__ void superquadric_contact(const KParams& K, double p0, double p1, double p2,
                                                     bool want_nj, SQContact& o) {
  const double p[3] = {p0, p1, p2};
  double d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) d[a] = -K.C[a] + p[a];

  // src/Superquadric.cpp:40-49: value += pow((p-C)/R, P) over the axes, then -= 1
  double v = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double u = (p[a] - K.C[a]) / K.R[a];
    double w;
    if (K.sq_ladder && fabs(u) >= DD_TINY && fabs(u) <= 0x1p+40) {
      w = dd_ipow(u, (unsigned)K.P[a]).hi;
      if (!(fabs(w) >= DD_TINY && fabs(w) <= DD_HUGE)) w = cpow(u, K.P[a]);
    } else {
      w = cpow(u, K.P[a]);
    }
    v += w;
  }
  v -= 1.0;
  o.val = v;

  AxisPowers ap[3];
  if (want_nj) {
#pragma unroll
    for (int a = 0; a < 3; ++a) axis_powers(K, a, d[a], ap[a]);
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) ap[a].pm1 = cpow(d[a], K.Pm1[a]);
  }

  // src/Superquadric.cpp:51-57 and 60-69
#pragma unroll
  for (int a = 0; a < 3; ++a) o.ej[a] = K.EJ[a] * ap[a].pm1;
  const double nrm = sqrt((o.ej[0] * o.ej[0] + o.ej[1] * o.ej[1]) + o.ej[2] * o.ej[2]);
#pragma unroll
  for (int a = 0; a < 3; ++a) o.en[a] = -o.ej[a] / nrm;

  if (!want_nj) return;

  // src/Superquadric.cpp:72-209
  double inv[3], T[3], Dg[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double t = K.C[a] - p[a];
    inv[a] = 1.0 / (t * t);
    T[a] = ((K.Rm2[a] * inv[a]) * K.Psq[a]) * ap[a].p2P;
    Dg[a] = (K.Kb[a] * ap[a].p2P) * inv[a];
  }
  // diagonal entries (a, a); b < c are the other two axes
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int b = a == 0 ? 1 : 0;
    const int c = a == 2 ? 1 : 2;
    double lead = K.Ka[a];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lead = lead * (k == a ? ap[a].pP : K.Rm2[k]);
      lead = lead * inv[k];
    }
    lead = lead * K.Pm1[a];
    lead = lead * 1.0;
    const double S = (T[b] + T[c]) + Dg[a];
    const double p2Pb = ap[b].p2P, p2Pc = ap[c].p2P;
    const double E = (((((((K.C[b] * K.C[b]) * K.Psq[c]) * p2Pc) * K.Rp2[b] +
                         (((K.C[c] * K.C[c]) * K.Psq[b]) * p2Pb) * K.Rp2[c]) +
                        (((p[b] * p[b]) * K.Psq[c]) * p2Pc) * K.Rp2[b]) +
                       (((p[c] * p[c]) * K.Psq[b]) * p2Pb) * K.Rp2[c]) -
                      ((((K.C[b] * p[b]) * K.Psq[c]) * p2Pc) * K.Rp2[b]) * 2.0) -
                     ((((K.C[c] * p[c]) * K.Psq[b]) * p2Pb) * K.Rp2[c]) * 2.0;
    o.nj[a][a] = lead / pow_three_halves(S) * E;
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
        lead = lead * ap[a].pm1;
        lead = lead * K.Psq[b];
        lead = lead * ap[b].p2Pm3;
        lead = lead * K.P2m2[b];
      } else {      // src/Superquadric.cpp:129, 173, 183
        lead = lead * K.Psq[b];
        lead = lead * ap[b].p2Pm3;
        lead = lead * K.P2m2[b];
        lead = lead * ap[a].pm1;
      }
      lead = lead * K.Rm2[b];
      lead = lead * 1.0;
      const double S = (K.Kb[oo] * ap[oo].p2Pm2 + K.Kb[a] * ap[a].p2Pm2) + (K.Psq[b] * ap[b].p2Pm2) * K.Rm2[b];
      o.nj[a][b] = lead / pow_three_halves(S) * (-1.0 / 2.0);
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
  load_ctab(K);
  __syncthreads();
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
// v2 (default): tile-stationary evaluation.
//   * a workgroup owns a tile of T consecutive instances; x, g, jac (and grad) of the whole tile
//     live in LDS ([T][n], [T][m], [T][nnz], [T][n]: the AoS image of the HBM records);
//   * the per-instance work is cut into segments (contact blocks in std::map order, the statics
//     values + force rows, the three torque rows, the cost) and every (segment, instance) work
//     item is one thread's job: 256 threads compute T*(N+4) items in lock-step;
//   * the finished tile is copied out linearly with 16-byte stores: tile boundaries fall on
//     128-byte lines (T*record is a multiple of 16 doubles), so every HBM line of g / jac is
//     written exactly once and whole.
// ------------------------------------------------------------------------------------------
// Segments: [0, N) contacts in map order, then N: statics values + rows 0-2, N+1..N+3: torque
// rows 3..5, N+4: cost (optional).

template <int WG>
__device__ __forceinline__ void copy_in(double* __restrict__ dst, const double* __restrict__ src, int count,
                                        int tid, bool vec) {
  if (vec) {
    const int pairs = count >> 1;
    const double2* s2 = reinterpret_cast<const double2*>(src);
    double2* d2 = reinterpret_cast<double2*>(dst);
    for (int e = tid; e < pairs; e += WG) d2[e] = s2[e];
    if ((count & 1) && tid == 0) dst[count - 1] = src[count - 1];
  } else {
    for (int e = tid; e < count; e += WG) dst[e] = src[e];
  }
}

// Entry-major ("SoA") copy-out of a tile image [valid][rec] to dst[q * batch + r] (dst = the
// output's base + the tile's first instance): lanes run along the instances, so each entry's run of
// the tile is one contiguous segment (512 B for a 64-instance tile).
template <int NTH, bool NT>
__device__ __forceinline__ void copy_out_soa(double* __restrict__ dst, int64_t batch, const double* __restrict__ src,
                                             int rec, int valid, int tid) {
  const int count = rec * valid;
  for (int e = tid; e < count; e += NTH) {
    const int q = e / valid, r = e - q * valid;
    const double v = src[r * rec + q];
    double* d = dst + (int64_t)q * batch + r;
    if (NT) __builtin_nontemporal_store(v, d);
    else *d = v;
  }
}

template <int WG, bool NT>
__device__ __forceinline__ void copy_out(double* __restrict__ dst, const double* __restrict__ src, int count,
                                         int tid) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int pairs = count >> 1;
    const double2* s2 = reinterpret_cast<const double2*>(src);
    double2* d2 = reinterpret_cast<double2*>(dst);
    for (int e = tid; e < pairs; e += WG) {
      if (NT) {
        const double2 v = s2[e];
        __builtin_nontemporal_store(v.x, &d2[e].x);
        __builtin_nontemporal_store(v.y, &d2[e].y);
      } else {
        d2[e] = s2[e];
      }
    }
    if ((count & 1) && tid == 0) dst[count - 1] = src[count - 1];
  } else {
    for (int e = tid; e < count; e += WG) dst[e] = src[e];
  }
}

// Copy-out of a tile image [valid][rec] to the records of instances rowb[r] (rec even: every record
// and every pair of it is 16-byte aligned), 16-byte stores: one record per wave at a time, lanes along
// it, so the record's address is wave-uniform (scalar) and each lane adds only its own offset — the
// flattened (row, pair) walk over the workgroup had cost a 64-bit index product per pair (the list
// tiles issued ~30 % more VALU instructions than the contiguous ones)
template <int WG, bool NT>
__device__ __forceinline__ void copy_out_rows(double* __restrict__ dst, const long long* __restrict__ rowb,
                                              const double* __restrict__ src, int rec, int valid, int tid) {
  const int r2 = rec >> 1;
  const int wave = tid >> 6, lane = tid & 63;
  const double2* s2 = reinterpret_cast<const double2*>(src);
  for (int r = wave; r < valid; r += WG / 64) {
    const int b = __builtin_amdgcn_readfirstlane((int)rowb[r]);
    double2* d = reinterpret_cast<double2*>(dst + (int64_t)b * rec);
    const double2* sr = s2 + r * r2;
    for (int q = lane; q < r2; q += 64) {
      const double2 v = sr[q];
      if (NT) {
        __builtin_nontemporal_store(v.x, &d[q].x);
        __builtin_nontemporal_store(v.y, &d[q].y);
      } else {
        d[q] = v;
      }
    }
  }
}

// one contact block (map position k, vector index i): g rows env(1) normal(3) cone(2),
// jac rows env p(3) | normal r: p(3) n_r(1) | cone 0: F(3) n(3) | cone 1: F(3) n(3)
template <int ENVK>
__device__ __forceinline__ void contact_item(const KParams& K, const double* __restrict__ xr, int kind, int k,
                                             double* __restrict__ Gr, double* __restrict__ Jr) {
  const int i = s_ct.map_order[k];
  const double* q = xr + 3 + 9 * i;
  const double F0 = q[0], F1 = q[1], F2 = q[2];
  const double p0 = q[3], p1 = q[4], p2 = q[5];
  const double n0 = q[6], n1 = q[7], n2 = q[8];
  const bool wg = K.want_g, wj = K.want_j;
  double* gk = Gr + 6 + (K.has_env ? 6 : 2) * k;
  double* jk = Jr + K.jbase + K.cstride * k;
  if (ENVK != CPL_ENV_NONE) {
    double gv[4], ej[3], nj[3][3];
    if (ENVK == CPL_ENV_GROUND || (ENVK == CPL_ENV_MIXED && kind == CPL_ENV_GROUND)) {
      // src/Ground.cpp:23-50
      gv[0] = p2 - K.ground_z;
      gv[1] = n0 - 0.0; gv[2] = n1 - 0.0; gv[3] = n2 - 1.0;
      ej[0] = 0.0; ej[1] = 0.0; ej[2] = 1.0;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) nj[r][c] = 0.0;
    } else {
      SQContact s;
      superquadric_contact(K, p0, p1, p2, wj, s);
      gv[0] = s.val;
      gv[1] = n0 - s.en[0]; gv[2] = n1 - s.en[1]; gv[3] = n2 - s.en[2];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        ej[r] = s.ej[r];
#pragma unroll
        for (int c = 0; c < 3; ++c) nj[r][c] = wj ? s.nj[r][c] : 0.0;
      }
    }
    if (wg) { gk[0] = gv[0]; gk[1] = gv[1]; gk[2] = gv[2]; gk[3] = gv[3]; }
    if (wj && K.fold == FOLD_NONE) {
      jk[0] = ej[0]; jk[1] = ej[1]; jk[2] = ej[2];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        jk[3 + 4 * r] = nj[r][0]; jk[4 + 4 * r] = nj[r][1]; jk[5 + 4 * r] = nj[r][2]; jk[6 + 4 * r] = 1.0;
      }
      jk += 15;
    } else if (wj && K.fold == FOLD_COMMON) {  // values only: the normal rows' n_r entry (1) skipped
      jk[0] = ej[0]; jk[1] = ej[1]; jk[2] = ej[2];
#pragma unroll
      for (int r = 0; r < 3; ++r) { jk[3 + 3 * r] = nj[r][0]; jk[4 + 3 * r] = nj[r][1]; jk[5 + 3 * r] = nj[r][2]; }
      jk += 12;
    }  // FOLD_GROUND: the Ground gradient (0,0,1), the zero normal Jacobian and the ones are all constant
    gk += 4;
  }
  // FrictionCone, src/Constraints/FrictionCone.cpp:30-103
  const double mu = K.mu;
  const double t1 = dot3(F0, F1, F2, n0, n1, n2);
  if (wg) {
    const double nF = dot3(n0, n1, n2, F0, F1, F2);
    const double u0 = F0 - nF * n0, u1 = F1 - nF * n1, u2 = F2 - nF * n2;
    gk[0] = -t1 + s_ct.F_thr[i];
    gk[1] = sqrt((u0 * u0 + u1 * u1) + u2 * u2) - mu * t1;
  }
  if (wj) {
    const double t2 = F0 - n0 * t1;
    const double t3 = F1 - n1 * t1;
    const double t4 = F2 - n2 * t1;
    const double t5 = F0 * n0;
    const double t6 = F1 * n1;
    const double t7 = F2 * n2;
    const double s = sqrt(t2 * t2 + t3 * t3 + t4 * t4);
    jk[0] = -n0; jk[1] = -n1; jk[2] = -n2;
    jk[3] = -F0; jk[4] = -F1; jk[5] = -F2;
    jk[6] = (t2 * (n0 * n0 - 1.0) * 2.0 + n0 * n1 * t3 * 2.0 + n0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n0;
    jk[7] = (t3 * (n1 * n1 - 1.0) * 2.0 + n0 * n1 * t2 * 2.0 + n1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n1;
    jk[8] = (t4 * (n2 * n2 - 1.0) * 2.0 + n0 * n2 * t2 * 2.0 + n1 * n2 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n2;
    jk[9] = (t2 * (t6 + t7 + t5 * 2.0) * 2.0 + F0 * n1 * t3 * 2.0 + F0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F0;
    jk[10] = (t3 * (t5 + t7 + t6 * 2.0) * 2.0 + F1 * n0 * t2 * 2.0 + F1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F1;
    jk[11] = (t4 * (t5 + t6 + t7 * 2.0) * 2.0 + F2 * n0 * t2 * 2.0 + F2 * n1 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F2;
  }
}

// CentroidalStatics::GetValues (src/Constraints/CentroidalStatics.cpp:37-61) and Jacobian rows 0-2
// (the I3 of every F_i, :93-95)
// pairs_j: the torque rows' CoM pairs written straight to their Jacobian entries (row q's first two)
// instead of com6 — the Superquadric tile, whose cone items write the rows' per-contact entries
__device__ __forceinline__ void statics_values_item(const KParams& K, const double* __restrict__ xr, double m_i,
                                                    double* __restrict__ Gr, double* __restrict__ Jr,
                                                    bool with_j = true, double* __restrict__ com6 = nullptr,
                                                    bool pairs_j = false) {
  const int N = K.N;
  if (pairs_j && K.want_j) {
    com6 = Jr + (K.fold == FOLD_NONE ? 3 * N : 0);  // row q's pair at com6[q * (2 + 4N) + {0, 1}]
  }
  const bool pairs = com6 != nullptr, vals = K.want_g != 0;
  if (pairs || vals) {
    // com6: the torque rows' CoM pairs (statics_row_item's a1, a2 for rows 3, 4, 5); vals: the six
    // statics values — every sum over the contacts in map order.  The contacts four at a time, their
    // map-order indices and x entries loaded before the sums (one contact per trip waited two
    // dependent LDS round trips each: the item was the longest of a 16-contact Superquadric tile's
    // first phase); each sum's order unchanged (bitwise)
    const double c0 = xr[0], c1 = xr[1], c2 = xr[2];
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, v5 = 0.0;
    double a[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < N; k0 += 4) {
      double q[4][6];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double* qq = xr + 3 + 9 * s_ct.map_order[k0 + u < N ? k0 + u : k0];
#pragma unroll
        for (int e = 0; e < 6; ++e) q[u][e] = qq[e];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u >= N) break;
        const double F0 = q[u][0], F1 = q[u][1], F2 = q[u][2];
        if (pairs) {
          a[0] -= -(-1.0) * F2; a[1] -= -(1.0) * F1;   // row 3: (e1, s1) = (2, -), (e2, s2) = (1, +)
          a[2] -= -(1.0) * F2;  a[3] -= -(-1.0) * F0;  // row 4: (2, +), (0, -)
          a[4] -= -(-1.0) * F1; a[5] -= -(1.0) * F0;   // row 5: (1, -), (0, +)
        }
        if (vals) {
          const double d0 = q[u][3] - c0, d1 = q[u][4] - c1, d2 = q[u][5] - c2;
          v0 += F0; v1 += F1; v2 += F2;
          v3 += d1 * F2 - d2 * F1;
          v4 += d2 * F0 - d0 * F2;
          v5 += d0 * F1 - d1 * F0;
        }
      }
    }
    if (pairs) {
      if (pairs_j) {
#pragma unroll
        for (int t = 0; t < 6; ++t) com6[(t >> 1) * (2 + 4 * N) + (t & 1)] = a[t];
      } else {
#pragma unroll
        for (int t = 0; t < 6; ++t) com6[t] = a[t];
      }
    }
    if (vals) {
      v0 -= K.wrench[0]; v1 -= K.wrench[1]; v2 -= K.wrench[2];
      v3 -= K.wrench[3]; v4 -= K.wrench[4]; v5 -= K.wrench[5];
      v0 += m_i * K.gravity[0]; v1 += m_i * K.gravity[1]; v2 += m_i * K.gravity[2];
      Gr[0] = v0; Gr[1] = v1; Gr[2] = v2; Gr[3] = v3; Gr[4] = v4; Gr[5] = v5;
    }
  }
  if (with_j && K.want_j && K.fold == FOLD_NONE)  // folded layouts skip the constant I3 blocks
    for (int e = 0; e < 3 * N; ++e) Jr[e] = 1.0;
}

// The statics Jacobian rows of one instance (statics_values_item's I3 blocks and statics_row_item's
// three torque rows), entry by entry with the lanes along the record: every value is the expression
// the two items compute (the CoM pairs' sums in map order), but consecutive lanes write consecutive
// doubles — where the records are written straight to HBM (tile kernel JD) one thread per row issued
// 50-70 stores to 50-70 different lines per wave instruction.
__device__ __forceinline__ void statics_rows_coop(const KParams& K, const double* __restrict__ xr,
                                                  const double* __restrict__ com6, double* __restrict__ Jr, int tid,
                                                  int nthreads) {
  const int N = K.N;
  const int RL = 2 + 4 * N;
  const int I3 = K.fold == FOLD_NONE ? 3 * N : 0;
  const int SJ = I3 + 3 * RL;
  for (int e = tid; e < SJ; e += nthreads) {
    double v = 1.0;
    if (e >= I3) {
      int w = e - I3;
      const int q = w >= 2 * RL ? 2 : (w >= RL ? 1 : 0);
      w -= q * RL;
      const int e1 = q == 2 ? 1 : 2;
      const int e2 = q == 0 ? 1 : 0;
      const double s1 = q == 1 ? 1.0 : -1.0;
      const double s2 = q == 1 ? -1.0 : 1.0;
      if (w < 2) {  // the CoM pair (summed by statics_values_item in map order)
        v = com6[2 * q + w];
      } else {
        const int i = (w - 2) >> 2, c = (w - 2) & 3;
        const double* F = xr + 3 + 9 * i;
        const double* p = F + 3;
        v = c == 0 ? s1 * (p[e1] - xr[e1]) : c == 1 ? s2 * (p[e2] - xr[e2]) : c == 2 ? -s1 * F[e1] : -s2 * F[e2];
      }
    }
    Jr[e] = v;
  }
}

// Torque row 3+q of CentroidalStatics::FillJacobianBlock (src/Constraints/CentroidalStatics.cpp:75-137):
// [CoM pair | per contact in column order: F pair, p pair].  For row q the F pair is
// (sF1*(p[e1]-c[e1]), sF2*(p[e2]-c[e2])) and the p pair / CoM accumulation uses (-sF1*F[e1], -sF2*F[e2]);
// negation is exact, so every entry keeps the reference's bits.
__device__ __forceinline__ void statics_row_item(const KParams& K, const double* __restrict__ xr, int q,
                                                 double* __restrict__ Jr) {
  const int N = K.N;
  // (e1, e2) and sign of the F-block entries: row3 (2,-)(1,+), row4 (2,+)(0,-), row5 (1,-)(0,+)
  const int e1 = q == 2 ? 1 : 2;
  const int e2 = q == 0 ? 1 : 0;
  const double s1 = q == 1 ? 1.0 : -1.0;
  const double s2 = q == 1 ? -1.0 : 1.0;
  const double ce1 = xr[e1], ce2 = xr[e2];
  double a1 = 0.0, a2 = 0.0;
  for (int k = 0; k < N; ++k) {  // CoM block: -= the p-block entries in map order (:119-136)
    const double* F = xr + 3 + 9 * s_ct.map_order[k];
    a1 -= -s1 * F[e1];
    a2 -= -s2 * F[e2];
  }
  double* row = Jr + (K.fold == FOLD_NONE ? 3 * N : 0) + q * (2 + 4 * N);
  row[0] = a1;
  row[1] = a2;
  for (int i = 0; i < N; ++i) {
    const double* F = xr + 3 + 9 * i;
    const double* p = F + 3;
    row[2 + 4 * i] = s1 * (p[e1] - ce1);
    row[3 + 4 * i] = s2 * (p[e2] - ce2);
    row[4 + 4 * i] = -s1 * F[e1];
    row[5 + 4 * i] = -s2 * F[e2];
  }
}

// MinimizeCentroidalVariables::GetCost / FillJacobianBlock, src/MinimizeCentroidalVariables.cpp:124-192
__device__ __forceinline__ double cost_value(const KParams& K, const double* __restrict__ xr) {
  const int N = K.N;
  double value = 0;
  for (int k = 0; k < N; ++k) {
    const int i = s_ct.map_order[k];
    const double* q = xr + 3 + 9 * i;
    const double e0 = q[3] - K.p_ref[i][0], e1 = q[4] - K.p_ref[i][1], e2 = q[5] - K.p_ref[i][2];
    const double h0 = q[0] - K.F_ref[i][0], h1 = q[1] - K.F_ref[i][1], h2 = q[2] - K.F_ref[i][2];
    value += 0.5 * K.W_p[i] * ((e0 * e0 + e1 * e1) + e2 * e2) + 0.5 * K.W_F[i] * ((h0 * h0 + h1 * h1) + h2 * h2);
  }
  const double r0 = xr[0] - K.com_ref[0], r1 = xr[1] - K.com_ref[1], r2 = xr[2] - K.com_ref[2];
  value += 0.5 * K.W_com * ((r0 * r0 + r1 * r1) + r2 * r2);
  return value;
}

__device__ __forceinline__ void cost_item(const KParams& K, const double* __restrict__ xr, double* __restrict__ f,
                                          double* __restrict__ Dr, const double* __restrict__ fscale = nullptr) {
  const int N = K.N;
  const double c0 = xr[0], c1 = xr[1], c2 = xr[2];
  if (K.want_f) *f = fscale ? cost_value(K, xr) * *fscale : cost_value(K, xr);
  if (K.want_grad) {
    Dr[0] = K.W_com * (c0 - K.com_ref[0]);
    Dr[1] = K.W_com * (c1 - K.com_ref[1]);
    Dr[2] = K.W_com * (c2 - K.com_ref[2]);
    for (int i = 0; i < N; ++i) {
      const double* q = xr + 3 + 9 * i;
      double* d = Dr + 3 + 9 * i;
      d[0] = K.W_F[i] * (q[0] - K.F_ref[i][0]);
      d[1] = K.W_F[i] * (q[1] - K.F_ref[i][1]);
      d[2] = K.W_F[i] * (q[2] - K.F_ref[i][2]);
      d[3] = K.W_p[i] * (q[3] - K.p_ref[i][0]);
      d[4] = K.W_p[i] * (q[4] - K.p_ref[i][1]);
      d[5] = K.W_p[i] * (q[5] - K.p_ref[i][2]);
      d[6] = 0.0; d[7] = 0.0; d[8] = 0.0;
    }
  }
}


// ---- Superquadric contacts in two phases (tile kernel) -----------------------------------
// Phase 1, one item per (instance, contact, axis): the powers of d = p_a - C_a and
// ((p_a - C_a)/R_a)^P_a, and 1/(C_a - p_a)^2, into an LDS scratch row of SQ_L doubles per contact.
// Phase 2, one item per (instance, contact, normal-Jacobian row): the three entries of that row
// from the scratch; row 0 also emits the environment value / Jacobian / normal, row 1 the cone.
// The environment-value term of axis a, pow((p_a-C_a)/R_a, P_a), is parked in the contact's
// normal-residual slot a of the staged g row (g[1+a] of the contact block): the phase-2 row-0 item
// sums the three terms before it overwrites those slots with the normal residuals.  Keeping it out
// of the scratch (18 instead of 21 doubles per contact) fits the 8-contact tile in 40 KiB of LDS,
// i.e. four resident workgroups per CU instead of three.
constexpr int SQ_L = 18;  // per contact: 3 axes x {pm1, pP, p2Pm3, p2Pm2, p2P, inv}
enum { L_PM1 = 0, L_PP, L_P2PM3, L_P2PM2, L_P2P, L_INV, L_AXIS };

template <bool AXL>
__device__ __forceinline__ void sq_axis_item(const KParams& K, const double* __restrict__ xr, int k, int a,
                                             double* __restrict__ Lc, double* __restrict__ Gr) {
  const int i = s_ct.map_order[k];
  const double pa = xr[6 + 9 * i + a];
  const double d = -axv<AXL>(K, AX_C, a) + pa;
  double* o = Lc + a * L_AXIS;
  if (K.want_g) {
    // src/Superquadric.cpp:45  pow((p-C)/R, P)
    const double u = (pa - axv<AXL>(K, AX_C, a)) / axv<AXL>(K, AX_R, a);
    double w;
    if (K.sq_ladder && fabs(u) >= DD_TINY && fabs(u) <= 0x1p+40) {
      w = dd_ipow(u, (unsigned)axv<AXL>(K, AX_P, a)).hi;
      if (!(fabs(w) >= DD_TINY && fabs(w) <= DD_HUGE)) w = cpow(u, axv<AXL>(K, AX_P, a));
    } else {
      w = cpow(u, axv<AXL>(K, AX_P, a));
    }
    Gr[6 + 6 * k + 1 + a] = w;
  }
  if (K.want_j) {
    AxisPowers ap;
    axis_powers_ax<AXL>(K, K.sq_ladder != 0, a, d, ap);
    o[L_PM1] = ap.pm1;
    o[L_PP] = ap.pP;
    o[L_P2PM3] = ap.p2Pm3;
    o[L_P2PM2] = ap.p2Pm2;
    o[L_P2P] = ap.p2P;
    const double t = axv<AXL>(K, AX_C, a) - pa;
    o[L_INV] = 1.0 / (t * t);
  } else {
    o[L_PM1] = cpow(d, axv<AXL>(K, AX_PM1, a));  // src/Superquadric.cpp:54-56 (normal value only)
  }
}

// FrictionCone rows of one contact (src/Constraints/FrictionCone.cpp:30-103)
__device__ __forceinline__ void cone_rows(const KParams& K, int i, const double* __restrict__ q, double* gk,
                                          double* jk) {
  const double F0 = q[0], F1 = q[1], F2 = q[2];
  const double n0 = q[6], n1 = q[7], n2 = q[8];
  const double mu = K.mu;
  const double t1 = dot3(F0, F1, F2, n0, n1, n2);
  if (K.want_g) {
    const double nF = dot3(n0, n1, n2, F0, F1, F2);
    const double u0 = F0 - nF * n0, u1 = F1 - nF * n1, u2 = F2 - nF * n2;
    gk[0] = -t1 + s_ct.F_thr[i];
    gk[1] = sqrt((u0 * u0 + u1 * u1) + u2 * u2) - mu * t1;
  }
  if (K.want_j) {
    const double t2 = F0 - n0 * t1;
    const double t3 = F1 - n1 * t1;
    const double t4 = F2 - n2 * t1;
    const double t5 = F0 * n0;
    const double t6 = F1 * n1;
    const double t7 = F2 * n2;
    const double s = sqrt(t2 * t2 + t3 * t3 + t4 * t4);
    jk[0] = -n0; jk[1] = -n1; jk[2] = -n2;
    jk[3] = -F0; jk[4] = -F1; jk[5] = -F2;
    jk[6] = (t2 * (n0 * n0 - 1.0) * 2.0 + n0 * n1 * t3 * 2.0 + n0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n0;
    jk[7] = (t3 * (n1 * n1 - 1.0) * 2.0 + n0 * n1 * t2 * 2.0 + n1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n1;
    jk[8] = (t4 * (n2 * n2 - 1.0) * 2.0 + n0 * n2 * t2 * 2.0 + n1 * n2 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n2;
    jk[9] = (t2 * (t6 + t7 + t5 * 2.0) * 2.0 + F0 * n1 * t3 * 2.0 + F0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F0;
    jk[10] = (t3 * (t5 + t7 + t6 * 2.0) * 2.0 + F1 * n0 * t2 * 2.0 + F1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F1;
    jk[11] = (t4 * (t5 + t6 + t7 * 2.0) * 2.0 + F2 * n0 * t2 * 2.0 + F2 * n1 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F2;
  }
}

// CONE = false: the row-1 item leaves the contact's friction cone to a separate item (sq_cone_item).
// AF >= 0: the axis a compile-time constant (a == AF): the three entries' chains in one basic block
template <bool AXL, bool CONE = true, int AF = -1>
__device__ __forceinline__ void sq_row_item(const KParams& K, const double* __restrict__ xr, int k, int a_arg,
                                            const double* __restrict__ Lc, double* __restrict__ Gr,
                                            double* __restrict__ Jr) {
  const int a = AF >= 0 ? AF : a_arg;
  const int i = s_ct.map_order[k];
  const double* q = xr + 3 + 9 * i;
  double* gk = Gr + 6 + 6 * k;
  double* jk = Jr + K.jbase + K.cstride * k;
  const bool fold = K.fold != FOLD_NONE;  // Superquadric / mixed fold: FOLD_COMMON
  if (a == 0) {
    // EnvironmentConstraint / EnvironmentNormal values and the env Jacobian row
    // (src/Superquadric.cpp:40-69; src/Constraints/EnvironmentConstraint.cpp:16-61; EnvironmentNormal.cpp:16-33)
    double v = 0.0;
    if (K.want_g) {  // the three terms parked by sq_axis_item
      v += gk[1];
      v += gk[2];
      v += gk[3];
      v -= 1.0;
    }
    const double ej0 = axv<AXL>(K, AX_EJ, 0) * Lc[0 * L_AXIS + L_PM1];
    const double ej1 = axv<AXL>(K, AX_EJ, 1) * Lc[1 * L_AXIS + L_PM1];
    const double ej2 = axv<AXL>(K, AX_EJ, 2) * Lc[2 * L_AXIS + L_PM1];
    const double nrm = sqrt((ej0 * ej0 + ej1 * ej1) + ej2 * ej2);
    if (K.want_g) {
      gk[0] = v;
      gk[1] = q[6] - -ej0 / nrm;
      gk[2] = q[7] - -ej1 / nrm;
      gk[3] = q[8] - -ej2 / nrm;
    }
    if (K.want_j) { jk[0] = ej0; jk[1] = ej1; jk[2] = ej2; }
  } else if (CONE && a == 1) {
    cone_rows(K, i, q, gk + 4, jk + (fold ? 12 : 15));
  }
  if (!K.want_j) return;
  // EnvironmentNormal p block row a = GetNormalJacobian row a (src/Superquadric.cpp:72-209), n_a = 1
  const int b = a == 0 ? 1 : 0;
  const int c = a == 2 ? 1 : 2;
  const double* La = Lc + a * L_AXIS;
  const double* Lb = Lc + b * L_AXIS;
  const double* Lcc = Lc + c * L_AXIS;
  const double p_b = q[3 + b], p_c = q[3 + c];
  double out[3];
  {  // diagonal (a, a)
    double lead = axv<AXL>(K, AX_KA, a);
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      lead = lead * (kk == a ? La[L_PP] : axv<AXL>(K, AX_RM2, kk));
      lead = lead * Lc[kk * L_AXIS + L_INV];
    }
    lead = lead * axv<AXL>(K, AX_PM1, a);
    lead = lead * 1.0;
    const double Tb = ((axv<AXL>(K, AX_RM2, b) * Lb[L_INV]) * axv<AXL>(K, AX_PSQ, b)) * Lb[L_P2P];
    const double Tc = ((axv<AXL>(K, AX_RM2, c) * Lcc[L_INV]) * axv<AXL>(K, AX_PSQ, c)) * Lcc[L_P2P];
    const double Dg = (axv<AXL>(K, AX_KB, a) * La[L_P2P]) * La[L_INV];
    const double S = (Tb + Tc) + Dg;
    const double p2Pb = Lb[L_P2P], p2Pc = Lcc[L_P2P];
    const double E = (((((((axv<AXL>(K, AX_C, b) * axv<AXL>(K, AX_C, b)) * axv<AXL>(K, AX_PSQ, c)) * p2Pc) * axv<AXL>(K, AX_RP2, b) +
                         (((axv<AXL>(K, AX_C, c) * axv<AXL>(K, AX_C, c)) * axv<AXL>(K, AX_PSQ, b)) * p2Pb) * axv<AXL>(K, AX_RP2, c)) +
                        (((p_b * p_b) * axv<AXL>(K, AX_PSQ, c)) * p2Pc) * axv<AXL>(K, AX_RP2, b)) +
                       (((p_c * p_c) * axv<AXL>(K, AX_PSQ, b)) * p2Pb) * axv<AXL>(K, AX_RP2, c)) -
                      ((((axv<AXL>(K, AX_C, b) * p_b) * axv<AXL>(K, AX_PSQ, c)) * p2Pc) * axv<AXL>(K, AX_RP2, b)) * 2.0) -
                     ((((axv<AXL>(K, AX_C, c) * p_c) * axv<AXL>(K, AX_PSQ, b)) * p2Pb) * axv<AXL>(K, AX_RP2, c)) * 2.0;
    out[a] = lead / pow_three_halves(S) * E;
  }
#pragma unroll
  for (int bb = 0; bb < 3; ++bb) {  // off-diagonals (a, bb)
    if (bb == a) continue;
    const int oo = 3 - a - bb;
    const double* Lbb = Lc + bb * L_AXIS;
    double lead = axv<AXL>(K, AX_KA, a);
    if (a < bb) {  // src/Superquadric.cpp:109, 119, 163
      lead = lead * La[L_PM1];
      lead = lead * axv<AXL>(K, AX_PSQ, bb);
      lead = lead * Lbb[L_P2PM3];
      lead = lead * axv<AXL>(K, AX_P2M2, bb);
    } else {       // src/Superquadric.cpp:129, 173, 183
      lead = lead * axv<AXL>(K, AX_PSQ, bb);
      lead = lead * Lbb[L_P2PM3];
      lead = lead * axv<AXL>(K, AX_P2M2, bb);
      lead = lead * La[L_PM1];
    }
    lead = lead * axv<AXL>(K, AX_RM2, bb);
    lead = lead * 1.0;
    const double S = (axv<AXL>(K, AX_KB, oo) * Lc[oo * L_AXIS + L_P2PM2] + axv<AXL>(K, AX_KB, a) * La[L_P2PM2]) +
                     (axv<AXL>(K, AX_PSQ, bb) * Lbb[L_P2PM2]) * axv<AXL>(K, AX_RM2, bb);
    out[bb] = lead / pow_three_halves(S) * (-1.0 / 2.0);
  }
  double* row = jk + 3 + (fold ? 3 : 4) * a;
  row[0] = out[0]; row[1] = out[1]; row[2] = out[2];
  if (!fold) row[3] = 1.0;
}

// the friction cone rows of contact block k (map order) of a Superquadric record, as sq_row_item's
// row-1 item computes them; statics (the Superquadric tile): also contact i's entries of the statics
// Jacobian — its three ones of the force rows and its four entries in each torque row, the values
// statics_row_item computes (the rows' CoM pairs: statics_values_item, pairs_j)
__device__ __forceinline__ void sq_cone_item(const KParams& K, const double* __restrict__ xr, int k,
                                             double* __restrict__ Gr, double* __restrict__ Jr,
                                             bool statics = false) {
  const int i = s_ct.map_order[k];
  cone_rows(K, i, xr + 3 + 9 * i, Gr + 6 + 6 * k + 4, Jr + K.jbase + K.cstride * k + (K.fold != FOLD_NONE ? 12 : 15));
  if (!statics || !K.want_j) return;
  const int N = K.N;
  if (K.fold == FOLD_NONE) { Jr[3 * k] = 1.0; Jr[3 * k + 1] = 1.0; Jr[3 * k + 2] = 1.0; }  // (3N ones, any order)
  const double* F = xr + 3 + 9 * i;
  const double* p = F + 3;
  double* rows = Jr + (K.fold == FOLD_NONE ? 3 * N : 0) + 2 + 4 * i;
#pragma unroll
  for (int q = 0; q < 3; ++q) {  // (e1, e2) and signs as statics_row_item
    const int e1 = q == 2 ? 1 : 2;
    const int e2 = q == 0 ? 1 : 0;
    const double s1 = q == 1 ? 1.0 : -1.0;
    const double s2 = q == 1 ? -1.0 : 1.0;
    double* row = rows + q * (2 + 4 * N);
    row[0] = s1 * (p[e1] - xr[e1]);
    row[1] = s2 * (p[e2] - xr[e2]);
    row[2] = -s1 * F[e1];
    row[3] = -s2 * F[e2];
  }
}

// JD: the Jacobian items write their entries straight to the output records (K.jdirect); a
// compile-time choice, so that every Jacobian store is a plain LDS or a plain global store: through a
// generic pointer they were FLAT stores, which count on lgkmcnt too — every later LDS wait of the
// thread then waited for its in-flight global stores.
// idx (optional, with d_count on the device): an instance list — tile position j evaluates instance
// idx[j] and its records are written in place (the Superquadric half of a mixed batch, launched for
// `batch` list entries at most; tiles past *d_count only write zero norm partials).  Not with JD / SoA.
// LIST (compile time): the tile rows are the instances idx[b0 ..] of a device-side instance list of
// *d_count entries (the kind split's Superquadric half), records written in place; the grid covers the
// largest possible list (batch / T tiles) and the workgroups past the list's tiles only write zero
// residual partials.  Without LIST the kernel is the contiguous one-tile-per-workgroup form (111
// VGPRs for Superquadric; a runtime list pointer and a tile loop in the same body had cost 162 VGPRs
// and a 36-byte spill, three waves per SIMD instead of four).
// The LDS-staged list tiles (the split's default Superquadric half) are held to four waves per SIMD:
// uncapped they took 129 VGPRs — two past the four-wave step — and ran three workgroups per CU where the
// contiguous tiles run four (127 with 2 spilled: the all-Superquadric 524 288 x 16 list 1.93 -> 1.53 ms,
// the 8-GPU shard of configs[3] 0.355 -> 0.317 ms, 1 048 576 x 16 50 / 50 +1.6 %; profiles/r6/split/)
template <int ENVK, int WG, bool NT, bool JD, bool LIST = false>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(LIST && !JD ? 4 : 1)))
void cpl_eval_tile_kernel(const KParams K, int64_t batch,
                                                            const double* __restrict__ x,
                                                            const double* __restrict__ mass,
                                                            const uint8_t* __restrict__ env_tag,
                                                            const int32_t* __restrict__ idx,
                                                            const int32_t* __restrict__ d_count,
                                                            double* __restrict__ g_out,
                                                            double* __restrict__ jac_out,
                                                            double* __restrict__ f_out,
                                                            double* __restrict__ grad_out,
                                                            double* __restrict__ norms_ws) {
  extern __shared__ __align__(16) double smem[];
  const int tid = threadIdx.x;
  const int T = K.T;
  const int n = K.n, m = K.m, nnz = K.nnz, N = K.N;
  const int64_t count = LIST ? (int64_t)*d_count : batch;
  // LIST: one workgroup per tile the list may hold (the list's length is known on the device only; a
  // persistent walk over the list's tiles measured slower: 149-155 VGPRs against 114, three waves per
  // SIMD instead of four — profiles/r4/ab_split5; and again in round 5 with the next tile's x
  // prefetched into registers, for the contiguous Superquadric tiles too: 149-165 VGPRs, sq8 0.395
  // against 0.307 ms, profiles/r5/).  The workgroups past the list's tiles leave before the table load.
  const int64_t b0 = (int64_t)blockIdx.x * T;
  // (LIST) the tile's list entries loaded before the list's length is known — the workspace holds
  // `batch` entries, so b0 + r < batch is in bounds (entries past the length are never used): the
  // length, then the entries, then the rows had been three dependent HBM round trips before any
  // compute (~10 % of a list tile's life; the contiguous tiles pay one)
  const int wave0 = tid >> 6;
  int spec_b = 0;
  long long spec_rb = 0;
  if (LIST) {
    if (b0 + wave0 < batch) spec_b = idx[b0 + wave0];
    if (tid < T && b0 + tid < batch) spec_rb = idx[b0 + tid];
  }
  if (LIST && b0 >= count) {  // past the list's tiles: zero partials
    NormAcc nacc;
    if (K.want_norms) partial_norms_waves(nacc, norms_ws + NORM_HDR, blockIdx.x);
    return;
  }
  load_ctab(K);
  __syncthreads();
  double mass_def = K.mass_default;  // a value (see cpl_eval_pipe_kernel)
  asm volatile("" : "+v"(mass_def));
  const int valid = (int)((count - b0) < T ? (count - b0) : T);
  long long* rowb = reinterpret_cast<long long*>(smem + K.offRB);  // (LIST) instance of each tile row
  auto inst = [&](int r) -> int64_t { return LIST ? (int64_t)rowb[r] : b0 + r; };
  double* X = smem;
  double* Gt = smem + K.offG;
  // the Jacobian rows: the LDS tile image, or (jdirect) the output records themselves
  double* Jt = JD ? jac_out + b0 * K.nnz : smem + K.offJ;
  // row r's Jacobian: the LDS image's, or (JD) the output record itself — of instance rowb[r] in a
  // list launch
  auto JR = [&](int r) -> double* { return (JD && LIST) ? jac_out + rowb[r] * nnz : Jt + r * nnz; };
  double* Dt = smem + K.offD;
  double* L = smem + K.offL;                                    // [T][LR] (SQ / mixed)
  int* lists = reinterpret_cast<int*>(smem + K.offI);          // sq_list[64], gr_list[64], n_sq
  constexpr bool HAS_SQ = ENVK == CPL_ENV_SUPERQUADRIC || ENVK == CPL_ENV_MIXED;

  if (LIST) {
    if (tid < valid) rowb[tid] = spec_rb;  // (published by the barrier before phase 1)
    // the tile's rows gathered through the list: one row per wave at a time, its source address
    // wave-uniform (the list entry a scalar load), lanes along the row, every load of a wave's rows
    // issued before their LDS stores (a flattened (row, column) walk with a 64-bit index product per
    // element had cost the list tiles ~30 % more VALU instructions than the contiguous copy-in)
    // (Superquadric list tiles, the mixed split's Superquadric half: the gather and the copy-out at a
    // raised wave priority: mixed16 2.35 -> 2.28 ms with the 4-instance LDS-staged tiles, r6)
    if (ENVK == CPL_ENV_SUPERQUADRIC && K.list_prio) __builtin_amdgcn_s_setprio(2);
    const int wave = tid >> 6, lane = tid & 63;
    constexpr int U = 4;  // (rows of up to 4 * 64 doubles in one pass)
    int bnext = spec_b;  // (row `wave`'s entry, loaded at the kernel's start)
    for (int r = wave; r < valid; r += WG / 64) {
      const int b = __builtin_amdgcn_readfirstlane(bnext);
      if (r + WG / 64 < valid) bnext = idx[b0 + r + WG / 64];
      const double* src = x + (int64_t)b * n;
      double* dst = X + r * n;
      for (int c0 = 0; c0 < n; c0 += U * 64) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int c = c0 + u * 64 + lane;
          v[u] = src[c < n ? c : n - 1];  // (a clamped address: a guarded load is a branch per element)
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int c = c0 + u * 64 + lane;
          if (c < n) dst[c] = v[u];
        }
      }
    }
    if (ENVK == CPL_ENV_SUPERQUADRIC && K.list_prio) __builtin_amdgcn_s_setprio(0);
  } else {
    // Superquadric tiles of 8+ instances (sq8): the copy-in and the copy-out issued at a raised wave
    // priority, so that a workgroup's memory phases are not queued behind the other resident
    // workgroups' VALU chains (sq8 0.296 -> 0.288 ms; the 4-instance tiles of 16-contact records lost
    // 3 % with it, so they keep the default; profiles/r5/sq_prio/)
    if (ENVK == CPL_ENV_SUPERQUADRIC && T >= 8) __builtin_amdgcn_s_setprio(2);
    copy_in<WG>(X, x + b0 * n, valid * n, tid, K.x_aligned16 != 0);
    if (ENVK == CPL_ENV_SUPERQUADRIC && T >= 8) __builtin_amdgcn_s_setprio(0);
  }
  {
    int n_sq = ENVK == CPL_ENV_SUPERQUADRIC ? valid : 0;
    if (ENVK == CPL_ENV_MIXED) {
      // compact the tile's instances by environment kind so that every wave runs one code path
      if (tid < 64) {
        const bool is_sq = tid < valid && env_tag[b0 + tid] == CPL_ENV_SUPERQUADRIC;
        const unsigned long long mask = __ballot(is_sq);
        if (tid < valid) {
          const int before = __popcll(mask & ((1ull << tid) - 1ull));
          if (is_sq) lists[before] = tid;
          else lists[64 + tid - before] = tid;
        }
        if (tid == 0) lists[128] = __popcll(mask);
      }
    }
    __syncthreads();
    if (ENVK == CPL_ENV_MIXED) n_sq = lists[128];
    const int n_gr = valid - n_sq;
    const bool compute = K.ablate != 1;

    // ---- phase 1: the Superquadric power ladders (into the LDS scratch); phase 2: the Superquadric
    // rows.  The items that do not read the scratch (Ground / no-env contacts, statics, cost) join
    // phase 1 for Superquadric batches, so that the two barrier-separated phases carry comparable work
    // (sq8 0.347 -> 0.329 ms), and phase 2 for mixed batches, where the tile's Ground contacts then
    // overlap the Superquadric rows (3.50 -> 3.44 ms for mixed16; profiles/r3/ab_*).  SQ items run
    // axis-major (item -> (axis, contact, instance)).
    constexpr bool OTHERS_FIRST = ENVK != CPL_ENV_MIXED;
    const bool wgj = K.want_g || K.want_j;
    // Superquadric batches (UAX): the items of one axis are padded to whole waves (PA items, a multiple
    // of 64), so the axis is wave-uniform — a scalar: the per-axis factors are scalar operands, the
    // power ladders' exponent loops uniform (with a lane-varying axis every ladder was a divergent loop
    // and every factor a per-lane select) — and (contact, tile row) = (kj >> logT, kj & (T - 1)) with
    // the rows past `valid` idle (no divisions).  Mixed tiles keep the ballot-compacted mapping, and so
    // does the kind split's Superquadric half (LIST): beside the Ground half on the other stream the
    // uniform-axis form ran the 1 048 576 x 16 mixed batch 7 % slower (2.74 against 2.55 ms, although
    // an all-Superquadric list alone ran 4 % faster; profiles/r5/ab_uax_list).
    constexpr bool UAX = ENVK == CPL_ENV_SUPERQUADRIC && !(LIST && JD);
    const int per_axis = UAX ? (N << K.logT) : N * n_sq;
    const int PA = UAX ? ((per_axis + 63) & ~63) : per_axis;
    const int r_ax = (HAS_SQ && wgj) ? 3 * PA : 0;
    const int r_gr = (ENVK != CPL_ENV_SUPERQUADRIC && wgj) ? N * n_gr : 0;
    // (JD: the statics J rows by statics_rows_coop; Superquadric tiles (SQST): the rows' per-contact
    // entries by the cone items of phase 2, their CoM pairs by the values item — three serial
    // 2 + 4N-entry row items had bounded phase 1)
    constexpr bool SQST = ENVK == CPL_ENV_SUPERQUADRIC && !JD;
    const int r_st = wgj ? ((JD || SQST) ? 1 : 4) * valid : 0;
    double* com6 = smem + K.offA;                        // (JD) [T][6]
    const int r_co = K.cost_seg >= 0 ? valid : 0;
    const int r_oth = r_gr + r_st + r_co;
    auto other_item = [&](int e) {
      if (e < r_gr) {
        const int j = e % n_gr, k = e / n_gr;
        const int r = ENVK == CPL_ENV_MIXED ? lists[64 + j] : j;
        contact_item<ENVK == CPL_ENV_NONE ? CPL_ENV_NONE : CPL_ENV_GROUND>(K, X + r * n, CPL_ENV_GROUND, k,
                                                                          Gt + r * m, JR(r));
        return;
      }
      e -= r_gr;
      if (e < r_st) {
        const int r = e % valid, sg = e / valid;
        const double* xr = X + r * n;
        if (sg == 0)
          statics_values_item(K, xr, mass ? mass[inst(r)] : mass_def, Gt + r * m, JR(r), !JD && !SQST,
                              JD && K.want_j ? com6 + 6 * r : nullptr, SQST);
        else if (K.want_j) statics_row_item(K, xr, sg - 1, JR(r));
        return;
      }
      e -= r_st;
      cost_item(K, X + e * n, f_out ? f_out + inst(e) : nullptr, Dt + e * n);
    };
    // mixed: the statics / cost items join phase 1 (beside the Superquadric ladders), the Ground
    // contacts phase 2 (beside the Superquadric rows) — with 8-instance tiles both phases then fit
    // one pass of the workgroup (232 and 256 items at the 1:1 mix)
    // Each phase as two loops over the same item -> thread mapping (Superquadric items, then the
    // others): one item function per loop body, so the register allocation of the two does not add up.
    const int items1 = r_ax + (OTHERS_FIRST ? r_oth : r_oth - r_gr);
    if (compute) {
      if (HAS_SQ && UAX)
        for (int it = tid; it < r_ax; it += WG) {
          const int a = __builtin_amdgcn_readfirstlane(it) / PA, kj = it - a * PA;
          const int k = kj >> K.logT, r = kj & (T - 1);
          if (kj < per_axis && r < valid) sq_axis_item<false>(K, X + r * n, k, a, L + r * K.LR + k * SQ_L, Gt + r * m);
        }
      else if (HAS_SQ)
        for (int it = tid; it < r_ax; it += WG) {
          const int a = it / per_axis, kj = it - a * per_axis;
          const int k = kj / n_sq, j = kj - k * n_sq;
          const int r = ENVK == CPL_ENV_MIXED ? lists[j] : j;
          sq_axis_item<ENVK == CPL_ENV_MIXED>(K, X + r * n, k, a, L + r * K.LR + k * SQ_L, Gt + r * m);
        }
      for (int it = tid; it < items1; it += WG)
        if (it >= r_ax) other_item(it - r_ax + (OTHERS_FIRST ? 0 : r_gr));
    }
    // LDS-only barriers from here on: the phases exchange LDS data only, and a __syncthreads would
    // first wait for every global store the items issued (f, and with jdirect the Jacobian rows)
    // (measurement only, ablation 8192: the phases' barriers skipped — wrong outputs, the barriers' cost)
    const bool phase_bar = (K.ablate & 8192) == 0;
    if (compute && HAS_SQ && n_sq > 0 && wgj && phase_bar) lds_barrier();
    if (compute) {
      const int r_rows = r_ax;
      // Superquadric batches: the friction cones as items of their own in phase 2 (the workgroup's
      // fourth wave, otherwise idle there: the row-1 items no longer carry them)
      constexpr bool CONE_ITEMS = ENVK == CPL_ENV_SUPERQUADRIC;
      const int r_cone = (CONE_ITEMS && wgj) ? (N << K.logT) : 0;  // (slots (contact, row) = (e >> logT, e & (T - 1)))
      const int items2 = r_rows + (OTHERS_FIRST ? 0 : r_gr) + r_cone;
      if (HAS_SQ && UAX)
        for (int it = tid; it < r_rows; it += WG) {
          const int a = __builtin_amdgcn_readfirstlane(it) / PA, kj = it - a * PA;
          const int k = kj >> K.logT, r = kj & (T - 1);
          if (kj < per_axis && r < valid) {  // a wave-uniform: the row item specialised on its axis — the
            // three entries' chains in one basic block, interleaved (97 -> 127 VGPRs, still four waves
            // per SIMD; bitwise; sq8 0.316 -> 0.299 ms, profiles/r5/sq_rowaf/)
            double* const Lr = L + r * K.LR + k * SQ_L;
            if (a == 0) sq_row_item<false, !CONE_ITEMS, 0>(K, X + r * n, k, a, Lr, Gt + r * m, JR(r));
            else if (a == 1) sq_row_item<false, !CONE_ITEMS, 1>(K, X + r * n, k, a, Lr, Gt + r * m, JR(r));
            else sq_row_item<false, !CONE_ITEMS, 2>(K, X + r * n, k, a, Lr, Gt + r * m, JR(r));
          }
        }
      else if (HAS_SQ)
        for (int it = tid; it < r_rows; it += WG) {
          const int a = it / per_axis, kj = it - a * per_axis;
          const int k = kj / n_sq, j = kj - k * n_sq;
          const int r = ENVK == CPL_ENV_MIXED ? lists[j] : j;
          // (the list tiles' waves also share one axis, but the axis-specialised row items cost their
          // kernel 144-149 VGPRs (three waves per SIMD): 2.55 -> 2.84 ms for mixed16, 2.64 capped at
          // four waves with 8-12 spilled VGPRs; profiles/r5/sq_rowaf/)
          sq_row_item<ENVK == CPL_ENV_MIXED, !CONE_ITEMS>(K, X + r * n, k, a, L + r * K.LR + k * SQ_L, Gt + r * m,
                                                          JR(r));
        }
      for (int it = tid; it < items2; it += WG) {
        if (it < r_rows) continue;
        if (CONE_ITEMS) {
          const int e = it - r_rows, k = e >> K.logT, r = e & (T - 1);
          if (r < valid) sq_cone_item(K, X + r * n, k, Gt + r * m, JR(r), SQST);
        } else {
          other_item(it - r_rows);
        }
      }
      if (JD && K.want_j) {  // the statics Jacobian rows, lanes along each record
        lds_barrier();  // (the CoM pairs of the values items)
        for (int r = 0; r < valid; ++r) statics_rows_coop(K, X + r * n, com6 + 6 * r, JR(r), tid, WG);
      }
    }
    if (phase_bar) lds_barrier();
    if (ENVK == CPL_ENV_SUPERQUADRIC && (LIST ? K.list_prio != 0 : T >= 8)) __builtin_amdgcn_s_setprio(2);
    // the residual partials first (from the LDS image), so that their stores are in flight with the
    // copy-out's instead of after them on every workgroup's tail; one partial slot per tile
    if (K.want_norms) {
      NormAcc nacc;
      nacc.init(tid, WG, m);
      nacc.add_tile(Gt, valid * m, tid, WG, m);
      partial_norms_waves(nacc, norms_ws + NORM_HDR, blockIdx.x);
    }
    if (K.ablate != 2 && LIST) {  // records written in place: row by row (g, jac rows are 16-byte aligned)
      if (K.want_g) copy_out_rows<WG, NT>(g_out, rowb, Gt, m, valid, tid);
      if (K.want_j && !JD) copy_out_rows<WG, NT>(jac_out, rowb, Jt, nnz, valid, tid);
      if (K.want_grad)
        for (int e = tid; e < valid * n; e += WG) {
          const int r = e / n;
          grad_out[rowb[r] * n + (e - r * n)] = Dt[e];
        }
    } else if (K.ablate != 2 && K.soa) {
      if (K.want_g) copy_out_soa<WG, NT>(g_out + b0, batch, Gt, m, valid, tid);
      if (K.want_j) copy_out_soa<WG, NT>(jac_out + b0, batch, Jt, nnz, valid, tid);
      if (K.want_grad) copy_out_soa<WG, NT>(grad_out + b0, batch, Dt, n, valid, tid);
    } else if (K.ablate != 2) {
      if (K.want_g) copy_out<WG, NT>(g_out + b0 * m, Gt, valid * m, tid);
      if (K.want_j && !JD) copy_out<WG, NT>(jac_out + b0 * nnz, Jt, valid * nnz, tid);
      if (K.want_grad) copy_out<WG, NT>(grad_out + b0 * n, Dt, valid * n, tid);
    }
  }
}


// ------------------------------------------------------------------------------------------
// v3: persistent, warp-specialised pipeline over tiles.
//   * a workgroup = NCW compute waves + 1 loader wave, resident for the whole launch, walking tiles
//     blockIdx.x, blockIdx.x + gridDim.x, ...;
//   * the loader wave DMAs the NEXT tile's x into the other half of a double-buffered LDS image
//     (global_load_lds_dwordx4, 1 KiB per wave-instruction) and stages its masses / env tags, while
//     the compute waves evaluate the current tile; the loader issues no stores, so its vmcnt drain
//     waits for its own loads only;
//   * the compute waves issue no global loads and synchronise with LDS-only barriers
//     (s_waitcnt lgkmcnt(0) + s_barrier), so their output stores keep draining across tiles;
//   * work items and the full-line copy-out are those of the tile kernel above.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;


// loader wave: DMA `count` doubles (16-B aligned source) into LDS; the odd last double is returned
// through *tail for a plain store after the drain
__device__ __forceinline__ void dma_tile(double* dst, const double* src, int count, int lane) {
  const int pieces = (count + 127) >> 7;
  for (int p = 0; p < pieces; ++p) {
    const int e = p * 128 + lane * 2;
    if (e + 1 < count) __builtin_amdgcn_global_load_lds((glb_void_t*)(src + e), (lds_void_t*)(dst + p * 128), 16, 0, 0);
  }
}

template <int CT, bool NT>
__device__ __forceinline__ void copy_out_ct(double* __restrict__ dst, const double* __restrict__ src, int count,
                                            int tid) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int pairs = count >> 1;
    const double2* s2 = reinterpret_cast<const double2*>(src);
    double2* d2 = reinterpret_cast<double2*>(dst);
    for (int e = tid; e < pairs; e += CT) {
      const double2 v = s2[e];
      if (NT) {
        __builtin_nontemporal_store(v.x, &d2[e].x);
        __builtin_nontemporal_store(v.y, &d2[e].y);
      } else {
        d2[e] = v;
      }
    }
    if ((count & 1) && tid == 0) dst[count - 1] = src[count - 1];
  } else {
    for (int e = tid; e < count; e += CT) dst[e] = src[e];
  }
}

template <int ENVK, int NCW, bool NT, bool SC = false>
__global__ __launch_bounds__(64 * (NCW + 1)) void cpl_eval_pipe_kernel(const KParams K, int64_t batch,
                                                                        const double* __restrict__ x,
                                                                        const double* __restrict__ mass,
                                                                        const uint8_t* __restrict__ env_tag,
                                                                        double* __restrict__ g_out,
                                                                        double* __restrict__ jac_out,
                                                                        double* __restrict__ f_out,
                                                                        double* __restrict__ grad_out,
                                                                        double* __restrict__ norms_ws) {
  constexpr int CT = 64 * NCW;  // compute threads
  constexpr bool HAS_SQ = ENVK == CPL_ENV_SUPERQUADRIC || ENVK == CPL_ENV_MIXED;
  extern __shared__ __align__(16) double smem[];
  if (K.gate && *K.gate == 0) return;  // (every thread of every workgroup: the same byte)
  load_ctab(K);
  // fused Lagrangian gradient: the CSC index of the structure in LDS (read per column, per entry)
  int* s_colp = reinterpret_cast<int*>(smem + K.offC);
  int* s_csck = s_colp + K.n + 1;
  int* s_cscr = s_csck + K.nnz;
  if (K.want_lgrad) {
    for (int i = threadIdx.x; i <= K.n; i += blockDim.x) s_colp[i] = K.col_ptr[i];
    for (int i = threadIdx.x; i < K.nnz; i += blockDim.x) {
      s_csck[i] = K.csc_k[i];
      s_cscr[i] = K.csc_row[i];
    }
  }
  __syncthreads();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const bool loader = (tid >> 6) == NCW;
  const int T = K.T;
  const int n = K.n, m = K.m, nnz = K.nnz, N = K.N;
  const int64_t ntiles = (batch + T - 1) / T;
  // buffer selection by offset from smem (an array of pointers would lose the LDS address space
  // and turn every access into a flat access that also counts in vmcnt)
  auto XB = [&](int bi) { return smem + (bi ? K.offX1 : 0); };
  auto MB = [&](int bi) { return smem + K.offMB + (bi ? T : 0); };
  auto TB = [&](int bi) { return reinterpret_cast<int*>(smem + K.offTB) + (bi ? T : 0); };
  double* Gt = smem + K.offG;
  double* Jt = smem + K.offJ;
  double* Dt = smem + K.offD;
  double* L = smem + K.offL;
  int* lists = reinterpret_cast<int*>(smem + K.offI);

  int64_t t = blockIdx.x;
  if (t >= ntiles) return;  // (never: the host sizes the grid to at most ntiles)
  // the default mass as a value: `mass ? mass[i] : K.mass_default` would otherwise select between a
  // global and a kernarg address — a flat load, with a full vmcnt/lgkmcnt wait, in the loader loop
  double mass_def = K.mass_default;
  asm volatile("" : "+v"(mass_def));  // a value from here on, never re-read through its address
  NormAcc acc;
  acc.init(tid, CT, m);

  // loader: stage tile `tt` into buffer `bi`; loads only (the drain comes later)
  double st_mass = 0.0, st_tail = 0.0;
  int st_tag = 0;
  auto stage = [&](int64_t tt, int bi) {
    const int64_t b0s = tt * T;
    const int vs = (int)((batch - b0s) < T ? (batch - b0s) : T);
    const int count = vs * n;
    dma_tile(XB(bi), x + b0s * n, count, lane);
    if ((count & 1) && lane == 0) st_tail = x[b0s * n + count - 1];
    if (lane < vs) {
      st_mass = mass ? mass[b0s + lane] : mass_def;
      if (ENVK == CPL_ENV_MIXED) st_tag = env_tag[b0s + lane];
    }
  };
  auto finish_stage = [&](int64_t tt, int bi) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int64_t b0s = tt * T;
    const int vs = (int)((batch - b0s) < T ? (batch - b0s) : T);
    const int count = vs * n;
    if ((count & 1) && lane == 0) XB(bi)[count - 1] = st_tail;
    if (lane < vs) {
      MB(bi)[lane] = st_mass;
      if (ENVK == CPL_ENV_MIXED) TB(bi)[lane] = st_tag;
    }
  };

  // The two roles run separate loops with the same barrier sequence per tile, so the compiler's
  // wait-count analysis never sees a pending LDS-DMA on the compute path (no vmcnt drains there).
  if (loader) {
    // (the loader at a raised wave priority: its few DMA / gather instructions are not queued behind
    // the compute waves' VALU chains — mixed16 -1.5 %, the rest neutral; profiles/r5/loader_prio/)
    __builtin_amdgcn_s_setprio(3);
    stage(t, 0);
    finish_stage(t, 0);
    lds_barrier();
    int cur = 0;
    for (; t < ntiles; t += gridDim.x) {
      const int64_t tn = t + gridDim.x;
      if (tn < ntiles) stage(tn, cur ^ 1);
      if (ENVK == CPL_ENV_MIXED) lds_barrier();
      if (HAS_SQ) lds_barrier();
      lds_barrier();
      if (tn < ntiles) finish_stage(tn, cur ^ 1);
      lds_barrier();
      cur ^= 1;
    }
  } else {
  lds_barrier();
  int cur = 0;
  for (; t < ntiles; t += gridDim.x) {
    const int64_t b0 = t * T;
    const int valid = (int)((batch - b0) < T ? (batch - b0) : T);
    const double* X = XB(cur);
    if (ENVK == CPL_ENV_MIXED) {
      if (tid < 64) {
        const bool is_sq = tid < valid && TB(cur)[tid] == CPL_ENV_SUPERQUADRIC;
        const unsigned long long msk = __ballot(is_sq);
        if (tid < valid) {
          const int before = __popcll(msk & ((1ull << tid) - 1ull));
          if (is_sq) lists[before] = tid;
          else lists[64 + tid - before] = tid;
        }
        if (tid == 0) lists[128] = __popcll(msk);
      }
      lds_barrier();
    }
    const int n_sq = ENVK == CPL_ENV_SUPERQUADRIC ? valid : (ENVK == CPL_ENV_MIXED ? lists[128] : 0);
    const int n_gr = valid - n_sq;
    const bool wgj = K.want_g || K.want_j;

    // ---- phase 1: the Superquadric power ladders with every item that does not read their scratch
    // (contacts without Superquadric, statics, cost); phase 2: the Superquadric rows (as the tile
    // kernel; SQ items axis-major)
    if (K.ablate != 1) {
      const int r_ax = (HAS_SQ && wgj) ? 3 * N * n_sq : 0;
      const int r_gr = (ENVK != CPL_ENV_SUPERQUADRIC && wgj) ? N * n_gr : 0;
      const int r_st = wgj ? 4 * valid : 0;
      const int r_co = K.cost_seg >= 0 ? valid : 0;
      const int items1 = r_ax + r_gr + r_st + r_co;
      const int per_axis = N * n_sq;
      for (int it = tid; it < items1; it += CT) {
        int e = it;
        if (HAS_SQ && e < r_ax) {
          const int a = e / per_axis, kj = e - a * per_axis;
          const int k = kj / n_sq, j = kj - k * n_sq;
          const int r = ENVK == CPL_ENV_MIXED ? lists[j] : j;
          sq_axis_item<ENVK == CPL_ENV_MIXED>(K, X + r * n, k, a, L + r * K.LR + k * SQ_L, Gt + r * m);
          continue;
        }
        e -= r_ax;
        if (e < r_gr) {
          const int j = e % n_gr, k = e / n_gr;
          const int r = ENVK == CPL_ENV_MIXED ? lists[64 + j] : j;
          if (!HAS_SQ && K.lg_active && !K.lg_active[(b0 + r) / K.y_repeat]) continue;
          contact_item<ENVK == CPL_ENV_NONE ? CPL_ENV_NONE : CPL_ENV_GROUND>(K, X + r * n, CPL_ENV_GROUND, k,
                                                                            Gt + r * m, Jt + r * nnz);
          continue;
        }
        e -= r_gr;
        if (e < r_st) {
          const int r = e % valid, sg = e / valid;
          if (!HAS_SQ && K.lg_active && !K.lg_active[(b0 + r) / K.y_repeat]) continue;
          const double* xr = X + r * n;
          if (sg == 0) statics_values_item(K, xr, MB(cur)[r], Gt + r * m, Jt + r * nnz);
          else if (K.want_j) statics_row_item(K, xr, sg - 1, Jt + r * nnz);
          continue;
        }
        e -= r_st;
        if (!HAS_SQ && K.lg_active && !K.lg_active[(b0 + e) / K.y_repeat]) continue;
        cost_item(K, X + e * n, f_out ? f_out + b0 + e : nullptr, Dt + e * n, SC ? K.sc_df + b0 + e : nullptr);
      }
      if (HAS_SQ) {
        lds_barrier();
        if (wgj) {
          const int items2 = 3 * per_axis;
          for (int it = tid; it < items2; it += CT) {
            const int a = it / per_axis, kj = it - a * per_axis;
            const int k = kj / n_sq, j = kj - k * n_sq;
            const int r = ENVK == CPL_ENV_MIXED ? lists[j] : j;
            sq_row_item<ENVK == CPL_ENV_MIXED>(K, X + r * n, k, a, L + r * K.LR + k * SQ_L, Gt + r * m, Jt + r * nnz);
          }
        }
      }
    } else if (HAS_SQ) {
      lds_barrier();
    }
    lds_barrier();  // the tile image is complete
    if (SC) {  // the scaled problem's values (the solve engine's k_apply_scaling, in the tile image)
      for (int e = tid; e < valid * m; e += CT) {
        const int r = e / m;
        Gt[e] = Gt[e] * K.sc_dc[(b0 + r) * m + (e - r * m)];
      }
      if (K.want_j)
        for (int e = tid; e < valid * nnz; e += CT) {
          const int r = e / nnz;
          Jt[e] = Jt[e] * K.sc_dc[(b0 + r) * m + K.sc_row[e - r * nnz]];
        }
      if (K.want_grad)
        for (int e = tid; e < valid * n; e += CT) Dt[e] = Dt[e] * K.sc_df[b0 + e / n];
      lds_barrier();
    }
    if (K.want_lgrad) {
      // grad f + J^T y per (instance, column), the operation order of cpl_lagrangian_grad (bitwise
      // the same result) without the Jacobian's round trip through HBM; a 0/0 entry counts as 0
      for (int e = tid; e < valid * n; e += CT) {
        const int r = e / n, j = e - r * n;
        if (K.lg_active && !K.lg_active[(b0 + r) / K.y_repeat]) continue;  // an inactive instance
        const double* jr = Jt + r * nnz;
        const double* yb = K.ly + ((b0 + r) / K.y_repeat) * m;
        double s = Dt[r * n + j];
        for (int q = s_colp[j]; q < s_colp[j + 1]; ++q) {
          double v = jr[s_csck[q]];
          v = v == v ? v : 0.0;
          s += v * yb[s_cscr[q]];
        }
        grad_out[(b0 + r) * n + j] = s;
      }
    } else if (K.ablate != 2 && K.soa) {
      if (K.want_g) copy_out_soa<CT, NT>(g_out + b0, batch, Gt, m, valid, tid);
      if (K.want_j) copy_out_soa<CT, NT>(jac_out + b0, batch, Jt, nnz, valid, tid);
      if (K.want_grad) copy_out_soa<CT, NT>(grad_out + b0, batch, Dt, n, valid, tid);
    } else if (K.ablate != 2) {
      if (K.want_g) copy_out_ct<CT, NT>(g_out + b0 * m, Gt, valid * m, tid);
      if (K.want_j) copy_out_ct<CT, NT>(jac_out + b0 * nnz, Jt, valid * nnz, tid);
      if (K.want_grad) copy_out_ct<CT, NT>(grad_out + b0 * n, Dt, valid * n, tid);
    }
    if (K.want_norms) acc.add_tile(Gt, valid * m, tid, CT, m);
    lds_barrier();  // next x landed, tile image free
    cur ^= 1;
  }
  }  // compute role
  if (K.want_norms) partial_norms(acc, norms_ws + NORM_HDR);  // the loader contributes zeros
}


// ------------------------------------------------------------------------------------------
// v4: table-driven records (Ground / no environment; IFOPT CSR values, instance-major).
//   The pipelined kernel's loader wave (double-buffered LDS DMA of the next tile's x) with another
//   compute side.  Every g / jac entry of these records is, up to its sign, one of: an element of x,
//   a constant (0, 1), or a value of a short per-contact / per-instance prologue (p - c, the friction
//   cone's values and row-1 derivatives, the Ground residuals, the statics sums).  So:
//     * a per-block opcode table (built once per launch in LDS) maps record position -> (source
//       area, offset, sign);
//     * per tile, one thread per (instance, contact) and per instance computes the prologue values
//       into an LDS scratch — the same operations in the same order as the work items of the other
//       kernels (bitwise the same values);
//     * the g and jac records are then a branch-free gather: lanes along the records, two entries per
//       lane, 16-byte non-temporal stores straight to HBM.
//   No output image lives in LDS, so large records (16 contacts: 6 KiB of outputs per instance) keep
//   large tiles.  Optional instance list idx [count]: tile position j evaluates instance idx[j] and
//   writes its records in place (the Ground half of a mixed batch); d_count: the list's length on the
//   device (the grid is sized for `batch`, tiles past the count idle).  Records must have an even
//   number of entries (m always; nnz = 6 + 42N with a surface, 6 + 27N without: even N).
// ------------------------------------------------------------------------------------------
// scratch per instance: [statics g (6) | CoM pairs (6) | per contact (vector order) ENT_PC values]
constexpr int ENT_PC = 15;  // d = p - c (3), cone row 1 (6), cone g (2), env g (1), normal g (3)
enum { EPC_D = 0, EPC_ROW1 = 3, EPC_CONEG = 9, EPC_ENVG = 11, EPC_NORMG = 12 };
constexpr unsigned OP_X = 0u << 28, OP_S = 1u << 28, OP_C = 2u << 28, OP_NEG = 1u << 31;

// the opcode of g entry q / jac entry q of the record (map order -> vector index via s_ct)
template <int ENVK>
__device__ __forceinline__ unsigned entry_op_g(int q, int S0) {
  constexpr int CR = ENVK == CPL_ENV_NONE ? 2 : 6;
  if (q < 6) return OP_S | (unsigned)q;
  const int u = q - 6, k = u / CR, w = u - k * CR;
  const unsigned ci = (unsigned)(S0 + ENT_PC * s_ct.map_order[k]);
  if (ENVK == CPL_ENV_NONE) return OP_S | (ci + EPC_CONEG + w);
  if (w == 0) return OP_S | (ci + EPC_ENVG);
  if (w < 4) return OP_S | (ci + EPC_NORMG + (w - 1));
  return OP_S | (ci + EPC_CONEG + (w - 4));
}
template <int ENVK>
__device__ __forceinline__ unsigned entry_op_j(int q, int N, int S0) {
  constexpr int CJ = ENVK == CPL_ENV_NONE ? 12 : 27;
  const int RL = 2 + 4 * N, JC = 3 * N + 3 * RL;
  if (q < 3 * N) return OP_C | 1u;  // the force-balance rows' I3 blocks (CentroidalStatics.cpp:93-95)
  if (q < JC) {                     // torque row 3 + qq (CentroidalStatics.cpp:75-137)
    int w = q - 3 * N;
    const int qq = w >= 2 * RL ? 2 : (w >= RL ? 1 : 0);
    w -= qq * RL;
    if (w < 2) return OP_S | (unsigned)(6 + 2 * qq + w);  // the CoM pair
    const int e1 = qq == 2 ? 1 : 2, e2 = qq == 0 ? 1 : 0;
    const bool s1neg = qq != 1, s2neg = qq == 1;  // s1 = (qq == 1 ? 1 : -1), s2 = (qq == 1 ? -1 : 1)
    const int i = (w - 2) >> 2, c = (w - 2) & 3;
    const unsigned ci = (unsigned)(S0 + ENT_PC * i);
    switch (c) {
      case 0: return OP_S | (ci + EPC_D + e1) | (s1neg ? OP_NEG : 0u);   // s1 (p - c)[e1]
      case 1: return OP_S | (ci + EPC_D + e2) | (s2neg ? OP_NEG : 0u);   // s2 (p - c)[e2]
      case 2: return OP_X | (unsigned)(3 + 9 * i + e1) | (s1neg ? 0u : OP_NEG);  // -s1 F[e1]
      default: return OP_X | (unsigned)(3 + 9 * i + e2) | (s2neg ? 0u : OP_NEG);  // -s2 F[e2]
    }
  }
  const int u = q - JC, k = u / CJ;
  int w = u - k * CJ;
  const int i = s_ct.map_order[k];
  if (ENVK != CPL_ENV_NONE) {
    // src/Ground.cpp:30-50: gradient (0, 0, 1), zero normal Jacobian; EnvironmentNormal's n_r block 1
    if (w < 3) return OP_C | (w == 2 ? 1u : 0u);
    if (w < 15) return OP_C | (((w - 3) & 3) == 3 ? 1u : 0u);
    w -= 15;
  }
  if (w < 3) return OP_X | (unsigned)(9 + 9 * i + w) | OP_NEG;  // cone row 0: -n (FrictionCone.cpp:79-81)
  if (w < 6) return OP_X | (unsigned)(3 + 9 * i + (w - 3)) | OP_NEG;  // -F (:91-93)
  return OP_S | (unsigned)(S0 + ENT_PC * i + EPC_ROW1 + (w - 6));   // row 1 (:82-101)
}

// loader wave: one row of `count` doubles from a 16-byte aligned source into LDS (dst 16-byte aligned):
// 16-byte DMA granules for the pairs (1 KiB per instruction), the odd last double as two dwords
__device__ __forceinline__ void dma_row16(double* dst, const double* src, int count, int lane) {
  const int pairs = count >> 1;
  for (int q = 0; q < pairs; q += 64)
    if (q + lane < pairs)
      __builtin_amdgcn_global_load_lds((glb_void_t*)(src + 2 * (q + lane)), (lds_void_t*)(dst + 2 * q), 16, 0, 0);
  if (count & 1) {
    const unsigned* s4 = reinterpret_cast<const unsigned*>(src + count - 1);
    if (lane < 2) __builtin_amdgcn_global_load_lds((glb_void_t*)(s4 + lane), (lds_void_t*)(dst + count - 1), 4, 0, 0);
  }
}

// loader wave: one row of `count` doubles (8-byte aligned source) into LDS with 4-byte DMA granules
__device__ __forceinline__ void dma_row4(double* dst, const double* src, int count, int lane) {
  const unsigned* s4 = reinterpret_cast<const unsigned*>(src);
  unsigned* d4 = reinterpret_cast<unsigned*>(dst);
  const int words = 2 * count;
  for (int q = 0; q < words; q += 64)
    if (q + lane < words) __builtin_amdgcn_global_load_lds((glb_void_t*)(s4 + q + lane), (lds_void_t*)(d4 + q), 4, 0, 0);
}

// the value of opcode op for tile row r: x row, scratch row or constant, sign applied as a sign-bit
// flip (bitwise the unary minus of the other kernels)
__device__ __forceinline__ double entry_value(unsigned op, const double* __restrict__ Xr, const double* __restrict__ Sr,
                                              const double* __restrict__ C) {
  const unsigned t = (op >> 28) & 3u;
  const double* base = t == 0 ? Xr : (t == 1 ? Sr : C);
  const double v = base[op & 0xffffffu];
  long long bits = __double_as_longlong(v);
  bits ^= (long long)(op & OP_NEG) << 32;
  return __longlong_as_double(bits);
}

template <int ENVK, bool NT>
__global__ __launch_bounds__(256) void cpl_eval_entry_kernel(const KParams K, int64_t batch,
                                                             const double* __restrict__ x,
                                                             const double* __restrict__ mass,
                                                             const int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ d_count,
                                                             double* __restrict__ g_out,
                                                             double* __restrict__ jac_out,
                                                             double* __restrict__ f_out,
                                                             double* __restrict__ grad_out,
                                                             double* __restrict__ norms_ws) {
  constexpr int NCW = 3, CT = 64 * NCW;  // compute waves + one loader wave
  extern __shared__ __align__(16) double smem[];
  load_ctab(K);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const bool loader = (tid >> 6) == NCW;
  const int T = K.T;
  const int n = K.n, m = K.m, nnz = K.nnz, N = K.N;
  const int S = 12 + ENT_PC * N;  // scratch doubles per instance
  auto XB = [&](int bi) { return smem + (bi ? K.offX1 : 0); };
  auto MB = [&](int bi) { return smem + K.offMB + (bi ? T : 0); };
  auto RB = [&](int bi) { return reinterpret_cast<long long*>(smem + K.offRB) + (bi ? T : 0); };
  double* SC = smem + K.offCS;                                  // [T][S]
  double* CN = smem + K.offST;                                  // constants 0, 1
  unsigned* OPG = reinterpret_cast<unsigned*>(smem + K.offST + 2);  // [m] then [nnz] opcodes
  unsigned* OPJ = OPG + m;
  __syncthreads();  // (s_ct)
  if (tid == 0) { CN[0] = 0.0; CN[1] = 1.0; }
  for (int q = tid; q < m; q += blockDim.x) OPG[q] = entry_op_g<ENVK>(q, 12);
  for (int q = tid; q < nnz; q += blockDim.x) OPJ[q] = entry_op_j<ENVK>(q, N, 12);
  const int64_t count = d_count ? (int64_t)*d_count : batch;
  const int64_t ntiles = (count + T - 1) / T;
  const bool contiguous = idx == nullptr && K.x_aligned16;
  // LDS row stride of x: n for contiguous tiles (one DMA stream), even for lists (every row slot 16-byte
  // aligned, so the rows whose source is aligned too take 16-byte granules)
  const int xs = contiguous ? n : (n + 1) & ~1;
  double mass_def = K.mass_default;  // a value (see cpl_eval_pipe_kernel)
  asm volatile("" : "+v"(mass_def));
  NormAcc acc;
  // the grid that walks the tiles: every workgroup, or (the kind split's Ground half beside a non-empty
  // Superquadric list, whose tiles the other slots of each CU take) the first grid_cap; the others
  // only write zero residual partials.  d_count[1] is the Superquadric list's length (the split's
  // counts), the same value in every workgroup.
  const int64_t G = (K.grid_cap > 0 && d_count && d_count[1] > 0 && (int64_t)gridDim.x > K.grid_cap)
                        ? (int64_t)K.grid_cap
                        : (int64_t)gridDim.x;
  int64_t t = (int64_t)blockIdx.x < G ? (int64_t)blockIdx.x : ntiles;
  __syncthreads();  // (the table)

  if (loader) {
    // (the loader at a raised wave priority: its few DMA / gather instructions are not queued behind
    // the compute waves' VALU chains — mixed16 -1.5 %, the rest neutral; profiles/r5/loader_prio/)
    __builtin_amdgcn_s_setprio(3);
    double st_mass = 0.0, st_tail = 0.0;
    long long st_b = 0;
    // (lists) the instances and masses of the tile staged next, loaded one tile ahead: the rows' DMA
    // then issues at once instead of after two dependent round trips (the list entry, then its mass)
    long long pf_b = 0;
    double pf_mass = 0.0;
    auto ids = [&](int64_t tt, long long& bo, double& mo) {
      const int64_t j0 = tt * T;
      const int vs = (int)((count - j0) < T ? (count - j0) : T);
      if (lane < vs) {
        const int b = idx ? idx[j0 + lane] : (int)(j0 + lane);
        bo = b;
        mo = mass ? mass[b] : mass_def;
      }
    };
    auto stage = [&](int64_t tt, int bi) {
      const int64_t j0 = tt * T;
      const int vs = (int)((count - j0) < T ? (count - j0) : T);
      if (contiguous) {
        ids(tt, st_b, st_mass);
        const int cnt = vs * n;
        dma_tile(XB(bi), x + j0 * n, cnt, lane);
        if ((cnt & 1) && lane == 0) st_tail = x[j0 * n + cnt - 1];
      } else {
        st_b = pf_b;
        st_mass = pf_mass;
        const int b = (int)st_b;
        // rows whose source and LDS slot are both 16-byte aligned take 16-byte granules (every row when n
        // is even; the even instances' rows when n is odd), the others 4-byte ones
        for (int r = 0; r < vs; ++r) {
          const int64_t br = (int64_t)__builtin_amdgcn_readlane(b, r);
          double* d = XB(bi) + r * xs;
          const double* src = x + br * n;
          if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) dma_row16(d, src, n, lane);
          else dma_row4(d, src, n, lane);
        }
        if (tt + G < ntiles) ids(tt + G, pf_b, pf_mass);
      }
    };
    auto finish_stage = [&](int64_t tt, int bi) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int64_t j0 = tt * T;
      const int vs = (int)((count - j0) < T ? (count - j0) : T);
      const int cnt = vs * n;
      if (contiguous && (cnt & 1) && lane == 0) XB(bi)[cnt - 1] = st_tail;
      if (lane < vs) {
        MB(bi)[lane] = st_mass;
        RB(bi)[lane] = st_b;
      }
    };
    if (t < ntiles) {
      if (!contiguous) ids(t, pf_b, pf_mass);
      stage(t, 0);
      finish_stage(t, 0);
    }
    lds_barrier();
    int cur = 0;
    for (; t < ntiles; t += G) {
      const int64_t tn = t + G;
      if (tn < ntiles) stage(tn, cur ^ 1);
      lds_barrier();  // (the compute waves' prologue)
      if (tn < ntiles) finish_stage(tn, cur ^ 1);
      lds_barrier();  // (the tile's entries)
      cur ^= 1;
    }
  } else {
    if (K.cw_prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (K.cw_prio == 2) __builtin_amdgcn_s_setprio(2);
    acc.init(tid, CT, m);
    lds_barrier();
    int cur = 0;
    const double mu = K.mu;
    for (; t < ntiles; t += G) {
      const int64_t j0 = t * T;
      const int valid = (int)((count - j0) < T ? (count - j0) : T);
      const double* X = XB(cur);
      const double* Mb = MB(cur);
      const long long* Rb = RB(cur);
      // ---- prologue: per (instance, contact) p - c, the cone's values and row-1 derivatives, the
      // Ground residuals; per instance the statics values and the torque rows' CoM pairs; the cost
      const int pc = valid * N;
      const int items = pc + valid + (K.want_f ? valid : 0);
      for (int it = tid; it < items; it += CT) {
        if (it < pc) {
          const int r = it / N, i = it - r * N;  // (vector order)
          const double* xr = X + r * xs;
          const double* q = xr + 3 + 9 * i;
          const double F0 = q[0], F1 = q[1], F2 = q[2], p0 = q[3], p1 = q[4], p2 = q[5];
          const double n0 = q[6], n1 = q[7], n2 = q[8];
          double* cs = SC + r * S + 12 + ENT_PC * i;
          cs[EPC_D + 0] = p0 - xr[0];  // statics_rows_coop's (p[e] - xr[e])
          cs[EPC_D + 1] = p1 - xr[1];
          cs[EPC_D + 2] = p2 - xr[2];
          // src/Constraints/FrictionCone.cpp:30-45 (values), :71-101 (contact_item's expressions)
          const double t1 = dot3(F0, F1, F2, n0, n1, n2);
          const double nF = dot3(n0, n1, n2, F0, F1, F2);
          const double u0 = F0 - nF * n0, u1 = F1 - nF * n1, u2 = F2 - nF * n2;
          cs[EPC_CONEG + 0] = -t1 + s_ct.F_thr[i];
          cs[EPC_CONEG + 1] = sqrt((u0 * u0 + u1 * u1) + u2 * u2) - mu * t1;
          const double t2 = F0 - n0 * t1;
          const double t3 = F1 - n1 * t1;
          const double t4 = F2 - n2 * t1;
          const double t5 = F0 * n0;
          const double t6 = F1 * n1;
          const double t7 = F2 * n2;
          const double s = sqrt(t2 * t2 + t3 * t3 + t4 * t4);
          double* jk = cs + EPC_ROW1 - 6;
          jk[6] = (t2 * (n0 * n0 - 1.0) * 2.0 + n0 * n1 * t3 * 2.0 + n0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n0;
          jk[7] = (t3 * (n1 * n1 - 1.0) * 2.0 + n0 * n1 * t2 * 2.0 + n1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n1;
          jk[8] = (t4 * (n2 * n2 - 1.0) * 2.0 + n0 * n2 * t2 * 2.0 + n1 * n2 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * n2;
          jk[9] = (t2 * (t6 + t7 + t5 * 2.0) * 2.0 + F0 * n1 * t3 * 2.0 + F0 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F0;
          jk[10] = (t3 * (t5 + t7 + t6 * 2.0) * 2.0 + F1 * n0 * t2 * 2.0 + F1 * n2 * t4 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F1;
          jk[11] = (t4 * (t5 + t6 + t7 * 2.0) * 2.0 + F2 * n0 * t2 * 2.0 + F2 * n1 * t3 * 2.0) * 1.0 / s * (-1.0 / 2.0) - mu * F2;
          if (ENVK != CPL_ENV_NONE) {  // src/Ground.cpp:23-50 (contact_item's gv)
            cs[EPC_ENVG] = p2 - K.ground_z;
            cs[EPC_NORMG + 0] = n0 - 0.0;
            cs[EPC_NORMG + 1] = n1 - 0.0;
            cs[EPC_NORMG + 2] = n2 - 1.0;
          }
        } else if (it < pc + valid) {
          // CentroidalStatics::GetValues (src/Constraints/CentroidalStatics.cpp:37-61) and the torque
          // rows' CoM pairs (:119-136), both in map order — statics_values_item's arithmetic
          const int r = it - pc;
          const double* xr = X + r * xs;
          double* st = SC + r * S;
          const double c0 = xr[0], c1 = xr[1], c2 = xr[2];
          double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, v5 = 0.0;
          double a[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
          for (int k = 0; k < N; ++k) {
            const double* q = xr + 3 + 9 * s_ct.map_order[k];
            const double F0 = q[0], F1 = q[1], F2 = q[2];
            const double d0 = q[3] - c0, d1 = q[4] - c1, d2 = q[5] - c2;
            v0 += F0; v1 += F1; v2 += F2;
            v3 += d1 * F2 - d2 * F1;
            v4 += d2 * F0 - d0 * F2;
            v5 += d0 * F1 - d1 * F0;
            a[0] -= -(-1.0) * F2; a[1] -= -(1.0) * F1;
            a[2] -= -(1.0) * F2;  a[3] -= -(-1.0) * F0;
            a[4] -= -(-1.0) * F1; a[5] -= -(1.0) * F0;
          }
          const double m_i = Mb[r];
          v0 -= K.wrench[0]; v1 -= K.wrench[1]; v2 -= K.wrench[2];
          v3 -= K.wrench[3]; v4 -= K.wrench[4]; v5 -= K.wrench[5];
          v0 += m_i * K.gravity[0]; v1 += m_i * K.gravity[1]; v2 += m_i * K.gravity[2];
          st[0] = v0; st[1] = v1; st[2] = v2; st[3] = v3; st[4] = v4; st[5] = v5;
#pragma unroll
          for (int u = 0; u < 6; ++u) st[6 + u] = a[u];
        } else {
          const int r = it - pc - valid;
          f_out[Rb[r]] = cost_value(K, X + r * xs);
        }
      }
      lds_barrier();
      // ---- g and the Jacobian values: a gather by the opcode tables, two entries per lane, lanes
      // along the tile's records (consecutive lanes, consecutive 16-byte pieces of one record)
      auto gather = [&](const unsigned* __restrict__ op, int rec, double* __restrict__ out, bool norms) {
        const int h2 = rec >> 1;
        const int total = valid * h2;
        int r = tid / h2, q2 = tid - r * h2;
        for (int e = tid; e < total; e += CT) {
          const uint2 o = reinterpret_cast<const uint2*>(op)[q2];
          const double* Xr = X + r * xs;
          const double* Sr = SC + r * S;
          const double v0 = entry_value(o.x, Xr, Sr, CN), v1 = entry_value(o.y, Xr, Sr, CN);
          if (norms) {
            const double a0 = row_violation(v0, s_ct.cone[2 * q2]), a1 = row_violation(v1, s_ct.cone[2 * q2 + 1]);
            acc.vmax = a0 > acc.vmax ? a0 : acc.vmax;
            acc.vsum += a0 * a0;
            acc.vmax = a1 > acc.vmax ? a1 : acc.vmax;
            acc.vsum += a1 * a1;
          }
          double2* d = reinterpret_cast<double2*>(out + Rb[r] * rec) + q2;
          if (NT) {
            __builtin_nontemporal_store(v0, &d->x);
            __builtin_nontemporal_store(v1, &d->y);
          } else {
            *d = make_double2(v0, v1);
          }
          q2 += CT;
          while (q2 >= h2) { q2 -= h2; ++r; }
        }
      };
      if (K.want_g) gather(OPG, m, g_out, K.want_norms != 0);
      if (K.want_j) gather(OPJ, nnz, jac_out, false);
      // ---- the cost gradient (MinimizeCentroidalVariables.cpp:151-192; cost_item's entries)
      if (K.want_grad) {
        const int total = valid * n;
        int r = tid / n, q = tid - r * n;
        for (int e = tid; e < total; e += CT) {
          const double* xr = X + r * xs;
          double v;
          if (q < 3) {
            v = K.W_com * (xr[q] - K.com_ref[q]);
          } else {
            const int i = (q - 3) / 9, w = (q - 3) - 9 * i;
            v = w < 3 ? K.W_F[i] * (xr[q] - K.F_ref[i][w]) : w < 6 ? K.W_p[i] * (xr[q] - K.p_ref[i][w - 3]) : 0.0;
          }
          grad_out[Rb[r] * n + q] = v;
          q += CT;
          while (q >= n) { q -= n; ++r; }
        }
      }
      lds_barrier();  // next x landed, scratch free
      cur ^= 1;
    }
  }
  if (K.want_norms) partial_norms(acc, norms_ws + NORM_HDR);  // the loader contributes zeros
}


// ------------------------------------------------------------------------------------------
// Exact Hessian of the Lagrangian f + y^T g over the free variables (Ground / no environment:
// the environment and normal rows are linear there, so only the cost, the torque rows of
// CentroidalStatics and the two FrictionCone rows carry curvature).  For an entry (u, v) of the
// variables x = [c | per contact (names order) F, p, n]:
//   cost:   W_com, W_F,i, W_p,i on the diagonal (src/MinimizeCentroidalVariables.cpp:124-148);
//   torque: rows 3+k = sum_i ((p_i - c) x F_i)_k  ->  d2/dp_a dF_b = E_ab, d2/dc_a dF_b = -E_ab,
//           E_ab = sum_k y_{3+k} eps_kab (src/Constraints/CentroidalStatics.cpp:37-61);
//   cone 0: -F.n                ->  d2/dF_a dn_b = -delta_ab
//   cone 1: |t| - mu s, s = F.n, t = F - s n (src/Constraints/FrictionCone.cpp:30-45):
//           Hess |t| = J^T (I - uu^T) J / |t| + sum_j u_j Hess t_j  (u = t / |t|), with
//           J_F = I - n n^T, J_n = -(n F^T + s I), d2 t_j/dF_a dn_b = -(delta_ab n_j + n_a delta_jb),
//           d2 t_j/dn_a dn_b = -(F_a delta_jb + F_b delta_ja); at |t| = 0 the |t| terms count as 0
//           (the reference's Jacobian is 0/0 there; the product path takes NaN as 0).
// One workgroup per instance: the same-contact (F, n) x (F, n) entries — the only ones with the
// cone's square root and divisions — are computed once per contact (36 per contact) into LDS, then
// the [nf, nf] output is written row-major with coalesced stores, every other entry computed in
// place (the cheap cost / torque terms).  Each entry is the same expression as a thread per entry
// (bitwise the same values); this layout keeps the cone's transcendental path off every wave.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double hessian_entry(const KParams& K, const double* __restrict__ xb,
                                                const double* __restrict__ yb, const int* s_pos, int uu, int vv) {
  // decode: kind 0 CoM, 1 F, 2 p, 3 n; contact i; axis a
  auto decode = [](int u, int& kind, int& i, int& a) {
    if (u < 3) { kind = 0; i = -1; a = u; return; }
    const int r = u - 3;
    i = r / 9;
    const int t = r - 9 * i;
    kind = 1 + t / 3;
    a = t - 3 * (t / 3);
  };
  int ku, iu, au, kv, iv, av;
  decode(uu, ku, iu, au);
  decode(vv, kv, iv, av);
  double h = 0.0;
  // cost (diagonal)
  if (uu == vv) h += ku == 0 ? K.W_com : (ku == 1 ? K.W_F[iu] : (ku == 2 ? K.W_p[iu] : 0.0));
  // torque rows: E_ab = sum_k y_{3+k} eps_kab
  auto E = [&](int a, int c) {
    if (a == c) return 0.0;
    const int k = 3 - a - c;                        // the third index
    const double sgn = ((a + 1) % 3 == c) ? 1.0 : -1.0;  // eps_{k a c} for (a, c) in cyclic order
    return sgn * yb[3 + k];
  };
  if (ku == 2 && kv == 1 && iu == iv) h += E(au, av);          // d2/dp_a dF_b
  else if (ku == 1 && kv == 2 && iu == iv) h += E(av, au);     // d2/dF_b dp_a
  else if (ku == 0 && kv == 1) h -= E(au, av);                 // d2/dc_a dF_b
  else if (ku == 1 && kv == 0) h -= E(av, au);
  // friction cone of the contact (F and n entries of one contact)
  if (iu == iv && iu >= 0 && (ku == 1 || ku == 3) && (kv == 1 || kv == 3)) {
    const double* q = xb + 3 + 9 * iu;
    const double F[3] = {q[0], q[1], q[2]};
    const double nn[3] = {q[6], q[7], q[8]};
    const int r0 = 6 + K.contact_rows * s_pos[iu] + (K.contact_rows - 2);
    const double y0 = yb[r0], y1 = yb[r0 + 1];
    const double sdot = (F[0] * nn[0] + F[1] * nn[1]) + F[2] * nn[2];
    const double t[3] = {F[0] - sdot * nn[0], F[1] - sdot * nn[1], F[2] - sdot * nn[2]};
    const double rr = sqrt((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
    const bool fn = (ku == 1 && kv == 3) || (ku == 3 && kv == 1);
    const int aF = ku == 1 ? au : av, an = ku == 3 ? au : av;  // (for the mixed block)
    if (fn && aF == an) h -= y0 + K.mu * y1;  // -F.n and -mu s: d2/dF_a dn_a = -1
    if (rr > 0.0 && rr < INFINITY && y1 != 0.0) {
      const double u[3] = {t[0] / rr, t[1] / rr, t[2] / rr};
      // columns of J for the two variables
      auto col = [&](int kind, int a, double* c) {
        for (int j = 0; j < 3; ++j)
          c[j] = kind == 1 ? ((j == a ? 1.0 : 0.0) - nn[j] * nn[a]) : -(nn[j] * F[a] + (j == a ? sdot : 0.0));
      };
      double cu[3], cv[3];
      col(ku, au, cu);
      col(kv, av, cv);
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
      h += y1 * ((jj - pu * pv) / rr + second);
    }
  }
  return h;
}

__global__ __launch_bounds__(256) void cpl_lagrangian_hessian_kernel(const KParams K, int64_t batch, int nf,
                                                                     const double* __restrict__ x,
                                                                     const double* __restrict__ y,
                                                                     const uint8_t* __restrict__ active,
                                                                     const int32_t* __restrict__ free_idx,
                                                                     double* __restrict__ H) {
  __shared__ int s_pos[CPL_MAX_CONTACTS];          // block position (map order) of contact i
  __shared__ double s_cone[CPL_MAX_CONTACTS * 36];  // (F, n) x (F, n) entries of contact i
  __shared__ int s_col[3 + 9 * CPL_MAX_CONTACTS];   // free index -> column of x
  const int64_t b = blockIdx.x;
  if (b >= batch || (active && !active[b])) return;  // (uniform per workgroup)
  const int tid = threadIdx.x;
  if (tid < K.N) s_pos[K.map_order[tid]] = tid;
  for (int k = tid; k < nf; k += blockDim.x) s_col[k] = free_idx[k];
  __syncthreads();
  const double* xb = x + b * (int64_t)K.n;
  const double* yb = y + b * (int64_t)K.m;
  // (F, n) x (F, n) blocks: local index 0-2 F_a (column 3 + 9i + a), 3-5 n_a (column 9 + 9i + a)
  for (int t = tid; t < 36 * K.N; t += blockDim.x) {
    const int i = t / 36, r = t - 36 * i, u6 = r / 6, v6 = r - 6 * (r / 6);
    const int uu = 3 + 9 * i + (u6 < 3 ? u6 : 3 + u6), vv = 3 + 9 * i + (v6 < 3 ? v6 : 3 + v6);
    s_cone[t] = hessian_entry(K, xb, yb, s_pos, uu, vv);
  }
  __syncthreads();
  double* Hb = H + b * (int64_t)nf * nf;
  // row-major walk of the output: (row, col) of entry tid + 256 s advanced incrementally
  const int step_r = blockDim.x / nf, step_c = blockDim.x - step_r * nf;
  int row = tid / nf, col = tid - row * nf;
  for (int e = tid; e < nf * nf; e += blockDim.x) {
    const int uu = s_col[row], vv = s_col[col];
    const int ru = uu - 3, rv = vv - 3;
    const int iu = ru / 9, iv = rv / 9, tu = ru - 9 * iu, tv = rv - 9 * iv;
    double h;
    if (uu >= 3 && vv >= 3 && iu == iv && (tu < 3 || tu >= 6) && (tv < 3 || tv >= 6))
      h = s_cone[36 * iu + 6 * (tu < 3 ? tu : tu - 3) + (tv < 3 ? tv : tv - 3)];
    else
      h = hessian_entry(K, xb, yb, s_pos, uu, vv);
    Hb[e] = h;
    row += step_r;
    col += step_c;
    if (col >= nf) { col -= nf; ++row; }
  }
}

// ------------------------------------------------------------------------------------------
// Residual norms of g against its bounds (per shard), deterministic two-stage reduction
// ------------------------------------------------------------------------------------------
constexpr int RN_BLOCK = 256;
constexpr int RN_GRID = 1024;

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

// Finish of the per-workgroup partial pairs: one workgroup of RF_BLOCK threads; each thread keeps
// RF_ILP independent accumulators fed by 16-byte loads of whole (max, sum) pairs, so a tile kernel's
// tens of thousands of partials cost a few memory round trips, not one per partial.  The combination
// order depends only on nparts (deterministic).
constexpr int RF_ILP = 8;

// With `chunk` (level 1 of a two-level finish): workgroup b reduces the pairs [b chunk, (b + 1) chunk)
// into out[2b], out[2b + 1].
template <int RF_BLOCK>
__global__ __launch_bounds__(RF_BLOCK) void cpl_residual_final(int nparts, const double* __restrict__ part,
                                                               double* __restrict__ out, int chunk = 0) {
  __shared__ double smax[RF_BLOCK / 64], ssum[RF_BLOCK / 64];
  if (chunk > 0) {
    const int first = (int)blockIdx.x * chunk;
    part += 2 * (size_t)first;
    out += 2 * (size_t)blockIdx.x;
    nparts = nparts - first < chunk ? nparts - first : chunk;
  }
  const double2* p2 = reinterpret_cast<const double2*>(part);
  const int tid = threadIdx.x;
  double am[RF_ILP], as[RF_ILP];
#pragma unroll
  for (int u = 0; u < RF_ILP; ++u) { am[u] = 0.0; as[u] = 0.0; }
  int e = tid;
  for (; e + (RF_ILP - 1) * RF_BLOCK < nparts; e += RF_ILP * RF_BLOCK) {
    double2 v[RF_ILP];
#pragma unroll
    for (int u = 0; u < RF_ILP; ++u) v[u] = p2[e + u * RF_BLOCK];
#pragma unroll
    for (int u = 0; u < RF_ILP; ++u) {
      am[u] = v[u].x > am[u] ? v[u].x : am[u];
      as[u] += v[u].y;
    }
  }
  for (; e < nparts; e += RF_BLOCK) {
    const double2 v = p2[e];
    am[0] = v.x > am[0] ? v.x : am[0];
    as[0] += v.y;
  }
  double vmax = 0.0, vsum = 0.0;
#pragma unroll
  for (int u = 0; u < RF_ILP; ++u) { vmax = am[u] > vmax ? am[u] : vmax; vsum += as[u]; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double om = __shfl_xor(vmax, o);
    const double os = __shfl_xor(vsum, o);
    vmax = om > vmax ? om : vmax;
    vsum += os;
  }
  if ((tid & 63) == 0) { smax[tid >> 6] = vmax; ssum[tid >> 6] = vsum; }
  __syncthreads();
  if (tid == 0) {
    double bm = 0.0, bs = 0.0;
    for (int w = 0; w < RF_BLOCK / 64; ++w) { bm = smax[w] > bm ? smax[w] : bm; bs += ssum[w]; }
    out[0] = bm;
    out[1] = bs;
  }
}

// ---- mixed batches split by environment kind: a stable partition of the instance indices by tag
// (every launch recomputes it: the tags may change between launches under the same pointer), the
// Ground instances to the entry kernel, the Superquadric ones to the Superquadric tile kernel, each
// writing its records in place.  Deterministic: the lists keep instance order, so the tiles (and the
// norm partials' summation order) are a function of the tags alone.
constexpr int PART_BLOCK = 1024;
__global__ __launch_bounds__(PART_BLOCK) void k_kind_count(int64_t batch, const uint8_t* __restrict__ tag,
                                                           int32_t* __restrict__ blk_sq) {
  __shared__ int wsum[PART_BLOCK / 64];
  const int64_t b = (int64_t)blockIdx.x * PART_BLOCK + threadIdx.x;
  const bool sq = b < batch && tag[b] == CPL_ENV_SUPERQUADRIC;
  const int c = __popcll(__ballot(sq));
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < PART_BLOCK / 64; ++w) t += wsum[w];
    blk_sq[blockIdx.x] = t;
  }
}
// The lists written in place of a scan kernel: each block sums the Superquadric counts of the blocks
// before it (its exclusive offset, an integer sum: any order gives the same value), and the last block
// sums them all for the two list lengths (counts[0] Ground, counts[1] Superquadric) — one launch and
// one single-workgroup Hillis-Steele pass fewer than a separate scan.
__global__ __launch_bounds__(PART_BLOCK) void k_kind_write(int64_t batch, int nblk, const uint8_t* __restrict__ tag,
                                                           const int32_t* __restrict__ blk_sq,
                                                           int32_t* __restrict__ idx_gr, int32_t* __restrict__ idx_sq,
                                                           int32_t* __restrict__ counts) {
  __shared__ int wsum[PART_BLOCK / 64];
  __shared__ long long wpre[PART_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool last = (int)blockIdx.x == nblk - 1;
  const int upto = last ? nblk : (int)blockIdx.x;  // the last block also sums its own count
  long long pre = 0;
  for (int i = (int)threadIdx.x; i < upto; i += PART_BLOCK)
    if (i < (int)blockIdx.x || last) pre += blk_sq[i];
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
  const int64_t b = (int64_t)blockIdx.x * PART_BLOCK + threadIdx.x;
  const bool in = b < batch;
  const bool sq = in && tag[b] == CPL_ENV_SUPERQUADRIC;
  const unsigned long long msk = __ballot(sq);
  if (lane == 0) {
    wsum[wave] = __popcll(msk);
    wpre[wave] = pre;
  }
  __syncthreads();
  long long tot = 0;  // (the last block: every block's count, its own included)
  for (int w = 0; w < PART_BLOCK / 64; ++w) tot += wpre[w];
  const int64_t off_sq = last ? tot - (blk_sq[blockIdx.x]) : tot;
  if (last && threadIdx.x == 0) {
    counts[1] = (int32_t)tot;
    counts[0] = (int32_t)(batch - tot);
  }
  int before = 0;  // Superquadric instances of the block before this wave
  for (int w = 0; w < wave; ++w) before += wsum[w];
  const int sq_rank = before + __popcll(msk & ((1ull << lane) - 1ull));
  const int local = (int)threadIdx.x;
  const int64_t off_gr = (int64_t)blockIdx.x * PART_BLOCK - off_sq;
  if (sq) idx_sq[off_sq + sq_rank] = (int32_t)b;
  else if (in) idx_gr[off_gr + (local - sq_rank)] = (int32_t)b;
}

// the kind lists' workspace, per (device, stream), grown on demand and never freed (a captured graph
// keeps its pointers; see NormWs): [idx_gr | idx_sq | blk_sq | blk_off | counts]
struct KindWs {
  int32_t* ptr = nullptr;
  int64_t cap = 0;
  std::vector<int32_t*> old;
};
static int32_t hip_fail(hipError_t e, const char* what);
static std::mutex g_kind_ws_mutex;
static std::map<std::pair<int, hipStream_t>, KindWs> g_kind_ws;

struct KindLists {
  int32_t *idx_gr, *idx_sq, *blk_sq, *blk_off, *counts;
};
static int32_t kind_workspace(hipStream_t stream, int64_t batch, KindLists* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_kind_ws_mutex);
  KindWs& w = g_kind_ws[{dev, stream}];
  if (w.cap < batch) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(CPL_ERR_RUNTIME,
                  "mixed batch: the per-stream kind-list workspace must grow, which a stream capture forbids; "
                  "launch the largest batch once on this stream before capturing");
    const int64_t nblk = (batch + PART_BLOCK - 1) / PART_BLOCK;
    int32_t* p = nullptr;
    e = hipMalloc(&p, sizeof(int32_t) * (size_t)(2 * batch + 2 * nblk + 4));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc kind lists");
    if (w.ptr) w.old.push_back(w.ptr);
    w.ptr = p;
    w.cap = batch;
  }
  const int64_t cap = w.cap, nblk = (cap + PART_BLOCK - 1) / PART_BLOCK;
  out->idx_gr = w.ptr;
  out->idx_sq = w.ptr + cap;
  out->blk_sq = w.ptr + 2 * cap;
  out->blk_off = out->blk_sq + nblk;
  out->counts = out->blk_off + nblk;
  return CPL_OK;
}

// `part` must have room for nparts + nparts / RF_CHUNK + 1 pairs (the norm workspaces hold 2 cap)
constexpr int RF_CHUNK = 8192;
// a side stream (and a fork / join event pair) per (device, stream) for the mixed split's two halves,
// created on first use and kept (a captured graph may hold them)
struct SideStream {
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
static std::mutex g_side_mutex;
static std::map<std::pair<int, hipStream_t>, SideStream> g_side;
static int32_t side_stream(hipStream_t stream, SideStream* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_side_mutex);
  SideStream& ss = g_side[{dev, stream}];
  if (!ss.side) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(CPL_ERR_RUNTIME, "mixed batch: launch once on this stream before capturing it (side stream)");
    // (default priority: at the greatest stream priority the same-process A/B gained 0.2-2 %, but in the
    // bench's default line, after the north-star loop, the mixed16 side field went 2.54 -> 3.02 ms and
    // its 8-GPU shard 0.39 -> 0.55 ms; profiles/r5/side_prio/)
    if ((e = hipStreamCreateWithFlags(&ss.side, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
    if ((e = hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ss.join, hipEventDisableTiming)) != hipSuccess) return hip_fail(e, "hipEventCreate");
  }
  *out = ss;
  return CPL_OK;
}

// whether a kind split can launch on `stream` now: outside a capture always; inside one only when the
// stream's kind-list workspace and side stream already exist at this size (the default then falls
// back to the interleaved mixed kernel — bitwise the same records — instead of failing the capture:
// the solve engine captures its first iteration directly)
static bool split_ready(hipStream_t stream, int64_t batch) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs == hipStreamCaptureStatusNone) return true;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  bool ws = false, side = false;
  {
    std::lock_guard<std::mutex> lk(g_kind_ws_mutex);
    auto it = g_kind_ws.find({dev, stream});
    ws = it != g_kind_ws.end() && it->second.cap >= batch;
  }
  {
    std::lock_guard<std::mutex> lk(g_side_mutex);
    auto it = g_side.find({dev, stream});
    side = it != g_side.end() && it->second.side != nullptr;
  }
  return ws && side;
}

static void launch_residual_final(int nparts, const double* part, double* out, hipStream_t s) {
  // 1024 threads: one load round trip for up to 8 192 partials (rocprof: 4.1 us at 768 partials,
  // 4.7 us on 256 threads — three dependent round trips in the tail loop).  Past 2 * RF_CHUNK
  // partials (the per-wave partials of a 1M-instance tile launch: ~10^6) one workgroup took 200 us:
  // a first level of ceil(nparts / RF_CHUNK) workgroups, each a contiguous chunk, then one workgroup
  // over their pairs (deterministic: the split depends on nparts only)
  if (nparts <= 2 * RF_CHUNK) {
    hipLaunchKernelGGL(cpl_residual_final<1024>, dim3(1), dim3(1024), 0, s, nparts, part, out, 0);
    return;
  }
  const int nb = (nparts + RF_CHUNK - 1) / RF_CHUNK;
  double* lvl = const_cast<double*>(part) + 2 * (size_t)nparts;
  hipLaunchKernelGGL(cpl_residual_final<1024>, dim3(nb), dim3(1024), 0, s, nparts, part, lvl, RF_CHUNK);
  hipLaunchKernelGGL(cpl_residual_final<1024>, dim3(1), dim3(1024), 0, s, nb, lvl, out, 0);
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
  K.contact_rows = D.contact_rows;
  K.want_norms = 0;
  K.x_aligned16 = (reinterpret_cast<uintptr_t>(d_x) & 15) == 0 ? 1 : 0;
  for (int k = 0; k < d->n_contacts; ++k) K.map_order[k] = (int8_t)d->map_order[k];
  K.mass_default = d->mass;
  for (int j = 0; j < 3; ++j) K.gravity[j] = d->gravity[j];
  for (int j = 0; j < 6; ++j) K.wrench[j] = d->wrench[j];
  K.mu = d->mu;
  K.ground_z = d->ground_z;
  // the instance-independent Superquadric factors (15 glibc pow calls): only for the environments
  // that read them, and cached per thread for the last (R, P) seen (the launch path is on the
  // single-instance callback's critical path)
  const bool sq = d->env_kind == CPL_ENV_SUPERQUADRIC || d->env_kind == CPL_ENV_MIXED;
  struct SqFactors {
    double R[3], P[3], EJ[3], Ka[3], Kb[3], Rm2[3], Rp2[3];
    bool valid = false;
  };
  thread_local SqFactors cache;
  if (sq && !(cache.valid && std::memcmp(cache.R, d->sq_R, sizeof(cache.R)) == 0 &&
              std::memcmp(cache.P, d->sq_P, sizeof(cache.P)) == 0)) {
    for (int a = 0; a < 3; ++a) {
      const double R = d->sq_R[a], P = d->sq_P[a];
      cache.R[a] = R; cache.P[a] = P;
      cache.EJ[a] = P / std::pow(R, P);
      cache.Ka[a] = P * std::pow(R, -P);
      cache.Kb[a] = (P * P) * std::pow(R, P * -2.0);
      cache.Rm2[a] = std::pow(R, -(P * 2.0));
      cache.Rp2[a] = std::pow(R, P * 2.0);
    }
    cache.valid = true;
  }
  for (int a = 0; a < 3; ++a) {
    const double C = d->sq_C[a], R = d->sq_R[a], P = d->sq_P[a];
    K.C[a] = C; K.R[a] = R; K.P[a] = P;
    if (sq) {
      K.EJ[a] = cache.EJ[a]; K.Ka[a] = cache.Ka[a]; K.Kb[a] = cache.Kb[a];
      K.Rm2[a] = cache.Rm2[a]; K.Rp2[a] = cache.Rp2[a];
    }
    K.Psq[a] = P * P;
    K.Pm1[a] = P - 1.0;
    K.P2[a] = P * 2.0;
    K.P2m2[a] = P * 2.0 - 2.0;
    K.P2m3[a] = P * 2.0 - 3.0;
  }
  K.sq_ladder = 1;
  for (int a = 0; a < 3; ++a) {
    const double P = d->sq_P[a];
    if (!(P >= 2.0 && P <= 64.0 && P == std::floor(P))) K.sq_ladder = 0;
  }
  for (int i = 0; i < CPL_MAX_CONTACTS; ++i) {
    K.F_thr[i] = d->F_thr[i];
    K.W_p[i] = d->W_p[i];
    K.W_F[i] = d->W_F[i];
    for (int j = 0; j < 3; ++j) { K.p_ref[i][j] = d->p_ref[i][j]; K.F_ref[i][j] = d->F_ref[i][j]; }
  }
  K.W_com = d->W_com;
  for (int j = 0; j < 3; ++j) K.com_ref[j] = d->com_ref[j];
  K.fold = FOLD_NONE;
  K.jbase = D.statics_nnz;
  K.cstride = D.contact_nnz;
  K.soa = 0;
}

static size_t eval_lds_bytes(int n) { return sizeof(double) * (size_t)(TILE * n + 2 * TILE * SROW); }

// Tuning knobs (cpl_set_tuning): kernel variant and the LDS budget of one workgroup.
// Variant 0 (auto, the default) takes the pipelined kernel for the HBM-bound environments (none,
// Ground) and the tile-stationary kernel for the VALU-bound ones (Superquadric, mixed), where the
// pipelined kernel's three compute waves per workgroup leave the FP64 pipes under-filled; mixed
// batches with the Jacobian written straight to the records (variant 4 forces that everywhere).
enum { VAR_AUTO = 0, VAR_ROWSTAGE = 1, VAR_PIPE = 2, VAR_TILE = 3, VAR_TILE_JD = 4, VAR_ENTRY = 5, VAR_SPLIT = 6,
       VAR_SPLIT_JD = 7 };
static int g_variant = VAR_AUTO;
static size_t g_lds_budget = 0;    // 0 = per-kernel default (tile 32 KiB, pipelined 48 KiB)
static int g_wg = 256;             // threads per tile workgroup (128 or 256)
static int g_nt = 1;               // non-temporal output stores
static int g_ablate = 0;           // measurement-only: 1 = skip the compute phase, 2 = skip the stores,
                                   // 4 = the kind split's halves one after the other on the launch stream,
                                   // 8 = the split's Ground half issued before the Superquadric half,
                                   // 16 / 64 / 128 = the split's Ground list at 48 / 36 / 32 KiB
                                   // (default 40), 32 = its Superquadric tiles at 40 KiB (default 48),
                                   // 256 / 512 = every Ground workgroup walking / two per CU
                                   // (default one per CU while the Superquadric list is non-empty),
                                   // 1024 / 2048 = the Ground half's compute waves at priority 1 / 2,
                                   // 4096 = the 4-instance Superquadric list tiles at the default priority,
                                   // 8192 = the tile kernel's phase barriers skipped (wrong outputs),
                                   // 16384 = the split's Superquadric grid for half the batch

static size_t tile_budget() { return g_lds_budget ? g_lds_budget : 48 * 1024; }
static size_t pipe_budget() { return g_lds_budget ? g_lds_budget : 48 * 1024; }
static bool use_rowstage() { return g_variant == VAR_ROWSTAGE; }
static bool use_pipe(const KParams& K) {
  if (!K.x_aligned16) return false;  // the LDS-DMA loader copies 16-byte granules
  if (g_variant == VAR_PIPE) return true;
  return g_variant == VAR_AUTO && (K.env_kind == CPL_ENV_NONE || K.env_kind == CPL_ENV_GROUND);
}

// size_without_j: the tile size is chosen as if the Jacobian were written straight to the records
// (the layouts that cannot, SoA, then stage it in a larger LDS image) so that every layout of a batch
// runs the same tiles and the fused per-tile residual partials reduce in the same order
static int32_t plan_tile(KParams& K, bool g, bool j, bool f, bool grad, int t_max = 64, bool size_without_j = false,
                         size_t budget = 0) {
  if (!budget) budget = tile_budget();
  K.want_g = g; K.want_j = j; K.want_f = f; K.want_grad = grad;
  const bool sq = K.env_kind == CPL_ENV_SUPERQUADRIC || K.env_kind == CPL_ENV_MIXED;
  K.LR = K.N * SQ_L + 1;  // odd instance stride of the SQ scratch: conflict-free LDS banks
  const size_t per = sizeof(double) * (size_t)(K.n + (g ? K.m : 0) + (j && !K.jdirect ? K.nnz : 0) +
                                               (grad ? K.n : 0) + (sq ? K.LR : 0) + (j && K.jdirect ? 6 : 0));
  const size_t per_t = size_without_j ? per - sizeof(double) * (size_t)(j && !K.jdirect ? K.nnz : 0) : per;
  const size_t fixed = sizeof(double) * 72 + sizeof(CTab);  // index lists + parameter table
  int T = 64, logT = 6;
  while (T > t_max) { T >>= 1; --logT; }
  while (T > 2 && (size_t)T * per_t + fixed > budget) { T >>= 1; --logT; }
  // (T >= 2 is even, so every tile of every record array starts on a 16-byte boundary; below 8 the
  // tile boundaries no longer fall on 128-byte lines — the price of more resident workgroups for
  // the large VALU-bound records)
  if ((size_t)T * per + fixed > 160 * 1024) return fail(CPL_ERR_UNSUPPORTED, "problem too large for one LDS tile");
  K.T = T; K.logT = logT;
  K.cost_seg = (f || grad) ? K.N + 4 : -1;
  K.S = K.N + 4 + ((f || grad) ? 1 : 0);
  K.offG = T * K.n;
  K.offJ = K.offG + (g ? T * K.m : 0);
  K.offD = K.offJ + (j && !K.jdirect ? T * K.nnz : 0);
  K.offL = K.offD + (grad ? T * K.n : 0);
  K.offA = K.offL + (sq ? T * K.LR : 0);
  K.offI = K.offA + (j && K.jdirect ? 6 * T : 0);
  K.offI = (K.offI + 1) & ~1;
  K.offRB = K.offI + 72;  // (instance lists) the tile rows' instances, T int64
  return CPL_OK;
}

// Pipelined kernel layout: x double buffer, masses and tags (double buffered), outputs, SQ scratch
static int32_t plan_pipe(KParams& K, bool g, bool j, bool f, bool grad, size_t extra_fixed = 0) {
  K.want_g = g; K.want_j = j; K.want_f = f; K.want_grad = grad;
  const bool sq = K.env_kind == CPL_ENV_SUPERQUADRIC || K.env_kind == CPL_ENV_MIXED;
  K.LR = K.N * SQ_L + 1;
  const size_t per = sizeof(double) * (size_t)(2 * K.n + 3 + (g ? K.m : 0) + (j ? K.nnz : 0) + (grad ? K.n : 0) +
                                               (sq ? K.LR : 0));
  const size_t fixed = sizeof(double) * (72 + 8) + sizeof(CTab) + extra_fixed;
  int T = 64, logT = 6;
  while (T > 8 && (size_t)T * per + fixed > pipe_budget()) { T >>= 1; --logT; }
  if ((size_t)T * per + fixed > 160 * 1024) return fail(CPL_ERR_UNSUPPORTED, "problem too large for one LDS tile");
  K.T = T; K.logT = logT;
  K.cost_seg = (f || grad) ? K.N + 4 : -1;
  K.S = K.N + 4 + ((f || grad) ? 1 : 0);
  auto up2 = [](int v) { return (v + 1) & ~1; };
  K.offX1 = up2(T * K.n);
  K.offMB = K.offX1 + up2(T * K.n);
  K.offTB = K.offMB + 2 * T;
  K.offG = K.offTB + T;  // 2*T ints
  K.offJ = K.offG + (g ? T * K.m : 0);
  K.offD = K.offJ + (j ? T * K.nnz : 0);
  K.offL = K.offD + (grad ? T * K.n : 0);
  K.offI = up2(K.offL + (sq ? T * K.LR : 0));
  return CPL_OK;
}

// Entry kernel layout (doubles): x double buffer, masses [2][T], row bases [2][T] (int64), the cone
// scratch [T][N][ENT_CS], the statics scratch [T][12]; T even, at most 64, the largest that fits the
// LDS budget (no output image: 16-contact records keep 12-instance tiles in 48 KiB)
static int32_t plan_entry(KParams& K, bool g, bool j, bool f, bool grad, bool list = false, size_t list_budget = 0) {
  K.want_g = g; K.want_j = j; K.want_f = f; K.want_grad = grad;
  const size_t per = sizeof(double) * (size_t)(2 * ((K.n + 1) & ~1) + 4 + K.N * ENT_PC + 12);
  const size_t fixed = sizeof(double) * (size_t)(8 + 2 + (K.m + K.nnz + 1) / 2) + sizeof(CTab);
  // default budget: 80 KiB for records of 12+ contacts (two workgroups per CU with ~18-instance
  // tiles: 16-contact Ground 0.81 ms against 0.88 / 1.05 ms at 64 / 48 KiB, profiles/r4), else 48 KiB
  // (instance lists, the kind split's Ground half: list_budget, 40 KiB — more loader waves per CU)
  const size_t budget = g_lds_budget ? g_lds_budget
                                     : (list && list_budget ? list_budget : (K.N >= 12 && !list ? 80 * 1024 : 48 * 1024));
  int T = 64;
  while (T > 2 && (size_t)T * per + fixed > budget) T -= 2;
  if ((size_t)T * per + fixed > 160 * 1024) return fail(CPL_ERR_UNSUPPORTED, "problem too large for one LDS tile");
  K.T = T;
  K.logT = 0;
  auto up2 = [](int v) { return (v + 1) & ~1; };
  const int xs = (K.n + 1) & ~1;  // (instance lists) even row stride
  K.offX1 = up2(T * xs);
  K.offMB = K.offX1 + up2(T * xs);
  K.offRB = K.offMB + 2 * T;
  K.offCS = K.offRB + 2 * T;                          // scratch [T][12 + ENT_PC N]
  K.offST = K.offCS + T * (12 + ENT_PC * K.N);        // constants (2), then the opcode tables
  K.offI = up2(K.offST + 2 + (K.m + K.nnz + 1) / 2);
  return CPL_OK;
}
// the entry-parallel kernel: forced (variants 5, 6), or by default for records of 12+ contacts (the
// 16-contact Ground records: 0.81 against the pipelined kernel's 1.11 ms at 524 288 instances; the
// pipelined kernel stays faster at 4 contacts, 0.40 against 0.45 ms at 1 048 576; profiles/r4)
static bool use_entry(const KParams& K, int32_t flags) {
  const bool want = g_variant == VAR_ENTRY || g_variant == VAR_SPLIT || (g_variant == VAR_AUTO && K.N >= 12);
  return want && flags == 0 && (K.nnz % 2) == 0 && (K.env_kind == CPL_ENV_NONE || K.env_kind == CPL_ENV_GROUND);
}
// mixed batches split by kind: forced (variants 6, 7) or by default (as variant 6 since round 6: the
// Superquadric half on LDS-staged uniform-axis list tiles — the contiguous kernel's code with the rows
// gathered through the list —, 1 048 576 x 16 in 2.21-2.41 ms against 2.47-2.62 for variant 7, whose
// Jacobian rows are written straight to the records; round 4: variant 7 2.64 ms against 3.28 for the
// then LDS-staged rows and 4.49 ms interleaved; profiles/r6/split/)
static bool use_split(const KParams& K, int32_t flags, int64_t batch) {
  return (g_variant == VAR_SPLIT || g_variant == VAR_SPLIT_JD || g_variant == VAR_AUTO) && flags == 0 &&
         K.env_kind == CPL_ENV_MIXED && batch <= 0x7fffffffLL;
}

struct PipeLaunch {
  const void* fn;
  size_t lds;
  int blocks_per_cu;
};

// Workspace of the fused residual norms: one partial pair per workgroup, per (device, stream) so
// that launches on different streams never share it.  Grown on demand, and a buffer is NEVER freed
// while the process runs: a HIP graph captured on the stream keeps the pointer it saw, so a later,
// larger launch on the same stream must not release it under the graph (the retired buffers are
// kept in `old`).  Growing needs hipMalloc, which a stream capture forbids: warm the launch up on
// the stream (one eager launch of the largest batch) before capturing it — a capture that would
// have to grow the workspace fails with CPL_ERR_RUNTIME instead.
struct NormWs {
  double* ptr = nullptr;
  size_t cap = 0;  // partial pairs
  std::vector<double*> old;
};
static std::mutex g_norm_ws_mutex;
static std::map<std::pair<int, hipStream_t>, NormWs> g_norm_ws;

static int32_t norm_workspace(hipStream_t stream, size_t blocks, double** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_norm_ws_mutex);
  NormWs& w = g_norm_ws[{dev, stream}];
  if (w.cap < blocks) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(CPL_ERR_RUNTIME,
                  "fused residual norms: the per-stream workspace must grow, which a stream capture forbids; "
                  "launch the largest batch once on this stream before capturing");
    const size_t cap = blocks < 4096 ? 4096 : blocks;
    double* p = nullptr;
    e = hipMalloc(&p, sizeof(double) * (NORM_HDR + 4 * cap));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc norms workspace");
    if (w.ptr) w.old.push_back(w.ptr);  // possibly captured by a graph: kept alive
    w.ptr = p;
    w.cap = cap;
  }
  *out = w.ptr;
  return CPL_OK;
}

// Launch geometry of the persistent pipelined kernel, cached per (device, kernel, LDS bytes): the
// CU count and the occupancy query cost host time on every launch otherwise (the single-instance
// TNLP path makes one launch per callback).
static std::mutex g_occ_mutex;
static std::map<std::tuple<int, const void*, size_t>, int64_t> g_occ;

static int64_t resident_blocks(const void* kern, size_t lds) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const auto key = std::make_tuple(dev, kern, lds);
  std::lock_guard<std::mutex> lk(g_occ_mutex);
  auto it = g_occ.find(key);
  if (it != g_occ.end()) return it->second;
  int cus = 256, per_cu = 1;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  const int64_t v = (int64_t)(cus > 0 ? cus : 256) * per_cu;
  g_occ.emplace(key, v);
  return v;
}

struct LGradArgs {
  const int32_t* col_ptr;
  const int32_t* csc_k;
  const int32_t* csc_row;
  const double* y;
  int32_t y_repeat;
  const uint8_t* active;
};

struct EvalScale {
  const double* df;
  const double* dc;
  const int32_t* row;
};

static int32_t launch_eval(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                           const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                           double* d_norms, hipStream_t stream, bool finish = true,
                           const LGradArgs* lg = nullptr, int32_t flags = 0, const EvalScale* sc = nullptr,
                           const uint8_t* gate = nullptr) {
  int32_t st = validate_desc(d);
  if (st) return st;
  if (flags & ~(CPL_EVAL_JAC_FOLDED | CPL_EVAL_SOA)) return fail(CPL_ERR_INVALID_ARGUMENT, "unknown eval flags");
  if (batch < 0) return fail(CPL_ERR_INVALID_ARGUMENT, "negative batch");
  if (batch == 0) {  // (an empty g may arrive as a null pointer)
    if (d_norms) {
      hipError_t e = hipMemsetAsync(d_norms, 0, 2 * sizeof(double), stream);
      if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync norms");
    }
    return CPL_OK;
  }
  if (d_norms && !d_g) return fail(CPL_ERR_INVALID_ARGUMENT, "residual norms need the g output");
  if (!d_x) return fail(CPL_ERR_INVALID_ARGUMENT, "x is required");
  if (d->env_kind == CPL_ENV_MIXED && !d_env_tag)
    return fail(CPL_ERR_INVALID_ARGUMENT, "mixed environment batch needs a per-instance env tag array");
  if ((batch + 7) / 8 > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "batch too large");
  if (!d_g && !d_jac && !d_f && !d_grad) return CPL_OK;
  KParams K;
  fill_params(d, K, d_x);
  K.gate = gate;  // (honoured by the pipelined kernel; the others evaluate regardless)
  if (flags & CPL_EVAL_JAC_FOLDED) {  // values-only Jacobian records (cpl_layout.hpp)
    K.fold = fold_level(d->env_kind);
    K.nnz = folded_nnz(K.N, d->env_kind);
    K.jbase = 6 + 12 * K.N;
    K.cstride = folded_contact_nnz(d->env_kind);
  }
  K.soa = (flags & CPL_EVAL_SOA) ? 1 : 0;
  K.want_norms = d_norms != nullptr;
  K.want_lgrad = 0;
  K.y_repeat = 1;
  K.col_ptr = K.csc_k = K.csc_row = nullptr;
  K.ly = nullptr;
  K.lg_active = nullptr;
  K.sc_df = K.sc_dc = nullptr;
  K.sc_row = nullptr;
  double* ws = nullptr;
  // (the scaled evaluation: the pipelined path only; the caller scales the others itself)
  if (sc && (lg || d_norms || K.soa || !use_pipe(K) || use_split(K, flags, batch) || use_entry(K, flags)))
    return CPL_ERR_UNSUPPORTED;
  if (lg && !use_pipe(K))
    return fail(CPL_ERR_UNSUPPORTED, "fused Lagrangian gradient: pipelined (Ground / no environment) path only");
  if (!lg && use_split(K, flags, batch) && (g_variant != VAR_AUTO || split_ready(stream, batch))) {
    // mixed batch split by kind: the stable partition, then the Ground instances through the entry
    // kernel and the Superquadric ones through the Superquadric tile kernel, records in place
    KindLists kl;
    if ((st = kind_workspace(stream, batch, &kl))) return st;
    const unsigned nblk = (unsigned)((batch + PART_BLOCK - 1) / PART_BLOCK);
    hipLaunchKernelGGL(k_kind_count, dim3(nblk), dim3(PART_BLOCK), 0, stream, batch, d_env_tag, kl.blk_sq);
    hipLaunchKernelGGL(k_kind_write, dim3(nblk), dim3(PART_BLOCK), 0, stream, batch, (int)nblk, d_env_tag, kl.blk_sq,
                       kl.idx_gr, kl.idx_sq, kl.counts);
    KParams Kg = K, Ks = K;
    // the Ground list at 40 KiB (1 048 576 x 16 mixed: 2.600 against 2.626 ms at 48 KiB, profiles/r4/
    // split_lds; measurement: ablation 16 gives it 48 KiB, 32 the Superquadric tiles 40 KiB)
    const size_t list_kb = (g_ablate & 16) ? 48 : (g_ablate & 64) ? 36 : (g_ablate & 128) ? 32 : 40;
    if ((st = plan_entry(Kg, d_g != nullptr, d_jac != nullptr, d_f != nullptr, d_grad != nullptr, true,
                         list_kb * 1024)))
      return st;
    Ks.jdirect = (g_variant == VAR_SPLIT_JD && d_jac) ? 1 : 0;
    // (measurement: ablation 32 = the Superquadric tiles at 40 KiB instead of 48 — within the noise beside
    // the capped Ground walkers below: 2.603 / 2.552 against 2.540 / 2.579 ms in two runs,
    // profiles/r4/split_grid)
    if ((st = plan_tile(Ks, d_g != nullptr, d_jac != nullptr, d_f != nullptr, d_grad != nullptr, 64, false,
                        (g_ablate & 32) ? 40 * 1024 : 0)))
      return st;
    Kg.ablate = Ks.ablate = g_ablate & 3;
    const bool sequential = (g_ablate & 4) != 0;
    using EntryT = void (*)(const KParams, int64_t, const double*, const double*, const int32_t*, const int32_t*,
                            double*, double*, double*, double*, double*);
    using TileT = void (*)(const KParams, int64_t, const double*, const double*, const uint8_t*, const int32_t*,
                           const int32_t*, double*, double*, double*, double*, double*);
    const EntryT ek = g_nt ? cpl_eval_entry_kernel<CPL_ENV_GROUND, true> : cpl_eval_entry_kernel<CPL_ENV_GROUND, false>;
    const TileT tk = Ks.jdirect ? (g_nt ? cpl_eval_tile_kernel<CPL_ENV_SUPERQUADRIC, 256, true, true, true>
                                        : cpl_eval_tile_kernel<CPL_ENV_SUPERQUADRIC, 256, false, true, true>)
                                : (g_nt ? cpl_eval_tile_kernel<CPL_ENV_SUPERQUADRIC, 256, true, false, true>
                                        : cpl_eval_tile_kernel<CPL_ENV_SUPERQUADRIC, 256, false, false, true>);
    const size_t lds_g = sizeof(double) * (size_t)Kg.offI;
    const size_t lds_s = sizeof(double) * (size_t)(Ks.offRB + Ks.T);
    const int64_t ntg = (batch + Kg.T - 1) / Kg.T;
    const int64_t want = resident_blocks(reinterpret_cast<const void*>(ek), lds_g);
    // the Ground half's persistent grid at full residency, of which one workgroup per CU walks the tiles
    // while the Superquadric list is non-empty (the other slots left to its tiles on the other stream:
    // 1 048 576 x 16 mixed 2.54-2.58 against 2.61 ms with every workgroup walking, profiles/r4/split_grid);
    // all of it when the batch is all Ground (the cap decided on the device, from the partition's
    // counts: 1.31 ms for 524 288 all-Ground mixed instances, as uncapped; a cap fixed at launch had
    // cost 2.37).  Measurement: ablation 256 = no cap, 512 = two per CU.
    // Not below 262 144 instances: at the 8-GPU shard of configs[3] (131 072 x 16) the capped walkers ran
    // ~90 us past the Superquadric half (0.432 ms capped against 0.394 uncapped; 262 144 / 524 288 /
    // 1 048 576: within noise either way, profiles/r5/split_cap)
    const int64_t want_g = want;
    if (!(g_ablate & 256) && batch >= (int64_t)1 << 18) {
      int dev = 0, cus = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      Kg.grid_cap = (int32_t)((g_ablate & 512) ? 2 * cus : cus);
    }
    Kg.cw_prio = (g_ablate & 1024) ? 1 : (g_ablate & 2048) ? 2 : 0;
    // the Superquadric list tiles' gather / copy-out at a raised wave priority (measurement: ablation
    // 4096 leaves the 4-instance tiles at the default priority)
    Ks.list_prio = ((g_ablate & 4096) && Ks.T < 8) ? 0 : 1;
    const unsigned grid_g = (unsigned)(ntg < want_g ? ntg : want_g);
    // every tile the list may hold (measurement only, ablation 16384: half of them — correct only for
    // batches with at most half their instances Superquadric, e.g. the bench's alternating tags — to
    // price the empty workgroups past the list)
    const int64_t grid_inst = (g_ablate & 16384) ? (batch + 1) / 2 : batch;
    const unsigned grid_s = (unsigned)((grid_inst + Ks.T - 1) / Ks.T);
    const size_t nparts = (size_t)grid_g + (size_t)grid_s * 4;
    if (K.want_norms && (st = norm_workspace(stream, nparts, &ws))) return st;
    // the two halves on two streams (fork after the partition, join before the norms' finish): the
    // memory-bound Ground records and the latency-bound Superquadric tiles share the CUs
    SideStream ss;
    if (!sequential) {
      if ((st = side_stream(stream, &ss))) return st;
      hipError_t e = hipEventRecord(ss.fork, stream);
      if (e == hipSuccess) e = hipStreamWaitEvent(ss.side, ss.fork, 0);
      if (e != hipSuccess) return hip_fail(e, "mixed split fork");
    }
    const bool ground_first = (g_ablate & 8) != 0;  // (measurement) the Ground half's launch issued first
    auto launch_s = [&]() {
      hipLaunchKernelGGL(tk, dim3(grid_s), dim3(256), lds_s, stream, Ks, batch, d_x, d_mass, d_env_tag, kl.idx_sq,
                         kl.counts + 1, d_g, d_jac, d_f, d_grad, ws ? ws + 2 * (size_t)grid_g : nullptr);
    };
    if (!ground_first) launch_s();
    hipLaunchKernelGGL(ek, dim3(grid_g), dim3(256), lds_g, sequential ? stream : ss.side, Kg, batch, d_x, d_mass,
                       kl.idx_gr, kl.counts, d_g, d_jac, d_f, d_grad, ws);
    if (ground_first) launch_s();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "mixed split launch");
    if (!sequential) {
      e = hipEventRecord(ss.join, ss.side);
      if (e == hipSuccess) e = hipStreamWaitEvent(stream, ss.join, 0);
      if (e != hipSuccess) return hip_fail(e, "mixed split join");
    }
    if (K.want_norms && finish) launch_residual_final((int)nparts, ws + NORM_HDR, d_norms, stream);
    return CPL_OK;
  }
  if (!lg && use_entry(K, flags)) {
    st = plan_entry(K, d_g != nullptr, d_jac != nullptr, d_f != nullptr, d_grad != nullptr);
    if (st) return st;
    K.ablate = g_ablate;
    const size_t lds = sizeof(double) * (size_t)K.offI;
    using KernT = void (*)(const KParams, int64_t, const double*, const double*, const int32_t*, const int32_t*,
                           double*, double*, double*, double*, double*);
    static const KernT table[2][2] = {
        {cpl_eval_entry_kernel<CPL_ENV_NONE, false>, cpl_eval_entry_kernel<CPL_ENV_NONE, true>},
        {cpl_eval_entry_kernel<CPL_ENV_GROUND, false>, cpl_eval_entry_kernel<CPL_ENV_GROUND, true>}};
    const KernT kern = table[K.env_kind == CPL_ENV_GROUND ? 1 : 0][g_nt ? 1 : 0];
    const int64_t ntiles = (batch + K.T - 1) / K.T;
    const int64_t want = resident_blocks(reinterpret_cast<const void*>(kern), lds);
    const unsigned grid = (unsigned)(ntiles < want ? ntiles : want);
    if (K.want_norms && (st = norm_workspace(stream, grid, &ws))) return st;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, stream, K, batch, d_x, d_mass, nullptr, nullptr, d_g, d_jac,
                       d_f, d_grad, ws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "cpl_eval_entry_kernel launch");
    if (K.want_norms && finish) launch_residual_final((int)grid, ws + NORM_HDR, d_norms, stream);
    return CPL_OK;
  }
  if (use_pipe(K)) {
    // the fused Lagrangian gradient computes jac and grad into the tile image and stores only d_grad
    // (the fused gradient also keeps the CSC index, (n + 1) + 2 nnz ints, in LDS)
    const int csc_doubles = lg ? (K.n + 1 + 2 * K.nnz + 1) / 2 : 0;
    st = lg ? plan_pipe(K, false, true, false, true, sizeof(double) * (size_t)csc_doubles)
            : plan_pipe(K, d_g != nullptr, d_jac != nullptr, d_f != nullptr, d_grad != nullptr);
    if (st) return st;
    K.offC = K.offI + 72;
    if (lg) {
      K.want_lgrad = 1;
      K.y_repeat = lg->y_repeat;
      K.col_ptr = lg->col_ptr;
      K.csc_k = lg->csc_k;
      K.csc_row = lg->csc_row;
      K.ly = lg->y;
      K.lg_active = lg->active;
    }
    K.ablate = g_ablate;
    const size_t lds = sizeof(double) * (size_t)(K.offC + csc_doubles);
    using KernT = void (*)(const KParams, int64_t, const double*, const double*, const uint8_t*, double*, double*,
                           double*, double*, double*);
    static const KernT table[4][2] = {
        {cpl_eval_pipe_kernel<CPL_ENV_NONE, 3, false>, cpl_eval_pipe_kernel<CPL_ENV_NONE, 3, true>},
        {cpl_eval_pipe_kernel<CPL_ENV_GROUND, 3, false>, cpl_eval_pipe_kernel<CPL_ENV_GROUND, 3, true>},
        {cpl_eval_pipe_kernel<CPL_ENV_SUPERQUADRIC, 3, false>, cpl_eval_pipe_kernel<CPL_ENV_SUPERQUADRIC, 3, true>},
        {cpl_eval_pipe_kernel<CPL_ENV_MIXED, 3, false>, cpl_eval_pipe_kernel<CPL_ENV_MIXED, 3, true>}};
    static const KernT table_sc[2][2] = {
        {cpl_eval_pipe_kernel<CPL_ENV_NONE, 3, false, true>, cpl_eval_pipe_kernel<CPL_ENV_NONE, 3, true, true>},
        {cpl_eval_pipe_kernel<CPL_ENV_GROUND, 3, false, true>, cpl_eval_pipe_kernel<CPL_ENV_GROUND, 3, true, true>}};
    if (sc && K.env_kind != CPL_ENV_NONE && K.env_kind != CPL_ENV_GROUND) return CPL_ERR_UNSUPPORTED;
    if (sc) {
      K.sc_df = sc->df;
      K.sc_dc = sc->dc;
      K.sc_row = sc->row;
    }
    const KernT kern = sc ? table_sc[K.env_kind == CPL_ENV_GROUND ? 1 : 0][g_nt ? 1 : 0] : table[K.env_kind][g_nt ? 1 : 0];
    const int64_t ntiles = (batch + K.T - 1) / K.T;
    const int64_t want = resident_blocks(reinterpret_cast<const void*>(kern), lds);
    unsigned grid = (unsigned)(ntiles < want ? ntiles : want);
    if (K.want_norms && (st = norm_workspace(stream, grid, &ws))) return st;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, stream, K, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f,
                       d_grad, ws);
    if (K.want_norms) {  // per-workgroup partials -> final pair
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return hip_fail(e, "cpl_eval_pipe_kernel launch");
      if (finish) launch_residual_final((int)grid, ws + NORM_HDR, d_norms, stream);
    }
  } else if (use_rowstage() && flags == 0) {  // (the row-staged kernel writes IFOPT records only)
    const size_t lds = eval_lds_bytes(K.n);
    if (lds > 160 * 1024) return fail(CPL_ERR_UNSUPPORTED, "problem too large for one LDS tile");
    const unsigned grid = (unsigned)((batch + TILE - 1) / TILE);
    hipLaunchKernelGGL(cpl_eval_kernel, dim3(grid), dim3(TILE), lds, stream, K, batch, d_x, d_mass, d_env_tag,
                       d_g, d_jac, d_f, d_grad);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "cpl_eval_kernel launch");
    // the row-staged kernel has no fused epilogue: a separate pass over g
    return d_norms && finish ? cpl_residual_norms(d, batch, d_g, d_norms, stream) : CPL_OK;
  } else {
    // records too large for 8 per 48 KiB tile (16 Superquadric / mixed contacts, ~10 KiB each) run as
    // 4-instance tiles on 256 threads: 1 048 576 x 16 mixed 3.17 ms against 3.99 ms for the 2-instance
    // tiles on 128 threads of round 1 and 4.18 ms for 8-instance tiles
    // (profiles/r2_v7/sweep_tiles_mixed16_*.jsonl)
    // mixed batches write the Jacobian straight to the output records (their ~10 KiB records leave
    // 4 instances per 48 KiB tile otherwise; without the Jacobian image the tile holds 8): mixed16
    // 4.23 -> 3.47 ms, interleaved A/B in one process (profiles/r3/abk_mixed16.jsonl); the
    // Superquadric records are small enough that the staged copy-out wins there (0.32 vs 0.42 ms)
    const bool jd = g_variant == VAR_TILE_JD || (g_variant == VAR_AUTO && K.env_kind == CPL_ENV_MIXED);
    K.jdirect = (jd && d_jac && !K.soa && g_wg == 256) ? 1 : 0;
    st = plan_tile(K, d_g != nullptr, d_jac != nullptr, d_f != nullptr, d_grad != nullptr, 64, jd && d_jac);
    const int wg = g_wg;
    if (st) return st;
    K.ablate = g_ablate;
    const size_t lds = sizeof(double) * (size_t)(K.offRB + K.T);
    const unsigned grid = (unsigned)((batch + K.T - 1) / K.T);
    const size_t nparts = (size_t)grid * (wg / 64);  // one partial pair per wave
    if (K.want_norms && (st = norm_workspace(stream, nparts, &ws))) return st;
    using KernT = void (*)(const KParams, int64_t, const double*, const double*, const uint8_t*, const int32_t*,
                           const int32_t*, double*, double*, double*, double*, double*);
#define CPL_TILE_KERNELS(E) \
  {cpl_eval_tile_kernel<E, 128, false, false>, cpl_eval_tile_kernel<E, 128, true, false>,        \
   cpl_eval_tile_kernel<E, 256, false, false>, cpl_eval_tile_kernel<E, 256, true, false>,        \
   cpl_eval_tile_kernel<E, 256, false, true>, cpl_eval_tile_kernel<E, 256, true, true>}
    static const KernT table[4][6] = {CPL_TILE_KERNELS(CPL_ENV_NONE), CPL_TILE_KERNELS(CPL_ENV_GROUND),
                                      CPL_TILE_KERNELS(CPL_ENV_SUPERQUADRIC), CPL_TILE_KERNELS(CPL_ENV_MIXED)};
#undef CPL_TILE_KERNELS
    const KernT kern = table[K.env_kind][(K.jdirect ? 4 : (wg == 256 ? 2 : 0)) + (g_nt ? 1 : 0)];
    hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), lds, stream, K, batch, d_x, d_mass, d_env_tag, nullptr, nullptr,
                       d_g, d_jac, d_f, d_grad, ws);
    if (K.want_norms) {  // per-tile partials -> final pair
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return hip_fail(e, "cpl_eval_tile_kernel launch");
      if (finish) launch_residual_final((int)nparts, ws + NORM_HDR, d_norms, stream);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_eval_kernel launch");
  return CPL_OK;
}

// ------------------------------------------------------------------------------------------
// The solve engine's backtracking line search after the first trial (cpl_accept.hpp
// LsBacktrackArgs): one wave per instance, the instances not searching leave at once.  A trial point
// x_t = unpack(w + alpha dw) is evaluated (f and g) by the eval work items of the tile kernel on this
// one instance (contacts, statics values, cost; Superquadric axis ladders, then rows) — the same
// arithmetic as the batched eval launch — and judged by ls_acceptable_wave exactly as
// cpl_ipm_judge_take judges the first trial.  The whole search runs in the kernel: the engine's
// iteration no longer waits for the host between trials (one trial per graph launch and a flag read
// back per trial cost ~55 us each; the lock-step batch makes as many trials as its slowest instance).
// GF (with FIRST): the second-order corrections' re-solves read the KKT factors from the workspace in
// global memory (kkt_wave_resolve_gg) — large batches, where the factors' LDS image bounded the waves
// per CU; small batches keep the LDS copy (their re-solve latency is the iteration's).
// AUGR (with FIRST; IPOPT's Jacobian regularisation on): a system marked rank deficient re-solves its
// corrections with the augmented factors (kkt_aug_resolve_wave) — its own instantiation, because the
// call raises the kernel's registers past two waves per SIMD; the default search keeps its occupancy
template <int ENVK, bool RESTO, bool FIRST, bool GF = false, bool AUGR = false>
__global__ __launch_bounds__(64) void cpl_ls_backtrack_kernel(const KParams K, const LsBacktrackArgs A) {
  extern __shared__ __align__(16) double smem[];
  __shared__ double s_f;
  const int64_t b = blockIdx.x;
  if (b >= A.batch) return;
  if (FIRST && A.aug_sel != 0 && (A.aug_sel == 1) == (A.aug_dc[b] != 0.0)) return;  // (the other launch's)
  const int lane = threadIdx.x;
  if (FIRST && !GF && A.with_post) {  // the post-step quantities and the search's setup of this instance
    ipm_post_step_one(A.post, b, A.setup);
    // lane 0 stored them to global memory; every lane reloads them below: a workgroup barrier (its
    // release / acquire fences wait for the stores and order the loads behind them — also if the block
    // ever holds more than one wave; one wave today, so the barrier itself costs nothing)
    __syncthreads();
  }
  const bool act = A.act[b] != 0;
  bool searching = act && A.searching[b] != 0;
  double al = A.alpha[b];
  double st_alpha = A.st_alpha[b];
  if (searching && (FIRST || A.max_trials > 0)) {
    const int n = A.n, m = A.m, nf = A.nf, nw = A.nw, N = K.N;
    constexpr bool SQK = ENVK == CPL_ENV_SUPERQUADRIC || ENVK == CPL_ENV_MIXED;
    const int nL = SQK ? N * SQ_L : 0;
    double* X = smem;
    double* G = X + n;
    double* wt = G + m;
    double* L = wt + nw;  // [N][SQ_L] Superquadric scratch
    double* Dv = L + nL;  // (FIRST) the second-order correction's step
    double* kk = smem + ((n + m + 2 * nw + nL + 1) & ~1);  // (FIRST) the KKT re-solve's LDS image
    load_ctab(K);
    __syncthreads();
    const double* wb = A.w + b * nw;
    const double* db = A.dw + b * nw;
    const double* Xb = A.Xbase + b * n;
    const double m_i = A.mass ? A.mass[b] : K.mass_default;
    const bool sq = ENVK == CPL_ENV_SUPERQUADRIC ||
                    (ENVK == CPL_ENV_MIXED && A.env_tag[b] == CPL_ENV_SUPERQUADRIC);
    const double a_min = A.a_min[b], mub = A.mu[b], tk = A.theta_k[b], pk = A.phi_k[b], g = A.gd[b];
    const uint8_t sw = A.switch_ok[b];
    const double thmax = A.theta_max[b];
    const double* ft = A.filt_t + b * A.nfilt;
    const double* fp = A.filt_p + b * A.nfilt;
    // One trial: the point w + step dir (cpl_ipm_trial_point's arithmetic), f and g there, theta and
    // the barrier objective, the acceptance test with the step al_j (cpl_ipm_judge_take's arithmetic).
    // Leaves the trial's g in G, its w in wt, its f in s_f.
    auto trial = [&](const double* dir, double step, double al_j, double& th_out, bool& aug) -> bool {
      __syncthreads();  // the LDS images of the previous trial are read no more
      for (int k = lane; k < nw; k += 64) wt[k] = wb[k] + step * dir[k];
      for (int j = lane; j < n; j += 64) {
        const int k = A.freepos[j];
        X[j] = k >= 0 ? wb[k] + step * dir[k] : Xb[j];
      }
      __syncthreads();
      // f and g of the trial point: the eval work items of one instance
      if (ENVK != CPL_ENV_NONE && ENVK != CPL_ENV_GROUND && sq) {
        for (int it = lane; it < 3 * N + 2; it += 64) {
          if (it < 3 * N) sq_axis_item<ENVK == CPL_ENV_MIXED>(K, X, it / 3, it % 3, L + (it / 3) * SQ_L, G);
          else if (it == 3 * N) statics_values_item(K, X, m_i, G, G);
          else cost_item(K, X, &s_f, nullptr);
        }
        __syncthreads();
        for (int it = lane; it < 3 * N; it += 64) sq_row_item<ENVK == CPL_ENV_MIXED>(K, X, it / 3, it % 3, L + (it / 3) * SQ_L, G, G);
      } else {
        for (int it = lane; it < N + 2; it += 64) {
          if (it < N)
            contact_item<ENVK == CPL_ENV_NONE ? CPL_ENV_NONE : CPL_ENV_GROUND>(K, X, CPL_ENV_GROUND, it, G, G);
          else if (it == N) statics_values_item(K, X, m_i, G, G);
          else cost_item(K, X, &s_f, nullptr);
        }
      }
      __syncthreads();
      if (A.dc) {  // the scaled problem's values (LsBacktrackArgs::df / dc)
        for (int r = lane; r < m; r += 64) G[r] = G[r] * A.dc[b * m + r];
        if (lane == 0) s_f = s_f * A.df[b];
        __syncthreads();
      }
      double th = 0.0;
      for (int r = lane; r < m; r += 64) {
        const int s = A.row_slack[r];
        th += fabs(s < 0 ? G[r] - A.gl[r] : G[r] - wt[nf + s]);
      }
      double lg = 0.0;
      for (int k = lane; k < nw; k += 64) {
        if (A.hasL[k]) lg += log(wt[k] - A.wl0[k]);
        if (A.hasU[k]) lg += log(A.wu0[k] - wt[k]);
      }
      double pn = 0.0, lpn = 0.0, prox = 0.0;
      if (RESTO) {  // (k_resto_judge's terms; th above is replaced by the restoration problem's)
        th = 0.0;
        for (int r = lane; r < m; r += 64) {
          const int s = A.row_slack[r];
          const double pt = A.pR[b * m + r] + al_j * A.dp[b * m + r], nt = A.nR[b * m + r] + al_j * A.dn[b * m + r];
          th += fabs((s < 0 ? G[r] - A.gl[r] : G[r] - wt[nf + s]) - pt + nt);
          pn += pt + nt;
          lpn += log(pt) + log(nt);
        }
        for (int k = lane; k < nf; k += 64) {
          const double dr = 1.0 / fmax(fabs(A.wR[b * nw + k]), 1.0);
          const double dx = wt[k] - A.wR[b * nw + k];
          prox += (dr * dr) * (dx * dx);
        }
      }
      th = wave_sum(th);
      lg = wave_sum(lg);
      double ph = s_f - mub * lg;
      if (RESTO) {
        pn = wave_sum(pn);
        lpn = wave_sum(lpn);
        prox = wave_sum(prox);
        ph = A.rho * pn + 0.5 * sqrt(mub) * prox - mub * lg - mub * lpn;
      }
      th_out = th;
      return ls_acceptable_wave(th, ph, tk, pk, g, al_j, sw, thmax, ft, fp, A.nfilt, &aug);
    };
    // the take of an accepted trial: its f, g, w (p, n) and step into the line-search state
    auto take = [&](double al_j, bool aug) {
      for (int r = lane; r < m; r += 64) A.st_g[b * m + r] = G[r];
      for (int k = lane; k < nw; k += 64) A.st_w[b * nw + k] = wt[k];
      if (RESTO)
        for (int r = lane; r < m; r += 64) {
          A.st_p[b * m + r] = A.pR[b * m + r] + al_j * A.dp[b * m + r];
          A.st_n[b * m + r] = A.nR[b * m + r] + al_j * A.dn[b * m + r];
        }
      if (lane == 0) {
        A.st_f[b] = s_f;
        A.st_alpha[b] = al_j;
        A.st_aug[b] = aug ? 1 : 0;
      }
      st_alpha = al_j;
      searching = false;
    };
    // The search as one loop with one trial call site (the trial is large: one inlined copy).
    // FIRST: the first trial at alpha_max, then IPOPT's second-order corrections of it: c_soc =
    // a c_k + c(trial) (accumulated a_soc c_soc + c(correction) from the second on), the step of
    // [M A^T; A 0] [dw; dy] = [r1; -c_soc] from the kept factors, its own fraction to the boundary,
    // the corrected point judged with the first trial's alpha; the next correction only while the
    // last one cut theta by kappa_soc (k_soc_begin_rhs / k_soc_rhs / k_soc_after's bookkeeping);
    // then alpha halved (k_halve2) and the backtracking trials (at most max_trials more).
    constexpr int KNW = 47, KM = 30;
    enum { S_FIRST, S_SOC, S_BACK };
    int stage = (FIRST && !RESTO) ? S_FIRST : S_BACK;
    int q = 0, tr = 0;
    double csoc = 0.0, a_soc = 0.0, th_old = 0.0;
    const int s_l = lane < m ? A.row_slack[lane] : -1;
    const double gl_l = lane < m ? A.gl[lane] : 0.0;
    auto cons = [&]() { return s_l >= 0 ? G[lane] - wt[nf + s_l] : G[lane] - gl_l; };  // lane < m
    while (searching && (stage != S_BACK || tr < A.max_trials)) {
      const double* dir = db;
      double step = al;
      if (FIRST && !RESTO && stage == S_SOC) {
        if (q > 0 && lane < m) csoc = a_soc * csoc + cons();
        double dwv, dyv;
        if (AUGR && A.aug_dc[b] != 0.0) {  // a regularised (augmented) system
          const Dd r = kkt_aug_resolve_wave(KNW, KM, A.aug_ws + b * kkt_aug_ws_per(KNW, KM), lane < KM ? -csoc : 0.0);
          dwv = r.a;
          dyv = r.b;
        } else if (GF)
          kkt_wave_resolve_gg<KNW, KM>(A.M + b * KNW * KNW, A.kkt_ws + b * kkt_ws_per(KNW, KM),
                                       lane < KNW ? A.r1[b * KNW + lane] : 0.0, lane < KM ? -csoc : 0.0, kk, &dwv,
                                       &dyv);
        else
          kkt_wave_resolve_g<KNW, KM>(A.M + b * KNW * KNW, A.kkt_ws + b * kkt_ws_per(KNW, KM),
                                      lane < KNW ? A.r1[b * KNW + lane] : 0.0, lane < KM ? -csoc : 0.0, kk, &dwv,
                                      &dyv);
        if (lane < nw) Dv[lane] = dwv;
        double r = INFINITY;  // cpl_ipm_max_step (primal)
        const double t = A.tau[b];
        for (int k = lane; k < nw; k += 64) {
          const double vk = wb[k], dk = dwv;
          if (A.hasL[k] && dk < 0.0) r = fmin(r, -t * (vk - A.wl0[k]) / dk);
          if (A.hasU[k] && dk > 0.0) r = fmin(r, -t * (A.wu0[k] - vk) / -dk);
        }
        a_soc = fmin(wave_min(r), 1.0);
        dir = Dv;
        step = a_soc;
      }
      double th;
      bool aug = false;
      if (trial(dir, step, al, th, aug)) {
        take(al, aug);
        break;
      }
      if (stage == S_FIRST && A.max_soc > 0 && th >= tk) {
        if (lane < m) csoc = al * A.c[b * m + lane] + cons();
        a_soc = al;
        th_old = th;
        stage = S_SOC;
        continue;
      }
      if (stage == S_SOC && ++q < A.max_soc && th <= LS_KAPPA_SOC * th_old) {
        th_old = th;
        continue;
      }
      if (stage == S_BACK) ++tr;
      stage = S_BACK;
      al = 0.5 * al;  // IPOPT: the next trial only above alpha_min
      searching = al > a_min;
    }
  }
  if (lane == 0) {
    if (act) {
      A.searching[b] = searching ? 1 : 0;
      A.alpha[b] = al;
    }
    if (RESTO) {
      if (searching) A.any[2] = 1;
    } else {
      if (searching) A.any[0] = 1;
      // a soft restoration candidate: no accepted trial (or in the soft phase, within its budget)
      const bool sn = A.soft_now[b] != 0;
      if (act && !A.tiny[b] && ((sn && A.soft_cnt[b] <= LS_MAX_SOFT_RESTO) || (!sn && !(st_alpha > 0.0))))
        A.any[1] = 1;
    }
  }
  if (!RESTO && A.soft_ws) {  // the soft restoration step's start (LsBacktrackArgs::soft_ws)
    const bool sn = A.soft_now[b] != 0;
    const bool t = act && !A.tiny[b] && ((sn && A.soft_cnt[b] <= LS_MAX_SOFT_RESTO) || (!sn && !(st_alpha > 0.0)));
    const double as = fmin(A.a_max[b], A.a_z[b]);
    const int nw = A.nw, n = A.n;
    for (int k = lane; k < nw; k += 64) A.soft_ws[b * nw + k] = A.w[b * nw + k] + (t ? as : 0.0) * A.dw[b * nw + k];
    for (int j = lane; j < n; j += 64) {
      const int k = A.freepos[j];
      A.soft_X[b * n + j] = k >= 0 ? A.w[b * nw + k] + (t ? as : 0.0) * A.dw[b * nw + k] : A.Xbase[b * n + j];
    }
    if (lane == 0) {
      A.soft_try[b] = t ? 1 : 0;
      A.a_soft[b] = as;
    }
  }
}

constexpr int64_t LS_GF_MIN = 2048;  // batches from this size re-solve from the factors in global memory
// the fused first-trial kernel takes the post-step prologue (with_post) below LS_GF_MIN only: in the
// global-factor form it would cost that kernel its second wave per SIMD (238 VGPRs + 24 AGPRs)
bool ls_post_prologue(int64_t batch) { return batch < LS_GF_MIN; }

int32_t ls_backtrack(const cpl_problem_desc* d, const LsBacktrackArgs& a, hipStream_t stream) {
  if (a.batch <= 0) return CPL_OK;
  if (a.batch > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "ls_backtrack: batch too large");
  KParams K;
  fill_params(d, K, a.w);
  if (K.n != a.n || K.m != a.m) return fail(CPL_ERR_INVALID_ARGUMENT, "ls_backtrack: problem dimensions differ");
  K.want_g = 1;
  K.want_f = 1;
  K.want_j = 0;
  K.want_grad = 0;
  K.fold = FOLD_NONE;
  const bool sq = d->env_kind == CPL_ENV_SUPERQUADRIC || d->env_kind == CPL_ENV_MIXED;
  if (d->env_kind == CPL_ENV_MIXED && !a.env_tag) return fail(CPL_ERR_INVALID_ARGUMENT, "ls_backtrack: mixed needs tags");
  const bool first = a.first != 0;
  if (a.with_post && (!first || a.batch >= LS_GF_MIN))
    return fail(CPL_ERR_INVALID_ARGUMENT, "ls_backtrack: the post-step prologue is for the first trial below LS_GF_MIN");
  if (first && (a.resto || a.nw != 47 || a.m != 30 || !a.c || !a.M || !a.r1 || !a.kkt_ws || !a.tau))
    return fail(CPL_ERR_INVALID_ARGUMENT, "ls_backtrack: the fused first trial needs a 47 x 30 system and its buffers");
  const size_t nL = sq ? (size_t)K.N * SQ_L : 0;
  size_t lds = sizeof(double) * ((size_t)a.n + a.m + a.nw + nL + 2);
  const bool gf = first && a.batch >= LS_GF_MIN;  // the re-solves' factors from global memory
  if (first)
    lds = sizeof(double) * ((((size_t)a.n + a.m + 2 * (size_t)a.nw + nL + 1) & ~(size_t)1) +
                            (gf ? 2 * 47 : KktWave<47, 30>::LDS));
  using KernT = void (*)(const KParams, const LsBacktrackArgs);
#define CPL_LS_KERNELS(R, F, G, AG)                                                                            \
  {cpl_ls_backtrack_kernel<CPL_ENV_NONE, R, F, G, AG>, cpl_ls_backtrack_kernel<CPL_ENV_GROUND, R, F, G, AG>,   \
   cpl_ls_backtrack_kernel<CPL_ENV_SUPERQUADRIC, R, F, G, AG>, cpl_ls_backtrack_kernel<CPL_ENV_MIXED, R, F, G, AG>}
  static const KernT table[6][4] = {CPL_LS_KERNELS(false, false, false, false), CPL_LS_KERNELS(true, false, false, false),
                                    CPL_LS_KERNELS(false, true, false, false), CPL_LS_KERNELS(false, true, true, false),
                                    CPL_LS_KERNELS(false, true, false, true), CPL_LS_KERNELS(false, true, true, true)};
#undef CPL_LS_KERNELS
  const bool augr = first && a.aug_ws && a.aug_dc;
  if (a.resto && (!a.pR || !a.nR || !a.dp || !a.dn || !a.wR || !a.st_p || !a.st_n))
    return fail(CPL_ERR_INVALID_ARGUMENT, "ls_backtrack: restoration search without its buffers");
  if (augr && gf) {  // large batches: the unmarked instances in the default instantiation, the marked in AUGR
    LsBacktrackArgs a1 = a, a2 = a;
    a1.aug_sel = 1;
    a2.aug_sel = 2;
    hipLaunchKernelGGL(table[3][K.env_kind], dim3((unsigned)a.batch), dim3(64), lds, stream, K, a1);
    hipLaunchKernelGGL(table[5][K.env_kind], dim3((unsigned)a.batch), dim3(64), lds, stream, K, a2);
  } else {
    hipLaunchKernelGGL(table[first ? (gf ? 3 : 2) + (augr ? 2 : 0) : (a.resto ? 1 : 0)][K.env_kind],
                       dim3((unsigned)a.batch), dim3(64), lds, stream, K, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_ls_backtrack_kernel launch");
  return CPL_OK;
}

// per-device residual workspace (RN_GRID partial pairs), allocated once
static std::mutex g_ws_mutex;
static double* g_ws[64] = {nullptr};

// (internal, the solve engine) cpl_eval_batch_ex of the NLP-scaled problem: f, grad times df[b], g, J
// times dc[b, row]; CPL_ERR_UNSUPPORTED (nothing launched) where the evaluation does not take the
// pipelined kernel — the caller then scales the outputs itself
int32_t eval_batch_scaled(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                          const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                          int32_t flags, const double* df, const double* dc, const int32_t* row, void* stream,
                          const uint8_t* gate) {
  const EvalScale sc{df, dc, row};
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, nullptr, (hipStream_t)stream, true,
                     nullptr, flags, &sc, gate);
}

// (internal, the solve engine) cpl_eval_batch_ex with a gate byte (KParams::gate)
int32_t eval_batch_gated(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                         const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                         int32_t flags, void* stream, const uint8_t* gate) {
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, nullptr, (hipStream_t)stream, true,
                     nullptr, flags, nullptr, gate);
}

}  // namespace cpl

using namespace cpl;

extern "C" {

int32_t cpl_eval_batch(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                       const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                       void* stream) {
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, nullptr, (hipStream_t)stream);
}

int32_t cpl_eval_lagrangian_grad(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                                 const uint8_t* d_env_tag, const int32_t* d_col_ptr, const int32_t* d_csc_k,
                                 const int32_t* d_csc_row, const double* d_y, int32_t y_repeat,
                                 const uint8_t* d_active, double* d_out, void* stream) {
  if (y_repeat < 1) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_eval_lagrangian_grad: y_repeat must be >= 1");
  if (batch > 0 && (!d_col_ptr || !d_csc_k || !d_csc_row || !d_y || !d_out))
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_eval_lagrangian_grad: missing buffer");
  const LGradArgs lg{d_col_ptr, d_csc_k, d_csc_row, d_y, y_repeat, d_active};
  // jac and grad f are computed into the tile image; only grad f + J^T y is stored (to d_out)
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, nullptr, nullptr, nullptr, d_out, nullptr, (hipStream_t)stream,
                     true, &lg);
}

int32_t cpl_lagrangian_hessian(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_y,
                               const uint8_t* d_active, const int32_t* d_free_idx, int32_t nf, double* d_H,
                               void* stream) {
  int32_t st = validate_desc(d);
  if (st) return st;
  if (d->env_kind != CPL_ENV_GROUND && d->env_kind != CPL_ENV_NONE)
    return fail(CPL_ERR_UNSUPPORTED, "cpl_lagrangian_hessian: Ground / no-environment problems only");
  KParams K;
  fill_params(d, K, d_x);
  if (batch < 0 || nf <= 0 || nf > K.n) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_lagrangian_hessian: bad sizes");
  if (batch == 0) return CPL_OK;
  if (!d_x || !d_y || !d_free_idx || !d_H) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_lagrangian_hessian: missing buffer");
  if (batch > 0x7fffffffLL) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_lagrangian_hessian: batch too large");
  hipLaunchKernelGGL(cpl_lagrangian_hessian_kernel, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, K, batch,
                     (int)nf, d_x, d_y, d_active, d_free_idx, d_H);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_lagrangian_hessian launch");
  return CPL_OK;
}

int32_t cpl_eval_batch_ex(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                          const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                          double* d_norms, int32_t flags, void* stream) {
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, d_norms, (hipStream_t)stream, true,
                     nullptr, flags);
}

int32_t cpl_eval_batch_norms(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                             const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                             double* d_norms, void* stream) {
  if (!d_norms) return fail(CPL_ERR_INVALID_ARGUMENT, "d_norms is required");
  return launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, d_norms, (hipStream_t)stream);
}

int32_t cpl_set_tuning(int32_t kernel_variant, int32_t tile_lds_kb, int32_t wg_threads, int32_t nt_stores,
                       int32_t ablate) {
  if (ablate < 0 || (ablate > 2 && (ablate & ~(4 | 8 | 16 | 32 | 64 | 128 | 256 | 512 | 1024 | 2048 | 4096 | 8192 | 16384))))
    return fail(CPL_ERR_INVALID_ARGUMENT, "unknown ablation");
  g_ablate = ablate;
  if (kernel_variant < VAR_AUTO || kernel_variant > VAR_SPLIT_JD) return fail(CPL_ERR_INVALID_ARGUMENT, "unknown kernel variant");
  if (tile_lds_kb != 0 && (tile_lds_kb < 8 || tile_lds_kb > 160))
    return fail(CPL_ERR_INVALID_ARGUMENT, "LDS budget out of [8, 160] KiB");
  if (wg_threads != 128 && wg_threads != 256) return fail(CPL_ERR_INVALID_ARGUMENT, "workgroup size must be 128 or 256");
  g_variant = kernel_variant;
  g_lds_budget = (size_t)tile_lds_kb * 1024;
  g_wg = wg_threads;
  g_nt = nt_stores ? 1 : 0;
  return CPL_OK;
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
  launch_residual_final((int)blocks, ws, d_out, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "cpl_residual_final launch");
  return CPL_OK;
}

int32_t cpl_time_eval_batch(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                            const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                            double* d_norms, void* stream, int32_t reps, double* ms_per_launch) {
  return cpl_time_eval_batch_ex(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, d_norms, 0, stream, reps,
                                ms_per_launch);
}

int32_t cpl_time_eval_batch_ex(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                               const uint8_t* d_env_tag, double* d_g, double* d_jac, double* d_f, double* d_grad,
                               double* d_norms, int32_t flags, void* stream, int32_t reps, double* ms_per_launch) {
  if (!ms_per_launch || reps < 1) return fail(CPL_ERR_INVALID_ARGUMENT, "bad timing arguments");
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t e0, e1;
  hipError_t e = hipEventCreate(&e0);
  if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
  e = hipEventCreate(&e1);
  if (e != hipSuccess) { (void)hipEventDestroy(e0); return hip_fail(e, "hipEventCreate"); }
  int32_t st = CPL_OK;
  (void)hipEventRecord(e0, s);
  // back-to-back eval kernels (with the fused per-workgroup norms when d_norms != NULL; the
  // one-workgroup finish, a separate kernel, is left out of the timed launches)
  for (int32_t r = 0; r < reps && st == CPL_OK; ++r)
    st = launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, d_norms, s, /*finish=*/false, nullptr,
                     flags);
  (void)hipEventRecord(e1, s);
  e = hipEventSynchronize(e1);
  if (st == CPL_OK && e != hipSuccess) st = hip_fail(e, "hipEventSynchronize");
  float ms = 0.0f;
  if (st == CPL_OK) {
    e = hipEventElapsedTime(&ms, e0, e1);
    if (e != hipSuccess) st = hip_fail(e, "hipEventElapsedTime");
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (st == CPL_OK) *ms_per_launch = (double)ms / reps;
  // leave d_norms valid for the caller
  if (st == CPL_OK && d_norms)
    st = launch_eval(d, batch, d_x, d_mass, d_env_tag, d_g, d_jac, d_f, d_grad, d_norms, s, true, nullptr, flags);
  return st;
}

}  // extern "C"
