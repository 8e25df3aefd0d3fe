// cpl_wave.hpp — wave-level reductions and broadcasts for the one-wave / one-workgroup-per-instance
// kernels of the solve loop (cpl_kkt.hip, cpl_ipm.hip), by DPP lane permutations: a VALU operand
// modifier, no LDS round trip (ds_bpermute, what __shfl_xor lowers to, costs an LDS-crossbar trip
// per dword on the reductions' critical path).  Every lane of the wave must execute them.
#pragma once

#include <hip/hip_runtime.h>

namespace cpl {

// v moved by the DPP permutation CTRL; lanes of rows outside ROW_MASK receive `old`.  An f64
// moves as its two dwords.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_mov(double v, double old = 0.0) {
  const long long bits = __double_as_longlong(v), ob = __double_as_longlong(old);
  if constexpr (ROW_MASK == 0xf && CTRL != 0x142 && CTRL != 0x143) {
    // a full-mask permutation within rows: every lane has a source, `old` is never read — no
    // register to pre-load with it (two v_mov per f64 fewer on every reduction step)
    (void)ob;
    const int lo = __builtin_amdgcn_mov_dpp((int)(bits & 0xffffffffLL), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(bits >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
  }
  const int lo = __builtin_amdgcn_update_dpp((int)(ob & 0xffffffffLL), (int)(bits & 0xffffffffLL), CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(ob >> 32), (int)(bits >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int DPP_QUAD_XOR1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int DPP_ROW_MIRROR = 0x140;      // lane i of a row of 16 <- lane 15 - i
constexpr int DPP_ROW_HALF_MIRROR = 0x141; // lane i of a half-row of 8 <- lane 7 - i
constexpr int DPP_ROW_BCAST15 = 0x142;     // lane 15 of each row -> the next row
constexpr int DPP_ROW_BCAST31 = 0x143;     // lane 31 -> rows 2 and 3

// Broadcast lane `src` (wave-uniform) of a double with two v_readlane_b32.
__device__ __forceinline__ double wave_bcast(double v, int src) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), src);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

struct OpSum { __device__ static double f(double a, double b) { return a + b; } };
struct OpMax { __device__ static double f(double a, double b) { return fmax(a, b); } };
struct OpMin { __device__ static double f(double a, double b) { return fmin(a, b); } };

// Reductions over aligned groups of 4 / 8 lanes, the result in every lane of the group.
template <class Op = OpSum>
__device__ __forceinline__ double group4_reduce(double v) {
  v = Op::f(v, dpp_mov<DPP_QUAD_XOR1>(v));
  return Op::f(v, dpp_mov<DPP_QUAD_XOR2>(v));
}
template <class Op = OpSum>
__device__ __forceinline__ double group8_reduce(double v) {
  v = group4_reduce<Op>(v);
  return Op::f(v, dpp_mov<DPP_ROW_HALF_MIRROR>(v));
}
__device__ __forceinline__ double group4_sum(double v) { return group4_reduce<OpSum>(v); }
__device__ __forceinline__ double group8_sum(double v) { return group8_reduce<OpSum>(v); }

// Reduction over the wave, in every lane: rows of 16 by DPP, rows combined into lane 63 by the
// two row broadcasts (lanes of the other rows keep their own value: op(v, v) = v for max / min,
// and v + 0 for the sum), then read out of lane 63.
template <class Op>
__device__ __forceinline__ double wave_reduce(double v, double ident) {
  v = group8_reduce<Op>(v);
  v = Op::f(v, dpp_mov<DPP_ROW_MIRROR>(v));
  v = Op::f(v, dpp_mov<DPP_ROW_BCAST15, 0xa>(v, ident));
  v = Op::f(v, dpp_mov<DPP_ROW_BCAST31, 0xc>(v, ident));
  return wave_bcast(v, 63);
}
__device__ __forceinline__ double wave_sum(double v) { return wave_reduce<OpSum>(v, 0.0); }
__device__ __forceinline__ double wave_max(double v) { return wave_reduce<OpMax>(v, -INFINITY); }
__device__ __forceinline__ double wave_min(double v) { return wave_reduce<OpMin>(v, INFINITY); }

}  // namespace cpl
