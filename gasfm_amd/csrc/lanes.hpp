// Cross-lane butterflies on DPP (data-parallel primitives) instead of ds_bpermute.
//
// __shfl_xor lowers to ds_bpermute_b32: an LDS round trip (~100+ cycles) per step, chained
// four deep in a 16-lane sum.  Within a 16-lane row the xor partners 1, 2 and 8 are DPP lane
// patterns (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_ror:8) folded into the consuming
// v_add as an operand modifier; xor 4 has no DPP pattern, but for a SUM over an aligned group
// the half-row mirror pairs quad 0 with quad 1 just as xor 4 does (same operands, same
// association: results are bitwise identical to the xor-shuffle sums).  Partners 16 and 32
// cross rows: gfx950's lane-swap instructions (xsum16 / xsum32 below).
#pragma once

#include <hip/hip_runtime.h>

namespace gasfm {

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Partners 16 and 32 (across 16-lane rows) on gfx950's VALU lane swaps instead of ds_bpermute
// (round 5): v_permlane16_swap_b32 vdst, vsrc swaps the odd rows of vdst with the even rows of
// vsrc, v_permlane32_swap_b32 the upper half of vdst with the lower half of vsrc.  With both
// operands = v, the two results hold (v of the even / lower partner, v of the odd / upper partner)
// in every lane: their sum is v + v[lane ^ 16] (resp. ^ 32) with the same two operands as the
// shuffle sum, so bitwise the same value (IEEE addition is commutative); the partner alone is a
// select by the lane's own row (half).
__device__ __forceinline__ float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// value of lane (lane ^ O)
template <int O>
__device__ __forceinline__ float xor_lane(float v) {
  if constexpr (O == 1)
    return dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  else if constexpr (O == 2)
    return dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  else if constexpr (O == 8)
    return dpp_mov<0x128>(v);  // row_ror:8 (== xor 8 within a 16-lane row)
  else if constexpr (O == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
  } else if constexpr (O == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
  } else
    return __shfl_xor(v, O);
}

// sum over aligned groups of N lanes (N a power of two <= 64); every lane gets the group sum
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (N >= 2) v += xor_lane<1>(v);
  if constexpr (N >= 4) v += xor_lane<2>(v);
  if constexpr (N >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: quad 0 <-> quad 1 of each half-row
  if constexpr (N >= 16) v += xor_lane<8>(v);
  if constexpr (N >= 32) v = xsum16(v);
  if constexpr (N >= 64) v = xsum32(v);
  return v;
}

// v summed with its partners lane ^ O for O = O0, 2*O0, ..., 32 (keeps lane % O0)
template <int O0>
__device__ __forceinline__ float xor_sum_from(float v) {
  if constexpr (O0 <= 1) v += xor_lane<1>(v);
  if constexpr (O0 <= 2) v += xor_lane<2>(v);
  if constexpr (O0 <= 4) v += xor_lane<4>(v);
  if constexpr (O0 <= 8) v += xor_lane<8>(v);
  if constexpr (O0 <= 16) v = xsum16(v);
  if constexpr (O0 <= 32) v = xsum32(v);
  return v;
}

}  // namespace gasfm
