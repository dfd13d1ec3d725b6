// Cross-lane butterflies on DPP (data-parallel primitives) instead of ds_bpermute.
//
// __shfl_xor lowers to ds_bpermute_b32: an LDS round trip (~100+ cycles) per step, chained
// four deep in a 16-lane sum.  Within a 16-lane row the xor partners 1, 2 and 8 are DPP lane
// patterns (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_ror:8) folded into the consuming
// v_add as an operand modifier; xor 4 has no DPP pattern, but for a SUM over an aligned group
// the half-row mirror pairs quad 0 with quad 1 just as xor 4 does (same operands, same
// association: results are bitwise identical to the xor-shuffle sums).  Partners 16 and 32
// cross rows and stay on __shfl_xor.
#pragma once

#include <hip/hip_runtime.h>

namespace gasfm {

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
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
  else
    return __shfl_xor(v, O);
}

// sum over aligned groups of N lanes (N a power of two <= 64); every lane gets the group sum
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (N >= 2) v += xor_lane<1>(v);
  if constexpr (N >= 4) v += xor_lane<2>(v);
  if constexpr (N >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: quad 0 <-> quad 1 of each half-row
  if constexpr (N >= 16) v += xor_lane<8>(v);
  if constexpr (N >= 32) v += __shfl_xor(v, 16);
  if constexpr (N >= 64) v += __shfl_xor(v, 32);
  return v;
}

// v summed with its partners lane ^ O for O = O0, 2*O0, ..., 32 (keeps lane % O0)
template <int O0>
__device__ __forceinline__ float xor_sum_from(float v) {
  if constexpr (O0 <= 1) v += xor_lane<1>(v);
  if constexpr (O0 <= 2) v += xor_lane<2>(v);
  if constexpr (O0 <= 4) v += xor_lane<4>(v);
  if constexpr (O0 <= 8) v += xor_lane<8>(v);
  if constexpr (O0 <= 16) v += __shfl_xor(v, 16);
  if constexpr (O0 <= 32) v += __shfl_xor(v, 32);
  return v;
}

}  // namespace gasfm
