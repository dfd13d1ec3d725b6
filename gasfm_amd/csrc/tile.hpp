// Wave-level building blocks shared by the row-tile kernels (edge_block.hip, node_block.hip).
//
// A wavefront (64 lanes) owns a 16-row tile at a time.  GEMM-shaped parts use the exact-fp32
// MFMA v_mfma_f32_16x16x4_f32 with lane l holding A[i = l&15][k = l>>4], B[k = l>>4][j = l&15]
// and C[row = 4(l>>4) + r][col = l&15] (r = 0..3).  Row reductions over a 16-lane group are
// DPP butterflies (lanes.hpp); reductions across the four lane groups use xor 16, 32.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lanes.hpp"

namespace gasfm {
namespace tile {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kW = 64;                  // wavefront
constexpr int kWaves = 4;               // waves per workgroup
constexpr int kThreads = kW * kWaves;
constexpr int TR = 16;                  // rows per tile

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Sum over the 16 lanes of a lane group (same l>>4).
__device__ __forceinline__ float sum16(float v) { return group_sum<16>(v); }
// Sum over the 4 lane groups (l>>4).
__device__ __forceinline__ float sum_groups(float v) { return xsum32(xsum16(v)); }

// Weight staging (once per workgroup): every thread issues ALL of its N / NT global loads before
// the first LDS store.  The plain `for (q = threadIdx.x; q < N; q += NT) L[f(q)] = W[q]` form
// compiles to one load + vmcnt(0) + branch per trip (the compiler cannot prove the trip
// condition uniform), i.e. ~N / NT serialised memory round trips (~20 us per kernel measured
// on the point kernels, paid before any tile work).  Requires blockDim.x == NT.
template <int N, int NT>
struct Stage {
  static constexpr int IT = (N + NT - 1) / NT;
  float v[IT];
  template <class Src>
  __device__ __forceinline__ void load(Src src) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int q = int(threadIdx.x) + k * NT;
      v[k] = src((N % NT == 0 || q < N) ? q : 0);
    }
  }
  template <class Dst>
  __device__ __forceinline__ void store(Dst dst) const {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int q = int(threadIdx.x) + k * NT;
      if (N % NT == 0 || q < N) dst(q, v[k]);
    }
  }
};

// Row-major [16 x W] tile from global (row stride ld floats, 16-byte aligned) into LDS (row
// stride LDT); rows >= nrows are zeros (nrows >= 1).  All global loads are issued before the
// LDS stores.
template <int W, int LDT>
__device__ __forceinline__ void load_tile(const float* __restrict__ X, int64_t ld, int64_t row0, int nrows,
                                          float* T, int lane) {
  constexpr int V = W / 4;            // float4 per row
  constexpr int STEPS = TR * V / kW;  // float4 per lane
  float4 v[STEPS];
#pragma unroll
  for (int u = 0; u < STEPS; ++u) {
    const int q = lane + kW * u;
    const int r = q / V, c = (q % V) * 4;
    // unconditional load of an in-range row, then zero: a load under a per-element condition
    // is branched around with a vmcnt(0) wait each, serialising the tile's loads
    v[u] = *reinterpret_cast<const float4*>(X + (row0 + (r < nrows ? r : 0)) * ld + c);
    if (r >= nrows) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < STEPS; ++u) {
    const int q = lane + kW * u;
    const int r = q / V, c = (q % V) * 4;
    float* d = T + r * LDT + c;
    d[0] = v[u].x;
    d[1] = v[u].y;
    d[2] = v[u].z;
    d[3] = v[u].w;
  }
}

// Row layout of a 16 x W tile (W = 32 or 64): lane l holds the float4 chunk l % (W/4) of rows
// l / (W/4) + (64 / (W/4)) * u, u < W/16 -- every load / store is a coalesced 16-byte access.
// rows_load issues all of a tile's loads before any use (clamped rows, zeroed past nrows).
template <int W>
__device__ __forceinline__ void rows_load(const float* __restrict__ P, int64_t ld, int64_t row0, int nrows,
                                          float4 (&v)[W / 16], int lane) {
  constexpr int V = W / 4, RS = kW / V;
#pragma unroll
  for (int u = 0; u < W / 16; ++u) {
    const int r = lane / V + RS * u;
    v[u] = *reinterpret_cast<const float4*>(P + (row0 + (r < nrows ? r : 0)) * ld + (lane % V) * 4);
    if (r >= nrows) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int W>
__device__ __forceinline__ void rows_store(float* __restrict__ P, int64_t ld, int64_t row0, int nrows,
                                           const float4 (&v)[W / 16], int lane) {
  constexpr int V = W / 4, RS = kW / V;
#pragma unroll
  for (int u = 0; u < W / 16; ++u) {
    const int r = lane / V + RS * u;
    if (r < nrows) *reinterpret_cast<float4*>(P + (row0 + r) * ld + (lane % V) * 4) = v[u];
  }
}
// LDS side (row stride LD, even: 8-byte aligned float2 accesses)
template <int W, int LD>
__device__ __forceinline__ void rows_to_lds(float* T, const float4 (&v)[W / 16], int lane) {
  constexpr int V = W / 4, RS = kW / V;
#pragma unroll
  for (int u = 0; u < W / 16; ++u) {
    float2* d = reinterpret_cast<float2*>(T + (lane / V + RS * u) * LD + (lane % V) * 4);
    d[0] = make_float2(v[u].x, v[u].y);
    d[1] = make_float2(v[u].z, v[u].w);
  }
}
template <int W, int LD>
__device__ __forceinline__ void rows_from_lds(const float* T, float4 (&v)[W / 16], int lane) {
  constexpr int V = W / 4, RS = kW / V;
#pragma unroll
  for (int u = 0; u < W / 16; ++u) {
    const float2* s = reinterpret_cast<const float2*>(T + (lane / V + RS * u) * LD + (lane % V) * 4);
    const float2 a = s[0], b = s[1];
    v[u] = make_float4(a.x, a.y, b.x, b.y);
  }
}

// Sum `N` floats per lane across the workgroup's waves (LDS scratch >= kWaves*N*kW floats,
// free for reuse); wave 0 returns the totals in v, summed in wave order (deterministic).
template <int N>
__device__ __forceinline__ void wg_reduce(float (&v)[N], float* scratch, int wave, int lane) {
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) scratch[(wave * N + k) * kW + lane] = v[k];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float s = 0.f;
      for (int w = 0; w < kWaves; ++w) s += scratch[(w * N + k) * kW + lane];
      v[k] = s;
    }
  }
}

// Ordered workgroup sum of N floats per lane (wave 0 returns the totals in v), in chunks that
// fit SF floats of LDS scratch: every wave stores its chunk values at once, then wave w' sums
// the values k = w', w' + NW, ... over the waves in wave order (0 + v_0 + v_1 + ...: the same
// bits as a serial wave-by-wave accumulation) in place, and wave 0 reads the totals back.
// Three barriers per chunk; the earlier one-wave-at-a-time form serialised NW x N dependent
// LDS read/write pairs (~25 us per launch for N = 112 over 8 waves, measured).
template <int N, int NW, int SF>
__device__ __forceinline__ void wg_reduce_ordered(float (&v)[N], float* scratch, int wave, int lane) {
  constexpr int CH = (SF / (NW * kW)) < N ? (SF / (NW * kW)) : N;  // values per chunk
  static_assert(CH >= 1, "wg_reduce_ordered: scratch too small");
#pragma unroll
  for (int k0 = 0; k0 < N; k0 += CH) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; ++k)
      if (k0 + k < N) scratch[(wave * CH + k) * kW + lane] = v[k0 + k];
    __syncthreads();
    for (int k = wave; k < CH && k0 + k < N; k += NW) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += scratch[(w * CH + k) * kW + lane];
      scratch[k * kW + lane] = s;  // wave 0's slot of value k (only this wave touches k here)
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int k = 0; k < CH; ++k)
        if (k0 + k < N) v[k0 + k] = scratch[k * kW + lane];
    }
  }
}

}  // namespace tile
}  // namespace gasfm
