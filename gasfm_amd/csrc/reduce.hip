// Deterministic column sums (bias / att / weight-gradient partials), ONE launch, no float atomics.
//   block (b, chunk) sums rows [b*R/B, (b+1)*R/B) of a 1024-column chunk into ws[b, chunk];
//   the last block of each chunk to finish (agent-scope release / relaxed ticket / acquire,
//   cdna_hip_programming.md §3 split-K recipe; correct for any block-to-XCD placement) sums
//   ws over b in block order and writes out[chunk].  B <= 64 keeps that serial sum short.
// Replaces the implicit reductions autograd performs for GATv2Conv.bias /
// GATv2Conv.att (PyG, layers.py:304-309 etc.) and LayerNorm/Linear biases.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {

constexpr int kColBlock = 256;
constexpr int kMaxColBlocks = 64;

static int colsum_blocks(int64_t rows) {
  const int64_t b = (rows + 127) / 128;
  return int(b < 1 ? 1 : (b > kMaxColBlocks ? kMaxColBlocks : b));
}

// Pass 1.  cols % 4 == 0 and 16-byte aligned rows: each thread owns a float4 column
// group (c4) and a row lane (rl); RL = 256 / (cols/4) row lanes stride the block's row
// range with 4 independent loads in flight, then the row lanes are summed through LDS
// in lane order.  Other shapes: thread per column, rows serial.
__global__ __launch_bounds__(kColBlock) void colsum_kernel(const float* __restrict__ A, int64_t rows, int cols,
                                                        int64_t ld, float* __restrict__ ws, float* __restrict__ out,
                                                        uint32_t* __restrict__ cnt) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int nb = gridDim.x;
  const int64_t r0 = rows * blockIdx.x / nb, r1 = rows * (blockIdx.x + 1) / nb;
  // blockIdx.y selects a chunk of up to 4*256 columns (wide partial matrices)
  const int cbase = blockIdx.y * 4 * kColBlock;
  A += cbase;
  ws += cbase;
  const int ccols = (cols - cbase) < 4 * kColBlock ? (cols - cbase) : 4 * kColBlock;
  const int C4 = ccols / 4;
  if ((cols & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0) {
    const int RL = kColBlock / C4;
    const int c4 = threadIdx.x % C4, rl = threadIdx.x / C4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rl < RL) {
      int64_t r = r0 + rl;
      for (; r + 3 * RL < r1; r += 4 * RL) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(A + (r + u * RL) * ld + 4 * c4);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc.x += v[u].x;
          acc.y += v[u].y;
          acc.z += v[u].z;
          acc.w += v[u].w;
        }
      }
      for (; r < r1; r += RL) {
        const float4 v = *reinterpret_cast<const float4*>(A + r * ld + 4 * c4);
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
    }
    reinterpret_cast<float4*>(sh)[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < C4) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int k = 0; k < RL; ++k) {
        const float4 v = reinterpret_cast<const float4*>(sh)[k * C4 + threadIdx.x];
        t.x += v.x;
        t.y += v.y;
        t.z += v.z;
        t.w += v.w;
      }
      reinterpret_cast<float4*>(ws + int64_t(blockIdx.x) * cols)[threadIdx.x] = t;
    }
  } else {
    for (int c = threadIdx.x; c < ccols; c += kColBlock) {
      float acc = 0.f;
      for (int64_t r = r0; r < r1; ++r) acc += A[r * ld + c];
      ws[int64_t(blockIdx.x) * cols + c] = acc;
    }
  }
  // publish this block's slab: drain, barrier, one release, one relaxed ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* flag = reinterpret_cast<uint32_t*>(sh);  // the one LDS array (its pass-1 use is over)
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(cnt + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = (t == uint32_t(nb - 1)) ? 1u : 0u;
  }
  __syncthreads();
  if (flag[0] == 0u) return;
  // last arriver of this chunk: acquire, then sum the nb slabs in block order
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int c = threadIdx.x; c < ccols; c += kColBlock) {
    float acc = 0.f;
    for (int b = 0; b < nb; ++b) acc += ws[int64_t(b) * cols + c];
    out[cbase + c] = acc;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace gasfm

using namespace gasfm;

extern "C" int64_t gasfm_colsum_ws_floats(int64_t rows, int32_t cols) {
  return int64_t(colsum_blocks(rows)) * cols;
}

extern "C" int32_t gasfm_colsum_counters(int32_t cols) { return (cols + 4 * kColBlock - 1) / (4 * kColBlock); }

extern "C" int gasfm_colsum(const float* A, int64_t rows, int32_t cols, int64_t ld, float* ws, float* out,
                            uint32_t* counters, void* stream) {
  GASFM_REQUIRE(rows >= 0 && cols > 0 && ld >= cols, "gasfm_colsum: rows=%lld cols=%d ld=%lld", (long long)rows,
                cols, (long long)ld);
  GASFM_REQUIRE(ws && out && counters && (rows == 0 || A), "gasfm_colsum: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = colsum_blocks(rows);
  const int nchunk = (cols + 4 * kColBlock - 1) / (4 * kColBlock);
  hipLaunchKernelGGL(colsum_kernel, dim3(nb, nchunk), dim3(kColBlock), 4 * kColBlock * sizeof(float), st, A, rows,
                     cols, ld, ws, out, counters);
  return launch_status("gasfm_colsum");
}
