// Deterministic column sums (bias / att / weight-gradient partials), ONE launch, no float atomics.
//   block (b, chunk) sums rows [b*R/B, (b+1)*R/B) of a 1024-column chunk into ws[b, chunk];
//   the last block of each chunk to finish sums ws over b in block order and writes
//   out[chunk].  Hand-off (cdna_hip_programming.md §3 / Guideline 16, sc1 form; correct for any
//   block-to-XCD placement): slabs stored write-through (sc1), drained, a relaxed agent-scope
//   ticket, and sc1 loads in the reducer -- no L2 writeback fence.  B <= 64 keeps the serial
//   sum short.
// Replaces the implicit reductions autograd performs for GATv2Conv.bias /
// GATv2Conv.att (PyG, layers.py:304-309 etc.) and LayerNorm/Linear biases.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {

constexpr int kColBlock = 256;
constexpr int kChunkCols = 256;  // columns per block: 64 float4 column groups x 4 row lanes
constexpr int kMaxColBlocks = 64;

// write-through (sc1) store of 16 bytes as two agent-scope 8-byte atomic stores
__device__ __forceinline__ void st_sc1(float* p, float4 v) {
  uint64_t a, b;
  __builtin_memcpy(&a, &v.x, 8);
  __builtin_memcpy(&b, &v.z, 8);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p) + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// >= 64 rows per block (each of a 256-column chunk's 4 row lanes requests its 16 rows at once),
// <= 64 blocks per column chunk.  Round 1 used 16 rows per block: 4x the workgroups, each a
// full load / publish / ticket / reduce latency chain, and 4x the slabs for the last arriver to
// fold (the end-of-backward batched sums ran at ~1 TB/s).
static int colsum_blocks(int64_t rows) {
  const int64_t b = (rows + 63) / 64;
  return int(b < 1 ? 1 : (b > kMaxColBlocks ? kMaxColBlocks : b));
}

// Pass 1.  cols % 4 == 0 and 16-byte aligned rows: each thread owns a float4 column
// group (c4) and a row lane (rl); RL = 256 / (cols/4) row lanes stride the block's row
// range with 4 independent loads in flight, then the row lanes are summed through LDS
// in lane order.  Other shapes: thread per column, rows serial.
// One block of a colsum: row block bx of nb, column chunk by (counter cnt[by]).
__device__ __forceinline__ void colsum_block(const float* __restrict__ A, int64_t rows, int cols, int64_t ld,
                                             float* __restrict__ ws, float* __restrict__ out,
                                             uint32_t* __restrict__ cnt, int bx, int nb, int by, float* sh) {
  const int64_t r0 = rows * bx / nb, r1 = rows * (bx + 1) / nb;
  // by selects a chunk of up to 256 columns (wide partial matrices)
  const int cbase = by * kChunkCols;
  A += cbase;
  ws += cbase;
  const int ccols = (cols - cbase) < kChunkCols ? (cols - cbase) : kChunkCols;
  const int C4 = ccols / 4;
  if ((cols & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0) {
    const int RL = kColBlock / C4;
    const int c4 = threadIdx.x % C4, rl = threadIdx.x / C4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rl < RL) {
      int64_t r = r0 + rl;
      for (; r + 15 * RL < r1; r += 16 * RL) {
        float4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const float4*>(A + (r + u * RL) * ld + 4 * c4);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          acc.x += v[u].x;
          acc.y += v[u].y;
          acc.z += v[u].z;
          acc.w += v[u].w;
        }
      }
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
      st_sc1(ws + int64_t(bx) * cols + 4 * threadIdx.x, t);
    }
  } else {
    for (int c = threadIdx.x; c < ccols; c += kColBlock) {
      float acc = 0.f;
      for (int64_t r = r0; r < r1; ++r) acc += A[r * ld + c];
      __hip_atomic_store(ws + int64_t(bx) * cols + c, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // publish: the slab was stored write-through (sc1), so no release fence (which would write
  // back every dirty L2 line of this XCD, e.g. the previous kernel's outputs): every wave
  // drains its stores, barrier, one relaxed agent-scope ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* flag = reinterpret_cast<uint32_t*>(sh);  // the one LDS array (its pass-1 use is over)
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(cnt + by, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = (t == uint32_t(nb - 1)) ? 1u : 0u;
  }
  __syncthreads();
  if (flag[0] == 0u) return;
  // last arriver of this chunk: every slab load is an sc1 (agent-scope) load, so no acquire
  // fence; slabs summed in block order (deterministic)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
  // RL2 thread groups split the slabs (b = g, g + RL2, ...); 8 independent sc1 loads in flight
  // per batch, added in b order; the groups are then added in group order through LDS
  const int RL2 = kColBlock / ccols > 0 ? kColBlock / ccols : 1;
  const int cg = ccols < kColBlock ? ccols : kColBlock;
  const int gi = threadIdx.x / cg;
  float* red = sh + 1;  // after the flag word
  for (int c0 = 0; c0 < ccols; c0 += cg) {
    const int c = c0 + int(threadIdx.x % cg);
    float acc = 0.f;
    if (gi < RL2 && c < ccols) {
      for (int b0 = gi; b0 < nb; b0 += 8 * RL2) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int b = b0 + u * RL2;
          // ws is already offset by cbase; clamped address, value zeroed (no per-element branch)
          v[u] = __hip_atomic_load(ws + int64_t(b < nb ? b : b0) * cols + c, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          if (b >= nb) v[u] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
      }
    }
    __syncthreads();
    red[threadIdx.x] = acc;
    __syncthreads();
    if (gi == 0 && c < ccols) {
      float t = 0.f;
      for (int g = 0; g < RL2; ++g) t += red[g * cg + threadIdx.x];
      out[cbase + c] = t;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + by, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kColBlock) void colsum_kernel(const float* __restrict__ A, int64_t rows, int cols,
                                                        int64_t ld, float* __restrict__ ws, float* __restrict__ out,
                                                        uint32_t* __restrict__ cnt) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  colsum_block(A, rows, cols, ld, ws, out, cnt, blockIdx.x, gridDim.x, blockIdx.y, sh);
}

// Several independent colsums in ONE launch (the weight-gradient partials of a whole backward
// pass, flushed together: gasfm_amd._native.param_colsum).  The grid is the concatenation of
// the jobs' (row block x column chunk) grids; a block finds its job by block range.
constexpr int kMaxJobs = 48;
struct ColsumJob {
  const float* A;
  float* ws;
  float* out;
  int64_t rows;
  int64_t ld;
  int cols, nb, nchunk, blk0, cnt0;
};
struct ColsumJobs {
  ColsumJob j[kMaxJobs];
  int n;
};

__global__ __launch_bounds__(kColBlock) void colsum_multi_kernel(ColsumJobs a, uint32_t* __restrict__ cnt) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  int q = 0;
  while (q + 1 < a.n && int(blockIdx.x) >= a.j[q + 1].blk0) ++q;
  const ColsumJob& J = a.j[q];
  const int local = int(blockIdx.x) - J.blk0;
  colsum_block(J.A, J.rows, J.cols, J.ld, J.ws, J.out, cnt + J.cnt0, local % J.nb, J.nb, local / J.nb, sh);
}

// ---------------------------------------------------------------- tall, narrow column sums
// Column sums of a CONTIGUOUS [rows, cols] matrix with few columns and many rows (bias
// gradients over E edge rows or n point rows: [4M, 2], [200k, 64], [200k, 3]).  The matrix is
// read as a flat array: element f belongs to column f % cols.  Thread t of a block handles
// flat elements t + 256 i; with S = lcm(cols, 256) and K = S / 256 accumulators, accumulator
// i % K only ever sees column (t + 256 (i % K)) % cols, so every load is a coalesced dword
// load and no index arithmetic is per element.  Block sums: the K x 256 accumulators go to
// LDS at flat position q = t + 256 j (column q % cols) and fold by halving strides that are
// multiples of cols (fixed order).  Then the colsum hand-off: slab ws[b, cols] stored
// write-through, one ticket, and the last block folds the [nb, cols] slab with the same flat
// routine.  Deterministic; one launch.
constexpr int kTallBlock = 256;
constexpr int kTallMaxK = 8;          // lcm(cols, 256) <= 2048
constexpr int kTallMaxSlab = 16384;   // nb * cols floats the last block reads

__host__ __device__ constexpr int gcd_i(int a, int b) { return b == 0 ? a : gcd_i(b, a % b); }

__host__ __device__ inline int tall_k(int cols) { return cols / gcd_i(cols, kTallBlock); }

// flat [n] -> per-column sums in lds[0, cols); every thread returns after the block barrier.
// atomic: sc1 (agent-scope) loads for the slab written by other blocks.
template <bool kAtomic>
__device__ __forceinline__ void tall_block_sum(const float* __restrict__ A, int64_t n, int cols, int K,
                                               float* __restrict__ lds) {
  const int t = threadIdx.x;
  const int U = K * ((8 + K - 1) / K);  // loads in flight per thread, a multiple of K
  float acc[kTallMaxK];
#pragma unroll
  for (int j = 0; j < kTallMaxK; ++j) acc[j] = 0.f;
  const int64_t step = int64_t(kTallBlock) * U;
  int64_t base = 0;
  for (; base + step <= n; base += step) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (u < U) {
        const float* q = A + base + t + int64_t(kTallBlock) * u;
        v[u] = kAtomic ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (u < U) acc[u % K] += v[u];
  }
  for (int u = 0; base + t + int64_t(kTallBlock) * u < n; ++u) {
    const float* q = A + base + t + int64_t(kTallBlock) * u;
    const float x = kAtomic ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
#pragma unroll
    for (int j = 0; j < kTallMaxK; ++j)
      if (j == u % K) acc[j] += x;
  }
  const int S = kTallBlock * K;
#pragma unroll
  for (int j = 0; j < kTallMaxK; ++j)
    if (j < K) lds[t + kTallBlock * j] = acc[j];
  __syncthreads();
  for (int stride = S / 2; stride >= cols && stride % cols == 0; stride /= 2) {
    for (int i = t; i < stride; i += kTallBlock) lds[i] += lds[i + stride];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kTallBlock) void colsum_tall_kernel(const float* __restrict__ A, int64_t rows, int cols,
                                                                 float* __restrict__ ws, float* __restrict__ out,
                                                                 uint32_t* __restrict__ cnt) {
  __shared__ float lds[kTallBlock * kTallMaxK];
  __shared__ uint32_t flag;
  const int K = tall_k(cols);
  const int nb = gridDim.x, b = blockIdx.x;
  const int64_t r0 = rows * b / nb, r1 = rows * (b + 1) / nb;
  tall_block_sum<false>(A + r0 * cols, (r1 - r0) * cols, cols, K, lds);
  if (threadIdx.x < cols)
    __hip_atomic_store(ws + int64_t(b) * cols + threadIdx.x, lds[threadIdx.x], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = (tk == uint32_t(nb - 1)) ? 1u : 0u;
  }
  __syncthreads();
  if (flag == 0u) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  tall_block_sum<true>(ws, int64_t(nb) * cols, cols, K, lds);
  if (threadIdx.x < cols) out[threadIdx.x] = lds[threadIdx.x];
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int tall_blocks(int64_t rows, int cols) {
  int64_t nb = (rows * cols + 8191) / 8192;  // >= 8k floats per block
  const int64_t cap = kTallMaxSlab / cols < 1024 ? kTallMaxSlab / cols : 1024;
  if (nb > cap) nb = cap;
  return int(nb < 1 ? 1 : nb);
}


// dst = src[0] + src[1] + ... + src[n-1] (in index order; float4 per thread, grid-stride).  The
// gradient of a tensor with n consumers in ONE pass: autograd would run n-1 full-size adds.
constexpr int kMaxSumSrc = 16;
struct SumSrcs {
  const float* p[kMaxSumSrc];
};

__global__ __launch_bounds__(256) void sum_n_kernel(SumSrcs s, int n, int64_t count4, float* __restrict__ dst) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < count4; i += int64_t(gridDim.x) * 256) {
    float4 acc = reinterpret_cast<const float4*>(s.p[0])[i];
    for (int k = 1; k < n; ++k) {
      const float4 v = reinterpret_cast<const float4*>(s.p[k])[i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    reinterpret_cast<float4*>(dst)[i] = acc;
  }
}

}  // namespace gasfm

using namespace gasfm;

extern "C" int32_t gasfm_colsum_tall_ok(int32_t cols) {
  return cols > 0 && cols <= kTallBlock && tall_k(cols) <= kTallMaxK ? 1 : 0;
}

extern "C" int64_t gasfm_colsum_tall_ws_floats(int64_t rows, int32_t cols) {
  return cols > 0 ? int64_t(tall_blocks(rows, cols)) * cols : 0;
}

extern "C" int gasfm_colsum_tall(const float* A, int64_t rows, int32_t cols, float* ws, float* out,
                                 uint32_t* counter, void* stream) {
  GASFM_REQUIRE(rows >= 0 && gasfm_colsum_tall_ok(cols), "gasfm_colsum_tall: rows=%lld cols=%d",
                (long long)rows, cols);
  GASFM_REQUIRE(ws && out && counter && (rows == 0 || A), "gasfm_colsum_tall: null pointer");
  const int nb = tall_blocks(rows, cols);
  hipLaunchKernelGGL(colsum_tall_kernel, dim3(nb), dim3(kTallBlock), 0, reinterpret_cast<hipStream_t>(stream), A,
                     rows, cols, ws, out, counter);
  return launch_status("gasfm_colsum_tall");
}

extern "C" int64_t gasfm_colsum_ws_floats(int64_t rows, int32_t cols) {
  return int64_t(colsum_blocks(rows)) * cols;
}

extern "C" int32_t gasfm_colsum_counters(int32_t cols) { return (cols + kChunkCols - 1) / kChunkCols; }

extern "C" int gasfm_colsum(const float* A, int64_t rows, int32_t cols, int64_t ld, float* ws, float* out,
                            uint32_t* counters, void* stream) {
  GASFM_REQUIRE(rows >= 0 && cols > 0 && ld >= cols, "gasfm_colsum: rows=%lld cols=%d ld=%lld", (long long)rows,
                cols, (long long)ld);
  GASFM_REQUIRE(ws && out && counters && (rows == 0 || A), "gasfm_colsum: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = colsum_blocks(rows);
  const int nchunk = (cols + kChunkCols - 1) / kChunkCols;
  hipLaunchKernelGGL(colsum_kernel, dim3(nb, nchunk), dim3(kColBlock), 4 * kColBlock * sizeof(float), st, A, rows,
                     cols, ld, ws, out, counters);
  return launch_status("gasfm_colsum");
}

extern "C" int gasfm_colsum_multi(int32_t n, const float* const* A, const int64_t* rows, const int32_t* cols,
                                  const int64_t* ld, float* const* ws, float* const* out, uint32_t* counters,
                                  void* stream) {
  GASFM_REQUIRE(n >= 0, "gasfm_colsum_multi: n=%d", n);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int base = 0; base < n; base += kMaxJobs) {
    ColsumJobs a{};
    int blocks = 0, cnt = 0;
    a.n = (n - base) < kMaxJobs ? (n - base) : kMaxJobs;
    for (int k = 0; k < a.n; ++k) {
      const int i = base + k;
      GASFM_REQUIRE(rows[i] >= 0 && cols[i] > 0 && ld[i] >= cols[i] && ws[i] && out[i] && (rows[i] == 0 || A[i]),
                    "gasfm_colsum_multi: job %d rows=%lld cols=%d ld=%lld", i, (long long)rows[i], cols[i],
                    (long long)ld[i]);
      const int nb = colsum_blocks(rows[i]);
      const int nchunk = (cols[i] + kChunkCols - 1) / kChunkCols;
      a.j[k] = ColsumJob{A[i], ws[i], out[i], rows[i], ld[i], cols[i], nb, nchunk, blocks, cnt};
      blocks += nb * nchunk;
      cnt += nchunk;
    }
    if (blocks == 0) continue;
    // each launch of the batch uses counters [0, cnt): launches on one stream run in order and
    // every counter is reset by its last arriver
    hipLaunchKernelGGL(colsum_multi_kernel, dim3(blocks), dim3(kColBlock), 4 * kColBlock * sizeof(float), st, a,
                       counters);
    const int s = launch_status("gasfm_colsum_multi");
    if (s != GASFM_OK) return s;
  }
  return GASFM_OK;
}

extern "C" int32_t gasfm_colsum_multi_counters(int32_t n, const int32_t* cols) {
  int best = 0;
  for (int base = 0; base < n; base += kMaxJobs) {
    int c = 0;
    for (int i = base; i < n && i < base + kMaxJobs; ++i) c += (cols[i] + kChunkCols - 1) / kChunkCols;
    best = c > best ? c : best;
  }
  return best;
}

extern "C" int gasfm_sum_n(int32_t n, const float* const* src, int64_t count, float* dst, void* stream) {
  GASFM_REQUIRE(n >= 1 && n <= kMaxSumSrc && count >= 0 && dst && src, "gasfm_sum_n: n=%d count=%lld", n,
                (long long)count);
  GASFM_REQUIRE(count % 4 == 0 && aligned16(dst), "gasfm_sum_n: count %% 4 and 16-byte alignment required");
  SumSrcs s{};
  for (int k = 0; k < n; ++k) {
    GASFM_REQUIRE(src[k] && aligned16(src[k]), "gasfm_sum_n: source %d null or unaligned", k);
    s.p[k] = src[k];
  }
  if (count == 0) return GASFM_OK;
  const int64_t c4 = count / 4;
  const int64_t want = (c4 + 255) / 256;
  const int grid = int(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(sum_n_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, s, n, c4, dst);
  return launch_status("gasfm_sum_n");
}
