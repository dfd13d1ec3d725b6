// Deterministic column sums (bias / att gradients): two passes, no atomics.
//   pass 1: block b sums rows [b*R/B, (b+1)*R/B) of every column into ws[b, :]
//   pass 2: one block sums ws over b in order.
// Replaces the implicit reductions autograd performs for GATv2Conv.bias /
// GATv2Conv.att (PyG, layers.py:304-309 etc.) and LayerNorm/Linear biases.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace gasfm {

constexpr int kColBlock = 256;
constexpr int kMaxColBlocks = 512;

static int colsum_blocks(int64_t rows) {
  const int64_t b = (rows + 255) / 256;
  return int(b < 1 ? 1 : (b > kMaxColBlocks ? kMaxColBlocks : b));
}

// Threads of a block cover (row lane, column) pairs: with cols <= 256 the block
// walks RPB = 256/cols rows at a time so that short rows still coalesce.
__global__ __launch_bounds__(kColBlock) void colsum_pass1(const float* __restrict__ A, int64_t rows, int cols,
                                                       int64_t ld, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int nb = gridDim.x;
  const int64_t r0 = rows * blockIdx.x / nb, r1 = rows * (blockIdx.x + 1) / nb;
  if (cols <= kColBlock) {
    const int rpb = kColBlock / cols;
    const int c = threadIdx.x % cols, rr = threadIdx.x / cols;
    float acc = 0.f;
    if (rr < rpb)
      for (int64_t r = r0 + rr; r < r1; r += rpb) acc += A[r * ld + c];
    sh[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < cols) {
      float t = 0.f;
      for (int k = 0; k < rpb; ++k) t += sh[k * cols + threadIdx.x];
      ws[int64_t(blockIdx.x) * cols + threadIdx.x] = t;
    }
  } else {
    for (int c = threadIdx.x; c < cols; c += kColBlock) {
      float acc = 0.f;
      for (int64_t r = r0; r < r1; ++r) acc += A[r * ld + c];
      ws[int64_t(blockIdx.x) * cols + c] = acc;
    }
  }
}

__global__ __launch_bounds__(kColBlock) void colsum_pass2(const float* __restrict__ ws, int nb, int cols,
                                                       float* __restrict__ out) {
  for (int c = blockIdx.x * kColBlock + threadIdx.x; c < cols; c += gridDim.x * kColBlock) {
    float acc = 0.f;
    for (int b = 0; b < nb; ++b) acc += ws[int64_t(b) * cols + c];
    out[c] = acc;
  }
}

}  // namespace gasfm

using namespace gasfm;

extern "C" int64_t gasfm_colsum_ws_floats(int64_t rows, int32_t cols) {
  return int64_t(colsum_blocks(rows)) * cols;
}

extern "C" int gasfm_colsum(const float* A, int64_t rows, int32_t cols, int64_t ld, float* ws, float* out,
                            void* stream) {
  GASFM_REQUIRE(rows >= 0 && cols > 0 && ld >= cols, "gasfm_colsum: rows=%lld cols=%d ld=%lld", (long long)rows,
                cols, (long long)ld);
  GASFM_REQUIRE(ws && out && (rows == 0 || A), "gasfm_colsum: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = colsum_blocks(rows);
  hipLaunchKernelGGL(colsum_pass1, dim3(nb), dim3(kColBlock), kColBlock * sizeof(float), st, A, rows, cols, ld, ws);
  int rc = launch_status("gasfm_colsum/pass1");
  if (rc) return rc;
  const int g2 = (cols + kColBlock - 1) / kColBlock;
  hipLaunchKernelGGL(colsum_pass2, dim3(g2), dim3(kColBlock), 0, st, ws, nb, cols, out);
  return launch_status("gasfm_colsum/pass2");
}
