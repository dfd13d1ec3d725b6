// The input embedding of GraphAttnSfMNet, gfx950: P = values W^T + b with W [2 x 2]
// (reference EmbeddingLayer, code/models/layers.py:992-1015: pos_emb_n_freq = 0 and
// post_embed_proj_dim = -1, i.e. one Linear(2, 2) on the E normalised measurements,
// graph_attn_sfm.py:53).
//
// hipBLASLt runs this [E x 2] x [2 x 2] product as a GEMM tile sweep (233 us at config 4's
// E = 4M) and its weight gradient as a split-K batched GEMM + column sums (~240 us); both are
// 32-64 MB streams.  Here:
//   embed2_fwd   two rows per lane as one float4 load and one float4 store;
//   embed2_bwd   dW = dP^T values and db = colsum(dP) as six running sums per lane, an ordered
//                workgroup reduction, and one partial row of 6 per workgroup for gasfm_colsum
//                (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

constexpr int kEmbThreads = 256;
constexpr int EMB_PART = 6;  // dW00 dW01 dW10 dW11 db0 db1

__global__ __launch_bounds__(kEmbThreads) void embed2_fwd_kernel(const float* __restrict__ X, int64_t E,
                                                                 const float* __restrict__ W,
                                                                 const float* __restrict__ b, float* __restrict__ Y) {
  const float w00 = W[0], w01 = W[1], w10 = W[2], w11 = W[3], b0 = b[0], b1 = b[1];
  const int64_t pairs = E / 2, stride = int64_t(gridDim.x) * kEmbThreads;
  for (int64_t q = int64_t(blockIdx.x) * kEmbThreads + threadIdx.x; q < pairs; q += stride) {
    const float4 x = reinterpret_cast<const float4*>(X)[q];
    reinterpret_cast<float4*>(Y)[q] = make_float4(fmaf(w01, x.y, fmaf(w00, x.x, b0)), fmaf(w11, x.y, fmaf(w10, x.x, b1)),
                                                  fmaf(w01, x.w, fmaf(w00, x.z, b0)), fmaf(w11, x.w, fmaf(w10, x.z, b1)));
  }
  if ((E & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const float x0 = X[2 * (E - 1)], x1 = X[2 * (E - 1) + 1];
    Y[2 * (E - 1)] = fmaf(w01, x1, fmaf(w00, x0, b0));
    Y[2 * (E - 1) + 1] = fmaf(w11, x1, fmaf(w10, x0, b1));
  }
}

__global__ __launch_bounds__(kEmbThreads) void embed2_bwd_kernel(const float* __restrict__ X,
                                                                 const float* __restrict__ dY, int64_t E,
                                                                 float* __restrict__ part) {
  float s[EMB_PART] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t pairs = E / 2, stride = int64_t(gridDim.x) * kEmbThreads;
  for (int64_t q = int64_t(blockIdx.x) * kEmbThreads + threadIdx.x; q < pairs; q += stride) {
    const float4 x = reinterpret_cast<const float4*>(X)[q];
    const float4 d = reinterpret_cast<const float4*>(dY)[q];
    s[0] = fmaf(d.x, x.x, fmaf(d.z, x.z, s[0]));
    s[1] = fmaf(d.x, x.y, fmaf(d.z, x.w, s[1]));
    s[2] = fmaf(d.y, x.x, fmaf(d.w, x.z, s[2]));
    s[3] = fmaf(d.y, x.y, fmaf(d.w, x.w, s[3]));
    s[4] += d.x + d.z;
    s[5] += d.y + d.w;
  }
  if ((E & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const float x0 = X[2 * (E - 1)], x1 = X[2 * (E - 1) + 1], d0 = dY[2 * (E - 1)], d1 = dY[2 * (E - 1) + 1];
    s[0] = fmaf(d0, x0, s[0]);
    s[1] = fmaf(d0, x1, s[1]);
    s[2] = fmaf(d1, x0, s[2]);
    s[3] = fmaf(d1, x1, s[3]);
    s[4] += d0;
    s[5] += d1;
  }
  // lanes -> wave (fixed butterfly), waves -> workgroup in wave order
  __shared__ float red[kEmbThreads / tile::kW][EMB_PART];
  const int lane = threadIdx.x & (tile::kW - 1), wave = threadIdx.x / tile::kW;
#pragma unroll
  for (int k = 0; k < EMB_PART; ++k) {
    float v = s[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < EMB_PART) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < kEmbThreads / tile::kW; ++w) v += red[w][threadIdx.x];
    part[int64_t(blockIdx.x) * EMB_PART + threadIdx.x] = v;
  }
}

int emb_grid(const void* fn, int64_t E) {
  return resident_grid(fn, kEmbThreads, 0, E / 2 > 0 ? E / 2 : 1, kEmbThreads);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

// Partial rows of gasfm_embed2_bwd (6 floats each: dW00 dW01 dW10 dW11 db0 db1); 0 when E <= 0.
extern "C" int32_t gasfm_embed2_part_rows(int64_t E) {
  return E > 0 ? emb_grid(reinterpret_cast<const void*>(&embed2_bwd_kernel), E) : 0;
}

extern "C" int gasfm_embed2_fwd(const float* X, int64_t E, const float* W, const float* b, float* Y, void* stream) {
  GASFM_REQUIRE(E >= 0, "gasfm_embed2_fwd: E < 0");
  if (E == 0) return GASFM_OK;
  GASFM_REQUIRE(X && W && b && Y && aligned16(X) && aligned16(Y), "gasfm_embed2_fwd: bad args");
  hipLaunchKernelGGL(embed2_fwd_kernel, dim3(emb_grid(reinterpret_cast<const void*>(&embed2_fwd_kernel), E)),
                     dim3(kEmbThreads), 0, reinterpret_cast<hipStream_t>(stream), X, E, W, b, Y);
  return launch_status("gasfm_embed2_fwd");
}

extern "C" int gasfm_embed2_bwd(const float* X, const float* dY, int64_t E, float* part, void* stream) {
  GASFM_REQUIRE(E >= 0, "gasfm_embed2_bwd: E < 0");
  if (E == 0) return GASFM_OK;
  GASFM_REQUIRE(X && dY && part && aligned16(X) && aligned16(dY), "gasfm_embed2_bwd: bad args");
  hipLaunchKernelGGL(embed2_bwd_kernel, dim3(gasfm_embed2_part_rows(E)), dim3(kEmbThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), X, dY, E, part);
  return launch_status("gasfm_embed2_bwd");
}
