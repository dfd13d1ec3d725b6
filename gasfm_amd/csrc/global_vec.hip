// Single-row (global node) LayerNorm -> ReLU -> Linear (+ residual), forward and backward, gfx950.
//
// The global node of every GASFM block is ONE row of 2048 features (layers.py:497-603):
//   norm_and_proj_global2view        Lin_2048->1024(relu(LN(g)))          layers.py:497-505
//   norm_and_proj_global2scenepoint  Lin_2048->64(relu(LN(g)))            layers.py:512-520
//   view2global / scenepoint2global lin_r on those rows (1024->1024, 64->64, PyG)
//   proj_view_and_scenepoint2global  Lin_1088->2048(cat) + g             layers.py:527-528, 590-592
//   pre-MLP + skip                   x + Lin_2048->2048(relu(LN(x)))       layers.py:594-603
//   lin_global of the projection update  Lin_2048->32,nobias(relu(LN(g)))  layers.py:928-935
// aten runs each as LayerNorm + clamp + a hipBLASLt GEMM with M = 1 (+ add), and the backward
// as two GEMMs (one of them an outer product), a bias reduce and three LayerNorm kernels; the
// M = 1 GEMMs take 11-56 us where streaming the weight takes 2-3 us.  Here:
//   gvec_fwd          one wave per output row, the whole weight row streamed with 16-B loads;
//                     every workgroup recomputes LN(x) of the single row into LDS.
//   gvec_bwd          grid = (K/64 column slabs) x (row chunks of 256): each workgroup streams
//                     its W slab once, writes dW = dy (x) h for it (a 2-D outer product) and a
//                     partial of dh = W^T dy over its rows; db = dy.
//   gvec_bwd_finish   one workgroup: dh = ordered sum of the chunk partials, ReLU mask,
//                     LayerNorm backward (dx, dgamma, dbeta), + dy when the residual is x.
// No atomics: deterministic.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kT = 256;       // threads per workgroup (4 waves)
constexpr int kSlab = 64;     // columns per backward workgroup
constexpr int kChunk = 256;   // rows per backward workgroup (64 per wave)
constexpr int kMaxK = 4096;
constexpr int kFinT = 1024;   // finish kernel threads

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Sum over the workgroup (blockDim = nT threads, nT/64 waves); result broadcast to all threads.
template <int nT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < nT / 64; ++w) s += scratch[w];  // fixed order: deterministic
  return s;
}

// mean and rstd of x[0..K) (two passes over the row, each thread strided)
template <int nT>
__device__ __forceinline__ void row_stats(const float* __restrict__ x, int K, float eps, float* scratch,
                                          float& mean, float& rstd) {
  float s = 0.f;
  for (int j = threadIdx.x; j < K; j += nT) s += x[j];
  mean = block_sum<nT>(s, scratch) / K;
  float q = 0.f;
  for (int j = threadIdx.x; j < K; j += nT) {
    const float d = x[j] - mean;
    q = fmaf(d, d, q);
  }
  rstd = rsqrtf(block_sum<nT>(q, scratch) / K + eps);
}

// y[i] = W[i,:] . h + b[i] (+ res[i]);  h = relu(LN(x)) if gam else x
__global__ __launch_bounds__(kT) void gvec_fwd_kernel(const float* __restrict__ x, int K,
                                                      const float* __restrict__ gam,
                                                      const float* __restrict__ bet, float eps,
                                                      const float* __restrict__ W, const float* __restrict__ b,
                                                      const float* __restrict__ res, float* __restrict__ y, int N) {
  __shared__ __attribute__((aligned(16))) float h[kMaxK];
  __shared__ float scratch[kT / 64];
  if (gam) {
    float mean, rstd;
    row_stats<kT>(x, K, eps, scratch, mean, rstd);
    for (int j = threadIdx.x; j < K; j += kT) h[j] = fmaxf(fmaf((x[j] - mean) * rstd, gam[j], bet[j]), 0.f);
  } else {
    for (int j = threadIdx.x; j < K; j += kT) h[j] = x[j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.x * (kT / 64) + wave;
  if (i >= N) return;
  const float* w = W + int64_t(i) * K;
  float a0 = 0.f, a1 = 0.f;
  int j = lane * 4;
#pragma unroll 4
  for (; j + 256 < K; j += 512) {
    const float4 u = *reinterpret_cast<const float4*>(w + j);
    const float4 v = *reinterpret_cast<const float4*>(w + j + 256);
    const float4 hu = *reinterpret_cast<const float4*>(h + j);
    const float4 hv = *reinterpret_cast<const float4*>(h + j + 256);
    a0 = fmaf(u.x, hu.x, fmaf(u.y, hu.y, fmaf(u.z, hu.z, fmaf(u.w, hu.w, a0))));
    a1 = fmaf(v.x, hv.x, fmaf(v.y, hv.y, fmaf(v.z, hv.z, fmaf(v.w, hv.w, a1))));
  }
  if (j < K) {
    const float4 u = *reinterpret_cast<const float4*>(w + j);
    const float4 hu = *reinterpret_cast<const float4*>(h + j);
    a0 = fmaf(u.x, hu.x, fmaf(u.y, hu.y, fmaf(u.z, hu.z, fmaf(u.w, hu.w, a0))));
  }
  const float acc = wave_sum(a0 + a1);
  if (lane == 0) y[i] = acc + (b ? b[i] : 0.f) + (res ? res[i] : 0.f);
}

// dW[i, j] = dy[i] h[j];  part[chunk, j] = sum_{i in chunk} dy[i] W[i, j];  db[i] = dy[i]
__global__ __launch_bounds__(kT) void gvec_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                      int K, const float* __restrict__ gam,
                                                      const float* __restrict__ bet, float eps,
                                                      const float* __restrict__ W, int N, float* __restrict__ dW,
                                                      float* __restrict__ db, float* __restrict__ part) {
  __shared__ float scratch[kT / 64];
  __shared__ float red[kT / 64][kSlab];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * kSlab + lane;
  float hj = x[j];
  if (gam) {
    float mean, rstd;
    row_stats<kT>(x, K, eps, scratch, mean, rstd);
    hj = fmaxf(fmaf((hj - mean) * rstd, gam[j], bet[j]), 0.f);
  }
  const int i0 = blockIdx.y * kChunk + wave * (kChunk / 4);
  const int i1 = min(i0 + kChunk / 4, N);
  // 16 rows per group: all 16 loads issued before any use (memory-level parallelism)
  constexpr int G = 16;
  float a0 = 0.f, a1 = 0.f;
  for (int ib = i0; ib < i1; ib += G) {
    float w[G], d[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int i = ib + u;
      const bool live = i < i1;
      const int ii = live ? i : i0;  // in-range address; value discarded
      d[u] = live ? dy[ii] : 0.f;
      w[u] = W[int64_t(ii) * K + j];
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int i = ib + u;
      if (i < i1) dW[int64_t(i) * K + j] = d[u] * hj;
      if (u & 1)
        a1 = fmaf(d[u], w[u], a1);
      else
        a0 = fmaf(d[u], w[u], a0);
    }
  }
  red[wave][lane] = a0 + a1;
  __syncthreads();
  if (wave == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kT / 64; ++w) s += red[w][lane];
    part[int64_t(blockIdx.y) * K + j] = s;
  }
  if (db && blockIdx.x == 0) {
    for (int r = threadIdx.x; r < kChunk; r += kT) {
      const int ii = blockIdx.y * kChunk + r;
      if (ii < N) db[ii] = dy[ii];
    }
  }
}

// dh = sum_c part[c, :];  dx = LN_bwd(mask * dh) (+ dy if resid); dgamma, dbeta
__global__ __launch_bounds__(kFinT) void gvec_bwd_finish_kernel(const float* __restrict__ part, int nchunks,
                                                                int K, const float* __restrict__ x,
                                                                const float* __restrict__ gam,
                                                                const float* __restrict__ bet, float eps,
                                                                const float* __restrict__ dy, int resid,
                                                                float* __restrict__ dx, float* __restrict__ dgam,
                                                                float* __restrict__ dbet) {
  __shared__ float scratch[kFinT / 64];
  constexpr int PER = kMaxK / kFinT;
  float dh[PER], xh[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int j = threadIdx.x + u * kFinT;
    float s = 0.f;
    if (j < K)
      for (int c = 0; c < nchunks; ++c) s += part[int64_t(c) * K + j];
    dh[u] = s;
  }
  if (gam) {
    float mean, rstd;
    row_stats<kFinT>(x, K, eps, scratch, mean, rstd);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      xh[u] = 0.f;
      if (j < K) {
        xh[u] = (x[j] - mean) * rstd;
        const float d = fmaf(xh[u], gam[j], bet[j]) > 0.f ? dh[u] : 0.f;
        dgam[j] = d * xh[u];
        dbet[j] = d;
        dh[u] = d * gam[j];  // now g = dh * gamma
        s1 += dh[u];
        s2 = fmaf(dh[u], xh[u], s2);
      }
    }
    s1 = block_sum<kFinT>(s1, scratch) / K;
    s2 = block_sum<kFinT>(s2, scratch) / K;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      if (j < K) dx[j] = rstd * (dh[u] - s1 - xh[u] * s2) + (resid ? dy[j] : 0.f);
    }
  } else {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      if (j < K) dx[j] = dh[u] + (resid ? dy[j] : 0.f);
    }
  }
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_gvec_bwd_chunks(int32_t N) { return N <= 0 ? 0 : (N + kChunk - 1) / kChunk; }

extern "C" int gasfm_gvec_fwd(const float* x, int32_t K, const float* ln_w, const float* ln_b, float eps,
                              const float* W, const float* b, int32_t N, const float* res, float* y, void* stream) {
  GASFM_REQUIRE(K > 0 && K <= kMaxK && K % kSlab == 0 && N > 0, "gasfm_gvec_fwd: K=%d (multiple of 64, <= %d), N=%d",
                K, kMaxK, N);
  GASFM_REQUIRE(x && W && y && (!ln_w || ln_b), "gasfm_gvec_fwd: null pointer");
  GASFM_REQUIRE(aligned16(W), "gasfm_gvec_fwd: W not 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gvec_fwd_kernel, dim3((N + 3) / 4), dim3(kT), 0, st, x, K, ln_w, ln_b, eps, W, b, res, y, N);
  return launch_status("gasfm_gvec_fwd");
}

extern "C" int gasfm_gvec_bwd(const float* dy, const float* x, int32_t K, const float* ln_w, const float* ln_b,
                              float eps, const float* W, int32_t N, int32_t resid, float* dx, float* dW, float* db,
                              float* dgam, float* dbet, float* part, void* stream) {
  GASFM_REQUIRE(K > 0 && K <= kMaxK && K % kSlab == 0 && N > 0, "gasfm_gvec_bwd: K=%d, N=%d", K, N);
  GASFM_REQUIRE(dy && x && W && dx && dW && part && (!ln_w || (ln_b && dgam && dbet)),
                "gasfm_gvec_bwd: null pointer");
  GASFM_REQUIRE(!resid || N == K, "gasfm_gvec_bwd: residual needs N == K");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int chunks = (N + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(gvec_bwd_kernel, dim3(K / kSlab, chunks), dim3(kT), 0, st, dy, x, K, ln_w, ln_b, eps, W, N, dW, db,
                     part);
  int s = launch_status("gasfm_gvec_bwd");
  if (s != GASFM_OK) return s;
  hipLaunchKernelGGL(gvec_bwd_finish_kernel, dim3(1), dim3(kFinT), 0, st, part, chunks, K, x, ln_w, ln_b, eps, dy,
                     resid, dx, dgam, dbet);
  return launch_status("gasfm_gvec_bwd_finish");
}
