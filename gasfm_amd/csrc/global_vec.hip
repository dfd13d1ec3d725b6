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
constexpr int kSlab = 256;    // columns per backward workgroup (4 per lane)
constexpr int kChunk = 128;   // rows per backward workgroup (32 per wave, requested at once)
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
  rstd = rsq_normal(block_sum<nT>(q, scratch) / K + eps);
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

// One backward workgroup: columns [slab*kSlab, +kSlab) (4 per lane, float4), rows
// [chunk*kChunk, +kChunk) (kChunk/4 per wave, all of a wave's W rows requested at once):
//   dW[i, j] = dy[i] h[j];  part[chunk, j] = sum_{i in chunk} dy[i] W[i, j];  db[i] = dy[i]
// h = relu(LN(x)) (or x); the W loads are issued before the LayerNorm statistics of x so both
// latencies overlap.  Clamped in-range addresses, values zeroed: no per-load branch.
__device__ __forceinline__ void gvec_bwd_body(const float* __restrict__ dy, const float* __restrict__ x, int K,
                                              const float* __restrict__ gam, const float* __restrict__ bet,
                                              float eps, const float* __restrict__ W, int N, float* __restrict__ dW,
                                              float* __restrict__ db, float* __restrict__ part, int slab, int chunk,
                                              float* scratch, float4* red) {
  constexpr int RW = kChunk / (kT / 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = slab * kSlab + 4 * lane;
  const bool jok = j < K;
  const int jc = jok ? j : 0;
  const int i0 = chunk * kChunk + wave * RW;
  float4 w[RW];
  float d[RW];
#pragma unroll
  for (int u = 0; u < RW; ++u) {
    const int i = i0 + u;
    const int ii = i < N ? i : N - 1;
    w[u] = *reinterpret_cast<const float4*>(W + int64_t(ii) * K + jc);
    d[u] = dy[ii];
  }
  float4 h = *reinterpret_cast<const float4*>(x + jc);
  if (gam) {
    float mean, rstd;
    row_stats<kT>(x, K, eps, scratch, mean, rstd);
    const float4 g4 = *reinterpret_cast<const float4*>(gam + jc), b4 = *reinterpret_cast<const float4*>(bet + jc);
    h = make_float4(fmaxf(fmaf((h.x - mean) * rstd, g4.x, b4.x), 0.f), fmaxf(fmaf((h.y - mean) * rstd, g4.y, b4.y), 0.f),
                    fmaxf(fmaf((h.z - mean) * rstd, g4.z, b4.z), 0.f), fmaxf(fmaf((h.w - mean) * rstd, g4.w, b4.w), 0.f));
  }
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
#pragma unroll
  for (int u = 0; u < RW; ++u) {
    const int i = i0 + u;
    const float du = i < N ? d[u] : 0.f;
    if (i < N && jok)
      *reinterpret_cast<float4*>(dW + int64_t(i) * K + j) = make_float4(du * h.x, du * h.y, du * h.z, du * h.w);
    float4& a = (u & 1) ? a1 : a0;
    a.x = fmaf(du, w[u].x, a.x);
    a.y = fmaf(du, w[u].y, a.y);
    a.z = fmaf(du, w[u].z, a.z);
    a.w = fmaf(du, w[u].w, a.w);
  }
  red[wave * 64 + lane] = make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
  __syncthreads();
  if (wave == 0 && jok) {
    float4 s4 = red[lane];
#pragma unroll
    for (int q = 1; q < kT / 64; ++q) {
      const float4 r = red[q * 64 + lane];
      s4.x += r.x;
      s4.y += r.y;
      s4.z += r.z;
      s4.w += r.w;
    }
    *reinterpret_cast<float4*>(part + int64_t(chunk) * K + j) = s4;
  }
  if (db && slab == 0) {
    for (int r = threadIdx.x; r < kChunk; r += kT) {
      const int ii = chunk * kChunk + r;
      if (ii < N) db[ii] = dy[ii];
    }
  }
}

__global__ __launch_bounds__(kT) void gvec_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                      int K, const float* __restrict__ gam,
                                                      const float* __restrict__ bet, float eps,
                                                      const float* __restrict__ W, int N, float* __restrict__ dW,
                                                      float* __restrict__ db, float* __restrict__ part) {
  __shared__ float scratch[kT / 64];
  __shared__ float4 red[kT];
  gvec_bwd_body(dy, x, K, gam, bet, eps, W, N, dW, db, part, blockIdx.x, blockIdx.y, scratch, red);
}

// NV sums over the workgroup in ONE barrier round (fixed order: deterministic); scratch holds
// nT/64 x NV floats.  Results broadcast to every thread.
template <int nT, int NV>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[wave * NV + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < nT / 64; ++w) t += scratch[w * NV + k];
    v[k] = t;
  }
}

// dh[u] = sum over the nchunks partial rows of column threadIdx.x + u*kFinT (chunk order), the
// chunk loop unrolled so that its loads are in flight together
template <int PER>
__device__ __forceinline__ void sum_parts(const float* __restrict__ part, int nchunks, int K, float (&dh)[PER]) {
#pragma unroll
  for (int u = 0; u < PER; ++u) dh[u] = 0.f;
  int c = 0;
  for (; c + 4 <= nchunks; c += 4) {
    float t[4][PER];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int j = threadIdx.x + u * kFinT;
        t[q][u] = j < K ? part[int64_t(c + q) * K + j] : 0.f;
      }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int u = 0; u < PER; ++u) dh[u] += t[q][u];
  }
  for (; c < nchunks; ++c)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      dh[u] += j < K ? part[int64_t(c) * K + j] : 0.f;
    }
}

// mean / rstd of the single row x (PER values per thread already loaded): two-pass, one barrier
// round per pass
template <int PER>
__device__ __forceinline__ void row_stats_reg(const float (&xv)[PER], int K, float eps, float* scratch, float& mean,
                                              float& rstd) {
  float s[1] = {0.f};
#pragma unroll
  for (int u = 0; u < PER; ++u) s[0] += xv[u];  // out-of-range entries are 0
  block_sums<kFinT, 1>(s, scratch);
  mean = s[0] / K;
  float q[1] = {0.f};
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int j = threadIdx.x + u * kFinT;
    const float d = j < K ? xv[u] - mean : 0.f;
    q[0] = fmaf(d, d, q[0]);
  }
  block_sums<kFinT, 1>(q, scratch);
  rstd = rsq_normal(q[0] / K + eps);
}

// dh = sum_c part[c, :];  dx = LN_bwd(mask * dh) (+ dy if resid); dgamma, dbeta.  Every global
// load is issued before the first barrier; the two LayerNorm-backward row sums share one round.
__global__ __launch_bounds__(kFinT) void gvec_bwd_finish_kernel(const float* __restrict__ part, int nchunks,
                                                                int K, const float* __restrict__ x,
                                                                const float* __restrict__ gam,
                                                                const float* __restrict__ bet, float eps,
                                                                const float* __restrict__ dy, int resid,
                                                                float* __restrict__ dx, float* __restrict__ dgam,
                                                                float* __restrict__ dbet) {
  __shared__ float scratch[(kFinT / 64) * 2];
  constexpr int PER = kMaxK / kFinT;
  float dh[PER], xv[PER], gv[PER], bv[PER], rv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int j = threadIdx.x + u * kFinT;
    const bool in = j < K;
    xv[u] = in ? x[j] : 0.f;
    gv[u] = (in && gam) ? gam[j] : 0.f;
    bv[u] = (in && gam) ? bet[j] : 0.f;
    rv[u] = (in && resid) ? dy[j] : 0.f;
  }
  sum_parts<PER>(part, nchunks, K, dh);
  if (gam) {
    float mean, rstd;
    row_stats_reg<PER>(xv, K, eps, scratch, mean, rstd);
    float xh[PER], sv[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      xh[u] = (xv[u] - mean) * rstd;
      const float d = (j < K && fmaf(xh[u], gv[u], bv[u]) > 0.f) ? dh[u] : 0.f;
      if (j < K) {
        dgam[j] = d * xh[u];
        dbet[j] = d;
      }
      dh[u] = d * gv[u];  // now g = dh * gamma
      sv[0] += dh[u];
      sv[1] = fmaf(dh[u], xh[u], sv[1]);
    }
    block_sums<kFinT, 2>(sv, scratch);
    const float s1 = sv[0] / K, s2 = sv[1] / K;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      if (j < K) dx[j] = rstd * (dh[u] - s1 - xh[u] * s2) + rv[u];
    }
  } else {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      if (j < K) dx[j] = dh[u] + rv[u];
    }
  }
}


// ---------------------------------------------------------------------------- batched problems
// Several independent single-row problems in ONE launch (the global hub, model.py: the three
// LayerNorm -> Linear consumers of a block's global row, then the two lin_r rows): the grid is
// the concatenation of the per-problem grids, each workgroup finds its problem by block range.
constexpr int kMaxProb = 4;

struct GvFwdProb {
  const float* x;
  const float* gam;
  const float* bet;
  const float* W;
  const float* b;
  const float* res;
  float* y;
  int K, N, blk0;
};
struct GvFwdArgs {
  GvFwdProb p[kMaxProb];
  int nprob;
  float eps;
};

__device__ __forceinline__ int find_prob(const int (&blk0)[kMaxProb], int nprob) {
  int pi = 0;
  while (pi + 1 < nprob && int(blockIdx.x) >= blk0[pi + 1]) ++pi;
  return pi;
}

__global__ __launch_bounds__(kT) void gvec_multi_fwd_kernel(GvFwdArgs a) {
  int blk0[kMaxProb];
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) blk0[q] = a.p[q].blk0;
  const GvFwdProb& p = a.p[find_prob(blk0, a.nprob)];
  __shared__ __attribute__((aligned(16))) float h[kMaxK];
  __shared__ float scratch[kT / 64];
  const int K = p.K;
  if (p.gam) {
    float mean, rstd;
    row_stats<kT>(p.x, K, a.eps, scratch, mean, rstd);
    for (int j = threadIdx.x; j < K; j += kT) h[j] = fmaxf(fmaf((p.x[j] - mean) * rstd, p.gam[j], p.bet[j]), 0.f);
  } else {
    for (int j = threadIdx.x; j < K; j += kT) h[j] = p.x[j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = (int(blockIdx.x) - p.blk0) * (kT / 64) + wave;
  if (i >= p.N) return;
  const float* w = p.W + int64_t(i) * K;
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
  if (lane == 0) p.y[i] = acc + (p.b ? p.b[i] : 0.f) + (p.res ? p.res[i] : 0.f);
}

struct GvBwdProb {
  const float* dy;
  const float* x;
  const float* gam;
  const float* bet;
  const float* W;
  float* dW;
  float* db;
  float* part;
  int K, N, blk0, slabs;
};
struct GvBwdArgs {
  GvBwdProb p[kMaxProb];
  int nprob;
  float eps;
};

// per problem exactly gvec_bwd_kernel: dW slab, db, part[chunk, j] = sum_{i in chunk} dy[i] W[i, j]
__global__ __launch_bounds__(kT) void gvec_multi_bwd_kernel(GvBwdArgs a) {
  int blk0[kMaxProb];
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) blk0[q] = a.p[q].blk0;
  const GvBwdProb& p = a.p[find_prob(blk0, a.nprob)];
  __shared__ float scratch[kT / 64];
  __shared__ float4 red[kT];
  const int local = int(blockIdx.x) - p.blk0;
  gvec_bwd_body(p.dy, p.x, p.K, p.gam, p.bet, a.eps, p.W, p.N, p.dW, p.db, p.part, local % p.slabs,
                local / p.slabs, scratch, red);
}

// groups of problems that share the input row x: dx = dres + sum over the group's problems of
// LN_bwd(mask * sum_c part[c]) (or the plain sum when the problem has no LayerNorm); dgamma,
// dbeta per problem.  One 1024-thread workgroup per group.
struct GvFinProb {
  const float* part;
  const float* gam;
  const float* bet;
  float* dgam;
  float* dbet;
  int nchunks;
};
struct GvFinGroup {
  const float* x;
  const float* dres;
  float* dx;
  int K, p0, np;
};
struct GvFinArgs {
  GvFinProb p[kMaxProb];
  GvFinGroup g[kMaxProb];
  float eps;
};

__global__ __launch_bounds__(kFinT) void gvec_multi_finish_kernel(GvFinArgs a) {
  // every problem's partial sums, gamma / beta and the shared row x are loaded before the first
  // barrier; the LayerNorm-backward row sums of all problems of the group share one round
  __shared__ float scratch[(kFinT / 64) * 2 * kMaxProb];
  const GvFinGroup& G = a.g[blockIdx.x];
  const int K = G.K;
  constexpr int PER = kMaxK / kFinT;
  float acc[PER], xv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int j = threadIdx.x + u * kFinT;
    acc[u] = (G.dres && j < K) ? G.dres[j] : 0.f;
    xv[u] = j < K ? G.x[j] : 0.f;
  }
  float dh[kMaxProb][PER];
  bool any_ln = false;
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) {
    if (q < G.np) {
      sum_parts<PER>(a.p[G.p0 + q].part, a.p[G.p0 + q].nchunks, K, dh[q]);
      any_ln |= a.p[G.p0 + q].gam != nullptr;
    }
  }
  float mean = 0.f, rstd = 1.f;
  if (any_ln) row_stats_reg<PER>(xv, K, a.eps, scratch, mean, rstd);
  float xh[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) xh[u] = (xv[u] - mean) * rstd;
  float sv[2 * kMaxProb];
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) {
    sv[2 * q] = sv[2 * q + 1] = 0.f;
    if (q >= G.np) continue;
    const GvFinProb& P = a.p[G.p0 + q];
    if (!P.gam) {
#pragma unroll
      for (int u = 0; u < PER; ++u) acc[u] += dh[q][u];
      continue;
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = threadIdx.x + u * kFinT;
      float d = 0.f, g = 0.f;
      if (j < K) {
        g = P.gam[j];
        d = fmaf(xh[u], g, P.bet[j]) > 0.f ? dh[q][u] : 0.f;
        P.dgam[j] = d * xh[u];
        P.dbet[j] = d;
      }
      dh[q][u] = d * g;
      sv[2 * q] += dh[q][u];
      sv[2 * q + 1] = fmaf(dh[q][u], xh[u], sv[2 * q + 1]);
    }
  }
  if (any_ln) block_sums<kFinT, 2 * kMaxProb>(sv, scratch);
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) {
    if (q >= G.np || !a.p[G.p0 + q].gam) continue;
    const float s1 = sv[2 * q] / K, s2 = sv[2 * q + 1] / K;
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] += rstd * (dh[q][u] - s1 - xh[u] * s2);
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int j = threadIdx.x + u * kFinT;
    if (j < K) G.dx[j] = acc[u];
  }
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_gvec_bwd_chunks(int32_t N) { return N <= 0 ? 0 : (N + kChunk - 1) / kChunk; }

extern "C" int gasfm_gvec_fwd(const float* x, int32_t K, const float* ln_w, const float* ln_b, float eps,
                              const float* W, const float* b, int32_t N, const float* res, float* y, void* stream) {
  GASFM_REQUIRE(K > 0 && K <= kMaxK && K % 64 == 0 && N > 0, "gasfm_gvec_fwd: K=%d (multiple of 64, <= %d), N=%d",
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
  GASFM_REQUIRE(K > 0 && K <= kMaxK && K % 64 == 0 && N > 0, "gasfm_gvec_bwd: K=%d, N=%d", K, N);
  GASFM_REQUIRE(dy && x && W && dx && dW && part && (!ln_w || (ln_b && dgam && dbet)),
                "gasfm_gvec_bwd: null pointer");
  GASFM_REQUIRE(!resid || N == K, "gasfm_gvec_bwd: residual needs N == K");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int chunks = (N + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(gvec_bwd_kernel, dim3((K + kSlab - 1) / kSlab, chunks), dim3(kT), 0, st, dy, x, K, ln_w, ln_b, eps, W, N, dW, db,
                     part);
  int s = launch_status("gasfm_gvec_bwd");
  if (s != GASFM_OK) return s;
  hipLaunchKernelGGL(gvec_bwd_finish_kernel, dim3(1), dim3(kFinT), 0, st, part, chunks, K, x, ln_w, ln_b, eps, dy,
                     resid, dx, dgam, dbet);
  return launch_status("gasfm_gvec_bwd_finish");
}

static bool gv_shape_ok(int K, int N) { return K > 0 && K <= kMaxK && K % 64 == 0 && N > 0; }

extern "C" int gasfm_gvec_multi_fwd(int32_t nprob, const float* const* x, const float* const* ln_w,
                                    const float* const* ln_b, const float* const* W, const float* const* b,
                                    const float* const* res, float* const* y, const int32_t* K, const int32_t* N,
                                    float eps, void* stream) {
  GASFM_REQUIRE(nprob >= 1 && nprob <= kMaxProb, "gasfm_gvec_multi_fwd: nprob=%d", nprob);
  GvFwdArgs a{};
  a.nprob = nprob;
  a.eps = eps;
  int blocks = 0;
  for (int q = 0; q < nprob; ++q) {
    GASFM_REQUIRE(gv_shape_ok(K[q], N[q]), "gasfm_gvec_multi_fwd: problem %d K=%d N=%d", q, K[q], N[q]);
    GASFM_REQUIRE(x[q] && W[q] && y[q] && (!ln_w[q] || ln_b[q]) && aligned16(W[q]),
                  "gasfm_gvec_multi_fwd: problem %d pointers", q);
    a.p[q] = GvFwdProb{x[q], ln_w[q], ln_b[q], W[q], b[q], res[q], y[q], K[q], N[q], blocks};
    blocks += (N[q] + 3) / 4;
  }
  for (int q = nprob; q < kMaxProb; ++q) a.p[q].blk0 = blocks;
  hipLaunchKernelGGL(gvec_multi_fwd_kernel, dim3(blocks), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream), a);
  return launch_status("gasfm_gvec_multi_fwd");
}

// Backward of a batch: per problem dW (and db when given), partials part[q] of
// [gasfm_gvec_bwd_chunks(N[q]) x K[q]]; then groups of problems sharing x: group g covers
// problems [g_p0[g], g_p0[g] + g_np[g]) and writes dx[g] = dres[g] (may be null) + the sum of the
// group's LayerNorm (or plain) backward terms.
extern "C" int gasfm_gvec_multi_bwd(int32_t nprob, const float* const* dy, const float* const* x,
                                    const float* const* ln_w, const float* const* ln_b, const float* const* W,
                                    const int32_t* K, const int32_t* N, float* const* dW, float* const* db,
                                    float* const* dgam, float* const* dbet, float* const* part, int32_t ngroups,
                                    const int32_t* g_p0, const int32_t* g_np, const float* const* dres,
                                    float* const* dx, float eps, void* stream) {
  GASFM_REQUIRE(nprob >= 1 && nprob <= kMaxProb && ngroups >= 1 && ngroups <= kMaxProb,
                "gasfm_gvec_multi_bwd: nprob=%d ngroups=%d", nprob, ngroups);
  GvBwdArgs a{};
  a.nprob = nprob;
  a.eps = eps;
  GvFinArgs f{};
  f.eps = eps;
  int blocks = 0;
  for (int q = 0; q < nprob; ++q) {
    GASFM_REQUIRE(gv_shape_ok(K[q], N[q]), "gasfm_gvec_multi_bwd: problem %d K=%d N=%d", q, K[q], N[q]);
    GASFM_REQUIRE(dy[q] && x[q] && W[q] && dW[q] && part[q] && (!ln_w[q] || (ln_b[q] && dgam[q] && dbet[q])),
                  "gasfm_gvec_multi_bwd: problem %d pointers", q);
    const int slabs = (K[q] + kSlab - 1) / kSlab, chunks = (N[q] + kChunk - 1) / kChunk;
    a.p[q] = GvBwdProb{dy[q], x[q], ln_w[q], ln_b[q], W[q], dW[q], db[q], part[q], K[q], N[q], blocks, slabs};
    blocks += slabs * chunks;
    f.p[q] = GvFinProb{part[q], ln_w[q], ln_b[q], dgam[q], dbet[q], chunks};
  }
  for (int q = nprob; q < kMaxProb; ++q) a.p[q].blk0 = blocks;
  for (int gi = 0; gi < ngroups; ++gi) {
    const int p0 = g_p0[gi], np = g_np[gi];
    GASFM_REQUIRE(p0 >= 0 && np >= 1 && p0 + np <= nprob && dx[gi], "gasfm_gvec_multi_bwd: group %d", gi);
    for (int q = p0; q < p0 + np; ++q)
      GASFM_REQUIRE(x[q] == x[p0] && K[q] == K[p0], "gasfm_gvec_multi_bwd: group %d mixes inputs", gi);
    f.g[gi] = GvFinGroup{x[p0], dres[gi], dx[gi], K[p0], p0, np};
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gvec_multi_bwd_kernel, dim3(blocks), dim3(kT), 0, st, a);
  int s = launch_status("gasfm_gvec_multi_bwd");
  if (s != GASFM_OK) return s;
  hipLaunchKernelGGL(gvec_multi_finish_kernel, dim3(ngroups), dim3(kFinT), 0, st, f);
  return launch_status("gasfm_gvec_multi_finish");
}
