// The camera (view) side of a GASFM block for SMALL row counts, gfx950: a camera-sharded rank's
// own rows (m / W: 125 at config 4 on 8 GPUs) or a training batch's ~60 cameras.  Same
// arithmetic as view_block.hip + the D x D products (round 3: 5 view kernels + 2 GEMM launches
// forward, 6 + 4 backward per block, each ~4-10 us of latency at these sizes); here the GEMMs
// carry their prologues / epilogues and the independent pieces of a pass share one launch:
//
//   forward   vc_tail_fwd  x = prev + agg Wp^T + bp, LN, h = relu(LN(x)) for the tile's whole rows
//                          (recomputed by every column block), view[:, cols] = x + bm + h Wm^T
//             vc_hub_fwd   roles: XL[:, cols] = v Wl^T + bl | SV = relu(LN_c v) Wv^T |
//                          t = relu(LN_a v) Wa^T + ba, XR = t Wr^T + br
//   backward  vc_hub_bwd1  roles: dacc[:, cols] = dXL Wl (+ d skip) with the LayerNorm-branch row-sum
//                          partials and parameter partials of its columns | dWl = dXL^T v tiles
//             vc_hub_bwd2  d v = dacc + LN_c / LN_a backward of the two 32-wide branches
//             vc_tail_bwd1 roles: dh[:, cols] = dv Wm with its LayerNorm row-sum partials |
//                          dWm = dv^T h tiles
//             vc_tail_bwd2 dx = dv + LN backward of dh (= d prev), dWp / dbp partials, d agg =
//                          dx Wp summed over column blocks by the tile's last-arriving workgroup
// (layers.py:345-360 Proj2View tail; :928-935 lin_view; :331 the next block's
// norm_and_proj_view2proj + lin_r; :551-556 graph_conv_view2global.lin_l).
//
// A workgroup = 8 waves; a GEMM tile = 16 rows x 32 columns, the K = D reduction split over the
// 8 waves (k index 16 u + 4 g + j of lane (g = l >> 4, c = l & 15), step (u, j)) and summed in
// wave order through LDS.  Parameter gradients leave as one partial row per 16-row tile in
// view_block.hip's layouts (gasfm_view_tail_part_cols / gasfm_view_hub_part_cols) for the
// batched end-of-backward column sum.  No float atomics: deterministic.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"
#include "lanes.hpp"

namespace gasfm {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWv = 64;
constexpr int NWV = 8;               // waves per workgroup
constexpr int NT = NWV * kWv;        // 512 threads
constexpr int TR = 16;               // rows per tile
constexpr int CW = 32;               // output columns per GEMM workgroup (two 16-column MFMA tiles)
constexpr int VA = 32;               // aggregation / projection width
constexpr int MAXD = 1024;
constexpr int LDX = MAXD + 4;        // LDS row stride of a 16 x D tile
constexpr int WGT = 256;             // weight-gradient role: columns of a workgroup (8 waves x 32)

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 z4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ float f4(const float4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }

// sum over the 32 lanes of a half-wave (lanes 0-31 / 32-63 stay apart)
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

struct Tile {
  int tile, cb, ncb, col0, nrows;
  int64_t row0;
};
__device__ __forceinline__ Tile tile_of(int b, int64_t m, int D) {
  Tile t;
  t.ncb = D / CW;
  t.tile = b / t.ncb;
  t.cb = b % t.ncb;
  t.col0 = t.cb * CW;
  t.row0 = int64_t(t.tile) * TR;
  t.nrows = int(m - t.row0 < TR ? m - t.row0 : TR);
  return t;
}

// 16 x D rows (row0.., clamped to valid rows) as KU float4 per thread, and their LDS stores
template <int KU>
__device__ __forceinline__ void rows_load(const float* __restrict__ A, int64_t lda, const Tile& t, float4 (&v)[KU]) {
  constexpr int V = KU * 32;
#pragma unroll
  for (int q = 0; q < KU; ++q) {
    const int idx = int(threadIdx.x) + q * NT, r = idx / V, c4 = idx % V;
    v[q] = *reinterpret_cast<const float4*>(A + (t.row0 + (r < t.nrows ? r : 0)) * lda + 4 * c4);
  }
}
template <int KU>
__device__ __forceinline__ void rows_store(float* X, const float4 (&v)[KU]) {
  constexpr int V = KU * 32;
#pragma unroll
  for (int q = 0; q < KU; ++q) {
    const int idx = int(threadIdx.x) + q * NT, r = idx / V, c4 = idx % V;
    *reinterpret_cast<float4*>(X + r * LDX + 4 * c4) = v[q];
  }
}
// a [D] LayerNorm affine pair staged as [gamma | beta] in LDS GB (threads 0..D/4-1: gamma, D/4..D/2-1: beta)
template <int KU>
__device__ __forceinline__ float4 affine_load(const float* __restrict__ gam, const float* __restrict__ bet) {
  constexpr int D = KU * 128;
  const int t = int(threadIdx.x);
  const int tc = t < D / 2 ? t : 0;
  return *reinterpret_cast<const float4*>((tc < D / 4 ? gam : bet) + 4 * (tc % (D / 4)));
}
template <int KU>
__device__ __forceinline__ void affine_store(float* GB, const float4& v) {
  constexpr int D = KU * 128;
  if (int(threadIdx.x) < D / 2) *reinterpret_cast<float4*>(GB + 4 * threadIdx.x) = v;
}

// 16 x D rows (row0.., clamped to valid rows) into LDS X (row stride LDX), float4 loads, all
// issued before the stores
template <int KU>
__device__ __forceinline__ void rows_to_lds(const float* __restrict__ A, int64_t lda, const Tile& t, float* X) {
  constexpr int D = KU * 128, V = D / 4, PER = TR * V / NT;  // float4 per thread
  float4 v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = int(threadIdx.x) + q * NT, r = idx / V, c4 = idx % V;
    v[q] = *reinterpret_cast<const float4*>(A + (t.row0 + (r < t.nrows ? r : 0)) * lda + 4 * c4);
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = int(threadIdx.x) + q * NT, r = idx / V, c4 = idx % V;
    *reinterpret_cast<float4*>(X + r * LDX + 4 * c4) = v[q];
  }
}

// row statistics of the LDS tile: thread (row = tid >> 5, seg = tid & 31) holds the row's columns
// seg + 32 i (i < D / 32) in xs; (mean, rstd) two-pass over them
template <int KU>
__device__ __forceinline__ void tile_stats(const float* X, float eps, float (&xs)[KU * 4], float& mean, float& rstd) {
  constexpr int D = KU * 128, PER = D / 32;
  const int row = int(threadIdx.x) >> 5, seg = int(threadIdx.x) & 31;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    xs[i] = X[row * LDX + seg + 32 * i];
    s += xs[i];
  }
  mean = half_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float d = xs[i] - mean;
    q = fmaf(d, d, q);
  }
  rstd = rsq_normal(half_sum(q) / D + eps);
}

// this wave's share (K range [kw KU 16, +KU 16)) of the 16 x 32 product A (LDS tile, rows of
// length D) x B, B[k][n] = W[col0 + n][k] (x W^T) with W rows prefetched in bw
template <int KU>
__device__ __forceinline__ void gemm_lds_wt(const float* X, const float4 (&bw)[2][KU], int k0, f32x4 (&acc)[2]) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    const float4 a = *reinterpret_cast<const float4*>(X + c * LDX + k0 + 16 * u + 4 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma(f4(a, j), f4(bw[t][u], j), acc[t]);
  }
}

template <int KU>
__device__ __forceinline__ void prefetch_wt(const float* __restrict__ W, int D, int col0, int k0, float4 (&bw)[2][KU]) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < KU; ++u)
      bw[t][u] = *reinterpret_cast<const float4*>(W + int64_t(col0 + 16 * t + c) * D + k0 + 16 * u + 4 * g);
}

// the 8 waves' partial C tiles summed in wave order into wave 0's acc (RED: 8 x 2 x 4 x 64 floats)
__device__ __forceinline__ void reduce_waves(float* RED, f32x4 (&acc)[2]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) RED[((wave * 2 + t) * 4 + r) * kWv + lane] = acc[t][r];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = RED[((0 * 2 + t) * 4 + r) * kWv + lane];
#pragma unroll
        for (int w = 1; w < NWV; ++w) s += RED[((w * 2 + t) * 4 + r) * kWv + lane];
        acc[t][r] = s;
      }
  }
}

// ---------------------------------------------------------------------------------- forward
// view[:, cols] = x + bm + relu(LN(x)) Wm^T,  x = prev + agg Wp^T + bp (whole rows per workgroup)
template <int KU, bool PREV>
__global__ __launch_bounds__(NT) void vc_tail_fwd_kernel(const float* __restrict__ prev, const float* __restrict__ agg,
                                                         int64_t m, const float* __restrict__ Wp,
                                                         const float* __restrict__ bp, const float* __restrict__ gam,
                                                         const float* __restrict__ bet, float eps,
                                                         const float* __restrict__ Wm, const float* __restrict__ bm,
                                                         float* __restrict__ view, float* __restrict__ xo,
                                                         float* __restrict__ ho, float2* __restrict__ rso) {
  constexpr int D = KU * 128;
  __shared__ __attribute__((aligned(16))) float X[TR * LDX];
  __shared__ float RED[NWV * 2 * 4 * kWv];
  __shared__ float XO[TR][CW + 1];
  __shared__ __attribute__((aligned(16))) float GB[2 * MAXD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const Tile t = tile_of(blockIdx.x, m, D);
  const int k0 = wave * KU * 16;
  // every load in the order of use (vmcnt counts in issue order: waiting for the prologue's
  // operands must not wait for the GEMM's W slab, requested last): prev rows, agg, the prologue's
  // Wp rows and bias, the LayerNorm affine, then Wm
  float4 pv[KU];
  if (PREV) rows_load<KU>(prev, D, t, pv);
  float4 ag[2];
  {
    const int64_t r = t.row0 + (c < t.nrows ? c : 0);
    ag[0] = *reinterpret_cast<const float4*>(agg + r * VA + 4 * g);
    ag[1] = *reinterpret_cast<const float4*>(agg + r * VA + 16 + 4 * g);
  }
  float4 wp[KU][2];
  float bpv[KU];
#pragma unroll
  for (int q = 0; q < KU; ++q) {  // D / 16 column tiles over 8 waves: wave w owns tiles w, w + 8, ...
    const int col = (wave + NWV * q) * 16 + c;
    wp[q][0] = *reinterpret_cast<const float4*>(Wp + col * VA + 4 * g);
    wp[q][1] = *reinterpret_cast<const float4*>(Wp + col * VA + 16 + 4 * g);
    bpv[q] = bp[col];
  }
  const float4 gb = affine_load<KU>(gam, bet);
  float4 bw[2][KU];
  prefetch_wt<KU>(Wm, D, t.col0, k0, bw);
  if (PREV) rows_store<KU>(X, pv);
  affine_store<KU>(GB, gb);
  __syncthreads();
  // x = prev + agg Wp^T + bp over the tile's whole rows
#pragma unroll
  for (int q = 0; q < KU; ++q) {
    const int col = (wave + NWV * q) * 16 + c;
    f32x4 xa = z4();
#pragma unroll
    for (int j = 0; j < 4; ++j) xa = mfma(f4(ag[0], j), f4(wp[q][0], j), xa);
#pragma unroll
    for (int j = 0; j < 4; ++j) xa = mfma(f4(ag[1], j), f4(wp[q][1], j), xa);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* d = X + (4 * g + r) * LDX + col;
      *d = xa[r] + bpv[q] + (PREV ? *d : 0.f);
    }
  }
  __syncthreads();
  // LayerNorm of the whole rows; the tile's own columns of x kept; h in place
  float xs[KU * 4], mean, rstd;
  tile_stats<KU>(X, eps, xs, mean, rstd);
  const int row = int(threadIdx.x) >> 5, seg = int(threadIdx.x) & 31;
  {
    const float xown = xs[t.cb];  // column col0 + seg
    XO[row][seg] = xown;
    const float hown = fmaxf(fmaf((xown - mean) * rstd, GB[t.col0 + seg], GB[D + t.col0 + seg]), 0.f);
    if (row < t.nrows) {
      xo[(t.row0 + row) * D + t.col0 + seg] = xown;
      ho[(t.row0 + row) * D + t.col0 + seg] = hown;
      if (t.cb == 0 && seg == 0) rso[t.row0 + row] = make_float2(mean, rstd);
    }
  }
#pragma unroll
  for (int i = 0; i < KU * 4; ++i) {
    const int col = seg + 32 * i;
    X[row * LDX + col] = fmaxf(fmaf((xs[i] - mean) * rstd, GB[col], GB[D + col]), 0.f);
  }
  __syncthreads();
  f32x4 acc[2] = {z4(), z4()};
  gemm_lds_wt<KU>(X, bw, k0, acc);
  reduce_waves(RED, acc);
  if (wave != 0) return;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int cl = 16 * tt + c, col = t.col0 + cl;
    const float b = bm[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      if (rr < t.nrows) view[(t.row0 + rr) * D + col] = acc[tt][r] + b + XO[rr][cl];
    }
  }
}

// roles (blockIdx): [0, T ncb) XL[:, cols] = v Wl^T + bl; [T ncb, + T) SV = relu(LN_c v) Wv^T (and
// the row statistics); [.. + T, + 2T) t = relu(LN_a v) Wa^T + ba, XR = t Wr^T + br
template <int KU>
__global__ __launch_bounds__(NT) void vc_hub_fwd_kernel(const float* __restrict__ v, int64_t m, float eps,
                                                        const float* __restrict__ Wl, const float* __restrict__ bl,
                                                        const float* __restrict__ gC, const float* __restrict__ bC,
                                                        const float* __restrict__ Wv, const float* __restrict__ gA,
                                                        const float* __restrict__ bA, const float* __restrict__ Wa,
                                                        const float* __restrict__ ba, const float* __restrict__ Wr,
                                                        const float* __restrict__ br, float* __restrict__ XL,
                                                        float* __restrict__ sv, float* __restrict__ to,
                                                        float* __restrict__ xr, int ldo, float2* __restrict__ rso) {
  constexpr int D = KU * 128;
  __shared__ __attribute__((aligned(16))) float X[TR * LDX];
  __shared__ float RED[NWV * 2 * 4 * kWv];
  __shared__ float Tt[TR][VA + 2];
  __shared__ __attribute__((aligned(16))) float GB[2 * MAXD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int ncb = D / CW, T = int((m + TR - 1) / TR);
  const int b = blockIdx.x;
  const int k0 = wave * KU * 16;
  float4 bw[2][KU];
  if (b < T * ncb) {  // ---- XL = v Wl^T + bl
    const Tile t = tile_of(b, m, D);
    float4 vr[KU];
    rows_load<KU>(v, D, t, vr);  // before the W slab: waiting for the rows does not wait for it
    prefetch_wt<KU>(Wl, D, t.col0, k0, bw);
    rows_store<KU>(X, vr);
    __syncthreads();
    f32x4 acc[2] = {z4(), z4()};
    gemm_lds_wt<KU>(X, bw, k0, acc);
    reduce_waves(RED, acc);
    if (wave != 0) return;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int col = t.col0 + 16 * tt + c;
      const float bb = bl[col];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < t.nrows) XL[(t.row0 + 4 * g + r) * D + col] = acc[tt][r] + bb;
    }
    return;
  }
  const bool branch_a = b >= T * ncb + T;  // t / XR role
  const Tile t = tile_of((b - T * ncb - (branch_a ? T : 0)) * ncb, m, D);
  float4 vr[KU];
  rows_load<KU>(v, D, t, vr);
  const float4 gbv = affine_load<KU>(branch_a ? gA : gC, branch_a ? bA : bC);
  prefetch_wt<KU>(branch_a ? Wa : Wv, D, 0, k0, bw);
  rows_store<KU>(X, vr);
  affine_store<KU>(GB, gbv);
  __syncthreads();
  float xs[KU * 4], mean, rstd;
  tile_stats<KU>(X, eps, xs, mean, rstd);
  const int row = int(threadIdx.x) >> 5, seg = int(threadIdx.x) & 31;
  if (!branch_a && seg == 0 && row < t.nrows) rso[t.row0 + row] = make_float2(mean, rstd);
#pragma unroll
  for (int i = 0; i < KU * 4; ++i) {
    const int col = seg + 32 * i;
    X[row * LDX + col] = fmaxf(fmaf((xs[i] - mean) * rstd, GB[col], GB[D + col]), 0.f);
  }
  __syncthreads();
  f32x4 acc[2] = {z4(), z4()};
  gemm_lds_wt<KU>(X, bw, k0, acc);
  reduce_waves(RED, acc);
  if (wave != 0) return;
  if (!branch_a) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < t.nrows) sv[(t.row0 + 4 * g + r) * ldo + 16 * tt + c] = acc[tt][r];
    return;
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const float bv = ba[16 * tt + c];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float tv = acc[tt][r] + bv;
      Tt[4 * g + r][16 * tt + c] = tv;
      if (4 * g + r < t.nrows) to[(t.row0 + 4 * g + r) * VA + 16 * tt + c] = tv;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  f32x4 ax[2] = {z4(), z4()};
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = Tt[c][4 * q + g];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) ax[tt] = mfma(a, Wr[(16 * tt + c) * VA + 4 * q + g], ax[tt]);
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const float bv = br[16 * tt + c];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < t.nrows) xr[(t.row0 + 4 * g + r) * ldo + 16 * tt + c] = ax[tt][r] + bv;
  }
}

// --------------------------------------------------------------------------------- backward
// weight-gradient role: C[I, J] = A[K, I]^T B[K, J] (K = m rows <= 256, A, B row-major with
// strides lda, ldb); a workgroup = 16 rows of C x 256 columns (8 waves x 32); every operand load
// issued before the first MFMA (rows past K read as 0)
template <int KQ>  // ceil(K / 16)
__device__ __forceinline__ void wgrad_tile(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                           int64_t ldb, int K, int i0, int j0, float* __restrict__ C, int64_t ldc) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  float a4[KQ][4], b4[KQ][2][4];
#pragma unroll
  for (int u = 0; u < KQ; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * u + 4 * g + j;
      const int kk = k < K ? k : K - 1;
      a4[u][j] = A[int64_t(kk) * lda + i0 + c];
      b4[u][0][j] = B[int64_t(kk) * ldb + j0 + c];
      b4[u][1][j] = B[int64_t(kk) * ldb + j0 + 16 + c];
    }
  f32x4 acc[2] = {z4(), z4()};
#pragma unroll
  for (int u = 0; u < KQ; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = 16 * u + 4 * g + j < K ? a4[u][j] : 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma(a, b4[u][t][j], acc[t]);
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) C[int64_t(i0 + 4 * g + r) * ldc + j0 + 16 * t + c] = acc[t][r];
}

// the A-in-global, B = W[k][col0 + n] (dy W) form: this wave's K share of dy[tile rows] W[:, cols]
template <int KU>
__device__ __forceinline__ void gemm_gw(const float* __restrict__ A, int64_t lda, const Tile& t,
                                        const float* __restrict__ W, int D, int k0, f32x4 (&acc)[2]) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const float* ap = A + (t.row0 + (c < t.nrows ? c : 0)) * lda + k0 + 4 * g;
  float4 av[KU];
  float bv[KU][4][2];
#pragma unroll
  for (int u = 0; u < KU; ++u) av[u] = *reinterpret_cast<const float4*>(ap + 16 * u);
#pragma unroll
  for (int u = 0; u < KU; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* bp = W + int64_t(k0 + 16 * u + 4 * g + j) * D + t.col0 + c;
      bv[u][j][0] = bp[0];
      bv[u][j][1] = bp[16];
    }
#pragma unroll
  for (int u = 0; u < KU; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) acc[tt] = mfma(f4(av[u], j), bv[u][j][tt], acc[tt]);
}

// hub partial-row layout (per tile): view_block.hip's HubPart
struct HubPart {
  int64_t WV, WA, GC, BC, GA, BA, BL, WR, BAB, BR, cols;
  __device__ __host__ explicit HubPart(int D)
      : WV(0), WA(int64_t(VA) * D), GC(2 * int64_t(VA) * D), BC(GC + D), GA(BC + D), BA(GA + D), BL(BA + D),
        WR(BL + D), BAB(WR + VA * VA), BR(BAB + VA), cols(BR + VA) {}
};

// dt = dxr Wr for the tile (16 x 32, C layout of wave w) into LDS DT[16][VA + 2]
__device__ __forceinline__ void tile_dt(const float* __restrict__ dxr, const float* __restrict__ Wr, const Tile& t,
                                        float (*DT)[VA + 2]) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int64_t r = t.row0 + (c < t.nrows ? c : 0);
  f32x4 d2[2] = {z4(), z4()};
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = c < t.nrows ? dxr[r * VA + 4 * q + g] : 0.f;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) d2[tt] = mfma(a, Wr[(4 * q + g) * VA + 16 * tt + c], d2[tt]);
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) DT[4 * g + r2][16 * tt + c] = d2[tt][r2];
}

// roles: [0, T ncb) dacc[:, cols] = dXL Wl (+ dres); [T ncb, + T ncb / 4) the LayerNorm-branch
// work of 4 column blocks (wave w: block 4 q + w / 2, branch c (w even: dsv, Wv) or a (w odd:
// dt = dxr Wr, Wa)): row-sum partials RSUM[row][cb] and the tile's parameter partials;
// [.., + D/16 x D/WGT) dWl = dXL^T v.  The three roles share nothing: they run side by side.
template <int KU, int KQ>
__global__ __launch_bounds__(NT) void vc_hub_bwd1_kernel(
    const float* __restrict__ v, const float2* __restrict__ rsv, int64_t m, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ Wv, const float* __restrict__ gA,
    const float* __restrict__ bA, const float* __restrict__ Wa, const float* __restrict__ t_in,
    const float* __restrict__ Wr, const float* __restrict__ Wl, const float* __restrict__ dsv,
    const float* __restrict__ dxr, const float* __restrict__ dxl, const float* __restrict__ dres,
    float* __restrict__ dacc, float* __restrict__ dWl, float4* __restrict__ RSUM, float* __restrict__ part) {
  constexpr int D = KU * 128;
  __shared__ float RED[NWV * 2 * 4 * kWv];
  __shared__ float SB[NWV][TR][VA + 2];  // per wave: its branch's 16 x 32 left operand (dsv or dt)
  __shared__ float HB[NWV][TR * CW];     // per wave: relu(LN_b v) rows of its columns
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int ncb = D / CW, T = int((m + TR - 1) / TR);
  const int b = blockIdx.x;
  if (b >= T * ncb + T * (ncb / 4)) {  // ---- dWl[o][i] = sum_r dXL[r][o] v[r][i]
    const int q = b - T * ncb - T * (ncb / 4), nwj = D / WGT;
    const int i0 = (q / nwj) * TR, j0 = (q % nwj) * WGT + wave * CW;
    wgrad_tile<KQ>(dxl, D, v, D, int(m), i0, j0, dWl, D);
    return;
  }
  if (b < T * ncb) {  // ---- dacc = dXL Wl (+ dres)
    const Tile t = tile_of(b, m, D);
    const int k0 = wave * KU * 16;
    float dr[2][4];
    if (wave == 0) {  // the epilogue's d skip rows, requested before the product
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = 4 * g + r;
          dr[tt][r] = dres ? dres[(t.row0 + (rr < t.nrows ? rr : 0)) * D + t.col0 + 16 * tt + c] : 0.f;
        }
    }
    f32x4 acc[2] = {z4(), z4()};
    gemm_gw<KU>(dxl, D, t, Wl, D, k0, acc);
    reduce_waves(RED, acc);
    if (wave != 0) return;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 4 * g + r;
        if (rr < t.nrows) dacc[(t.row0 + rr) * D + t.col0 + 16 * tt + c] = acc[tt][r] + dr[tt][r];
      }
    return;
  }
  // ---- branch work
  const int q0 = b - T * ncb;
  const int tile = q0 / (ncb / 4);
  const int cb = (q0 % (ncb / 4)) * 4 + (wave >> 1);
  const bool ba_ = wave & 1;
  const Tile t = tile_of(tile * ncb + cb, m, D);
  const HubPart P(D);
  float* out = part + int64_t(t.tile) * P.cols;
  // every load first (clamped rows; masked where consumed)
  float sl[4][2], wrv[VA / 4][2], wbv[VA / 4][2], vv[2][4], dlv[2][4], gg[2], bb[2];
  float2 st[4];
  const float* Wb = ba_ ? Wa : Wv;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = 4 * g + r;
    const int64_t rw = t.row0 + (rr < t.nrows ? rr : 0);
    st[r] = rsv[rw];
    // branch c: the dsv rows; branch a: the dxr rows (dt = dxr Wr below)
    const float* src = ba_ ? dxr : dsv;
    sl[r][0] = src[rw * VA + c];
    sl[r][1] = src[rw * VA + 16 + c];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      vv[tt][r] = v[rw * D + t.col0 + 16 * tt + c];
      dlv[tt][r] = ba_ ? 0.f : dxl[rw * D + t.col0 + 16 * tt + c];
    }
  }
#pragma unroll
  for (int q = 0; q < VA / 4; ++q)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      wbv[q][tt] = Wb[(4 * q + g) * D + t.col0 + 16 * tt + c];
      wrv[q][tt] = ba_ ? Wr[(4 * q + g) * VA + 16 * tt + c] : 0.f;
    }
  const float* gptr = ba_ ? gA : gC;
  const float* bptr = ba_ ? bA : bC;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    gg[tt] = gptr[t.col0 + 16 * tt + c];
    bb[tt] = bptr[t.col0 + 16 * tt + c];
  }
  float(*S)[VA + 2] = SB[wave];
  // the branch's left operand rows in LDS (zero past nrows)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = 4 * g + r;
    S[rr][c] = rr < t.nrows ? sl[r][0] : 0.f;
    S[rr][16 + c] = rr < t.nrows ? sl[r][1] : 0.f;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (ba_) {  // dt = dxr Wr (C layout) replaces the dxr rows
    f32x4 d2[2] = {z4(), z4()};
#pragma unroll
    for (int q = 0; q < VA / 4; ++q) {
      const float a = S[c][4 * q + g];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) d2[tt] = mfma(a, wrv[q][tt], d2[tt]);
    }
    if (t.cb == 0) {  // dWr = dxr^T t, dbr = sum dxr (the dxr rows still in S)
      float tv[4][2];
#pragma unroll
      for (int q = 0; q < TR / 4; ++q) {
        const int rr = 4 * q + g;
        const int64_t rw = t.row0 + (rr < t.nrows ? rr : 0);
        tv[q][0] = rr < t.nrows ? t_in[rw * VA + c] : 0.f;
        tv[q][1] = rr < t.nrows ? t_in[rw * VA + 16 + c] : 0.f;
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f32x4 wr[2] = {z4(), z4()};
#pragma unroll
        for (int q = 0; q < TR / 4; ++q) {
          const float a = S[4 * q + g][16 * mt + c];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) wr[tt] = mfma(a, tv[q][tt], wr[tt]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) out[P.WR + (16 * mt + 4 * g + r) * VA + 16 * tt + c] = wr[tt][r];
      }
      if (lane < VA) {
        float sr = 0.f;
#pragma unroll
        for (int rr = 0; rr < TR; ++rr) sr += S[rr][lane];
        out[P.BR + lane] = sr;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[4 * g + r][16 * tt + c] = d2[tt][r];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (t.cb == 0 && lane < VA) {
      float sa = 0.f;
#pragma unroll
      for (int rr = 0; rr < TR; ++rr) sa += S[rr][lane];
      out[P.BAB + lane] = sa;
    }
  }
  // dh[r][col] = sum_n S[r][n] Wb[n][col]  (C layout: rows 4g + r, column c of tile tt)
  f32x4 dh[2] = {z4(), z4()};
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = S[c][4 * q + g];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) dh[tt] = mfma(a, wbv[q][tt], dh[tt]);
  }
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  float dgp[2] = {0.f, 0.f}, dbp[2] = {0.f, 0.f}, dlp[2] = {0.f, 0.f};
  float* H = HB[wave];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      const bool live = rr < t.nrows;
      const float xh = (vv[tt][r] - st[r].x) * st[r].y;
      const float pre = fmaf(xh, gg[tt], bb[tt]);
      const float dy = (live && pre > 0.f) ? dh[tt][r] : 0.f;
      H[rr * CW + 16 * tt + c] = live ? fmaxf(pre, 0.f) : 0.f;
      dgp[tt] = fmaf(dy, xh, dgp[tt]);
      dbp[tt] += dy;
      s1[r] = fmaf(dy, gg[tt], s1[r]);
      s2[r] = fmaf(dy * gg[tt], xh, s2[r]);
      dlp[tt] += live ? dlv[tt][r] : 0.f;
    }
  }
  // row partial sums over the 32 columns (16 lanes c, 2 tiles) -> RSUM[row][cb], branch c in
  // (x, y), branch a in (z, w)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a1 = s1[r], a2 = s2[r];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      a1 += __shfl_xor(a1, o);
      a2 += __shfl_xor(a2, o);
    }
    const int rr = 4 * g + r;
    if (c == 0 && rr < t.nrows)
      reinterpret_cast<float2*>(RSUM + (t.row0 + rr) * ncb + t.cb)[ba_ ? 1 : 0] = make_float2(a1, a2);
  }
  // column partials over the tile rows (4 lane groups)
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    float a = dgp[tt], bsum = dbp[tt], l = dlp[tt];
    a = xsum32(xsum16(a));
    bsum = xsum32(xsum16(bsum));
    l = xsum32(xsum16(l));
    if (g == 0) {
      const int col = t.col0 + 16 * tt + c;
      out[(ba_ ? P.GA : P.GC) + col] = a;
      out[(ba_ ? P.BA : P.BC) + col] = bsum;
      if (!ba_) out[P.BL + col] = l;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // dW_b[n][col] = sum_r S[r][n] relu(LN_b v)[r][col]: A[i = n][k = r] = S[r][n], B[k = r][j] = h
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x4 w2[2] = {z4(), z4()};
#pragma unroll
    for (int q = 0; q < TR / 4; ++q) {
      const float a = S[4 * q + g][16 * mt + c];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) w2[tt] = mfma(a, H[(4 * q + g) * CW + 16 * tt + c], w2[tt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
        out[(ba_ ? P.WA : P.WV) + int64_t(16 * mt + 4 * g + r) * D + t.col0 + 16 * tt + c] = w2[tt][r];
  }
}

// d v[:, cols] = dacc + rstd (gv_c - S1c - x_hat S2c) + rstd (gv_a - S1a - x_hat S2a), in place on
// dacc; S = (sum over column blocks of RSUM) / D; gv_b = relu'(LN_b v) (S_b W_b)[:, cols] gamma_b.
// One workgroup (4 waves) per (tile, 64 columns): wave = (column half, branch ... ) -- each wave
// one 16 x 16 column tile of the 32-column block of its half
template <int KU>
__global__ __launch_bounds__(256) void vc_hub_bwd2_kernel(
    const float* __restrict__ v, const float2* __restrict__ rsv, int64_t m, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ Wv, const float* __restrict__ gA,
    const float* __restrict__ bA, const float* __restrict__ Wa, const float* __restrict__ Wr,
    const float* __restrict__ dsv, const float* __restrict__ dxr, const float4* __restrict__ RSUM,
    float* __restrict__ dacc) {
  constexpr int D = KU * 128;
  __shared__ float DT[TR][VA + 2], SD[TR][VA + 2];
  __shared__ float4 SM[TR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int ncb = D / CW;
  const int64_t row0 = int64_t(blockIdx.x / (D / 64)) * TR;
  const int nrows = int(m - row0 < TR ? m - row0 : TR);
  const int col = (blockIdx.x % (D / 64)) * 64 + wave * 16 + c;
  Tile t;
  t.row0 = row0;
  t.nrows = nrows;
  if (wave == 0) tile_dt(dxr, Wr, t, DT);
  if (wave == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      const int64_t rw = row0 + (rr < nrows ? rr : 0);
      SD[rr][c] = rr < nrows ? dsv[rw * VA + c] : 0.f;
      SD[rr][16 + c] = rr < nrows ? dsv[rw * VA + 16 + c] : 0.f;
    }
  }
  if (wave == 2 && lane < TR) {
    float4 a4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane < nrows)
      for (int q = 0; q < ncb; ++q) {
        const float4 p = RSUM[(row0 + lane) * ncb + q];
        a4.x += p.x;
        a4.y += p.y;
        a4.z += p.z;
        a4.w += p.w;
      }
    SM[lane] = make_float4(a4.x / D, a4.y / D, a4.z / D, a4.w / D);
  }
  __syncthreads();
  f32x4 dhc = z4(), dha = z4();
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    dhc = mfma(SD[c][4 * q + g], Wv[(4 * q + g) * D + col], dhc);
    dha = mfma(DT[c][4 * q + g], Wa[(4 * q + g) * D + col], dha);
  }
  const float gc = gC[col], bc = bC[col], ga = gA[col], bav = bA[col];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = 4 * g + r;
    if (rr >= nrows) continue;
    const float2 st = rsv[row0 + rr];
    const float4 sm = SM[rr];
    const int64_t o = (row0 + rr) * D + col;
    const float xh = (v[o] - st.x) * st.y;
    const float gvc = (fmaf(xh, gc, bc) > 0.f ? dhc[r] : 0.f) * gc;
    const float gva = (fmaf(xh, ga, bav) > 0.f ? dha[r] : 0.f) * ga;
    dacc[o] += st.y * (gvc - sm.x - xh * sm.y) + st.y * (gva - sm.z - xh * sm.w);
  }
}

// tail part-row layout (per tile): view_block.hip's [dWp (D x 32) | dbp | dgamma | dbeta | dbm]
__device__ __forceinline__ int64_t tail_cols(int D) { return int64_t(D) * VA + 4 * D; }

// roles: [0, T ncb) dh[:, cols] = dv Wm, the LayerNorm-backward row-sum partials of the columns
// (RSUMT[row][cb] = (sum gv, sum gv x_hat), gv = relu'(LN x) dh gamma) and the tile's dgamma /
// dbeta / dbm column partials; [T ncb, + D/16 x D/WGT) dWm = dv^T h
template <int KU, int KQ>
__global__ __launch_bounds__(NT) void vc_tail_bwd1_kernel(const float* __restrict__ dv, const float* __restrict__ x,
                                                          const float* __restrict__ h, const float2* __restrict__ rsx,
                                                          int64_t m, const float* __restrict__ gam,
                                                          const float* __restrict__ bet, const float* __restrict__ Wm,
                                                          float* __restrict__ dh, float* __restrict__ dWm,
                                                          float2* __restrict__ RSUMT, float* __restrict__ part) {
  constexpr int D = KU * 128;
  __shared__ float RED[NWV * 2 * 4 * kWv];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int ncb = D / CW, T = int((m + TR - 1) / TR);
  const int b = blockIdx.x;
  if (b >= T * ncb) {  // ---- dWm[o][i] = sum_r dv[r][o] h[r][i]
    const int q = b - T * ncb, nwj = D / WGT;
    wgrad_tile<KQ>(dv, D, h, D, int(m), (q / nwj) * TR, (q % nwj) * WGT + wave * CW, dWm, D);
    return;
  }
  const Tile t = tile_of(b, m, D);
  const int k0 = wave * KU * 16;
  // wave 0's epilogue operands, requested before the product
  float xv[2][4], dvv[2][4], gv2[2], bv2[2];
  float2 st[4];
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) st[r] = rsx[t.row0 + (4 * g + r < t.nrows ? 4 * g + r : 0)];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int col = t.col0 + 16 * tt + c;
      gv2[tt] = gam[col];
      bv2[tt] = bet[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t o = (t.row0 + (4 * g + r < t.nrows ? 4 * g + r : 0)) * D + col;
        xv[tt][r] = x[o];
        dvv[tt][r] = dv[o];
      }
    }
  }
  f32x4 acc[2] = {z4(), z4()};
  gemm_gw<KU>(dv, D, t, Wm, D, k0, acc);
  reduce_waves(RED, acc);
  if (wave != 0) return;
  float* out = part + int64_t(t.tile) * tail_cols(D);
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int col = t.col0 + 16 * tt + c;
    const float gv = gv2[tt], bv = bv2[tt];
    float dgp = 0.f, dbp = 0.f, dmp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      const bool live = rr < t.nrows;
      const float xh = (xv[tt][r] - st[r].x) * st[r].y;
      const float d = acc[tt][r];
      if (live) dh[(t.row0 + rr) * D + col] = d;
      const float dy = (live && fmaf(xh, gv, bv) > 0.f) ? d : 0.f;
      dgp = fmaf(dy, xh, dgp);
      dbp += dy;
      dmp += live ? dvv[tt][r] : 0.f;
      s1[r] = fmaf(dy, gv, s1[r]);
      s2[r] = fmaf(dy * gv, xh, s2[r]);
    }
    dgp = xsum32(xsum16(dgp));
    dbp = xsum32(xsum16(dbp));
    dmp = xsum32(xsum16(dmp));
    if (g == 0) {
      out[int64_t(D) * VA + D + col] = dgp;
      out[int64_t(D) * VA + 2 * D + col] = dbp;
      out[int64_t(D) * VA + 3 * D + col] = dmp;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a1 = s1[r], a2 = s2[r];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      a1 += __shfl_xor(a1, o);
      a2 += __shfl_xor(a2, o);
    }
    const int rr = 4 * g + r;
    if (c == 0 && rr < t.nrows) RSUMT[(t.row0 + rr) * ncb + t.cb] = make_float2(a1, a2);
  }
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// dx[:, cols] = dv + rstd (gv - S1 - x_hat S2) (= d prev), the tile's dWp / dbp column partials,
// and d agg = dx Wp.  A workgroup (4 waves) per (tile, 128 columns), wave w one 32-column block;
// the waves' d agg partials are summed in LDS (wave order), the group partial handed to the tile's
// last-arriving workgroup (write-through stores, one ticket), which sums the groups in order.
// Every global load of a phase is issued before its first use (clamped rows, masked where used).
constexpr int TB2_T = 256, TB2_W = TB2_T / kWv, TB2_COLS = TB2_W * CW;
__global__ __launch_bounds__(TB2_T) void vc_tail_bwd2_kernel(const float* __restrict__ dv, const float* __restrict__ dh,
                                                             const float* __restrict__ x,
                                                             const float2* __restrict__ rsx,
                                                             const float* __restrict__ agg, int64_t m, int D,
                                                             const float* __restrict__ gam,
                                                             const float* __restrict__ bet,
                                                             const float* __restrict__ Wp,
                                                             const float2* __restrict__ RSUMT, float* __restrict__ dx,
                                                             float* __restrict__ dagg, float* __restrict__ ws,
                                                             uint32_t* __restrict__ cnt, float* __restrict__ part) {
  __shared__ float DX[TB2_W][TR][CW + 1], AG[TR][VA + 1], DA[TB2_W][TR * VA];
  __shared__ float S1[TR], S2[TR];
  __shared__ uint32_t flag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int ncb = D / CW, ngrp = D / TB2_COLS;
  const int tile = blockIdx.x / ngrp, grp = blockIdx.x % ngrp;
  const int64_t row0 = int64_t(tile) * TR;
  const int nrows = int(m - row0 < TR ? m - row0 : TR);
  const int col0 = grp * TB2_COLS + wave * CW;
  float* out = part + int64_t(tile) * tail_cols(D);
  // ---- every load first
  float xv[2][4], hv[2][4], dvv[2][4], gv[2], bv[2];
  float2 st[4];
  float wpv[CW / 4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r) st[r] = rsx[row0 + (4 * g + r < nrows ? 4 * g + r : 0)];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int col = col0 + 16 * tt + c;
    gv[tt] = gam[col];
    bv[tt] = bet[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t e = (row0 + (4 * g + r < nrows ? 4 * g + r : 0)) * D + col;
      xv[tt][r] = x[e];
      hv[tt][r] = dh[e];
      dvv[tt][r] = dv[e];
    }
  }
#pragma unroll
  for (int q = 0; q < CW / 4; ++q)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) wpv[q][tt] = Wp[(col0 + 4 * q + g) * VA + 16 * tt + c];
  {  // row sums of the LayerNorm backward: thread (row = tid >> 4, k = tid & 15) sums blocks k, k + 16, ..
    const int row = int(threadIdx.x) >> 4, k = int(threadIdx.x) & 15;
    const int64_t rw = row0 + (row < nrows ? row : 0);
    float a = 0.f, b = 0.f;
    for (int q = k; q < ncb; q += 16) {
      const float2 p = RSUMT[rw * ncb + q];
      a += p.x;
      b += p.y;
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      a += __shfl_xor(a, o);
      b += __shfl_xor(b, o);
    }
    if (k == 0) {
      S1[row] = a / D;
      S2[row] = b / D;
    }
  }
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      const int64_t rw = row0 + (rr < nrows ? rr : 0);
      const float a0 = agg[rw * VA + c], a1 = agg[rw * VA + 16 + c];
      AG[rr][c] = rr < nrows ? a0 : 0.f;
      AG[rr][16 + c] = rr < nrows ? a1 : 0.f;
    }
  }
  __syncthreads();
  // ---- dx, its column partials
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int cl = 16 * tt + c, col = col0 + cl;
    float dbp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      const float xh = (xv[tt][r] - st[r].x) * st[r].y;
      const float gvv = (fmaf(xh, gv[tt], bv[tt]) > 0.f ? hv[tt][r] : 0.f) * gv[tt];
      const float o = rr < nrows ? dvv[tt][r] + st[r].y * (gvv - S1[rr] - xh * S2[rr]) : 0.f;
      if (rr < nrows) dx[(row0 + rr) * D + col] = o;
      DX[wave][rr][cl] = o;
      dbp += o;
    }
    dbp = xsum32(xsum16(dbp));
    if (g == 0) out[int64_t(D) * VA + col] = dbp;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // dWp[col][j] = sum_r dx[r][col] agg[r][j]: A[i = col][k = r], B[k = r][j]
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x4 w2[2] = {z4(), z4()};
#pragma unroll
    for (int q = 0; q < TR / 4; ++q) {
      const float a = DX[wave][4 * q + g][16 * mt + c];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) w2[tt] = mfma(a, AG[4 * q + g][16 * tt + c], w2[tt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) out[int64_t(col0 + 16 * mt + 4 * g + r) * VA + 16 * tt + c] = w2[tt][r];
  }
  // d agg partial of the wave's columns: A[i = r][k = col] = dx, B[k = col][j] = Wp[col][j]
  f32x4 da[2] = {z4(), z4()};
#pragma unroll
  for (int q = 0; q < CW / 4; ++q) {
    const float a = DX[wave][c][4 * q + g];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) da[tt] = mfma(a, wpv[q][tt], da[tt]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) DA[wave][(4 * g + r) * VA + 16 * tt + c] = da[tt][r];
  __syncthreads();
  // the group partial (waves summed in order), 2 values per thread, handed over write-through
  float* slot = ws + (int64_t(tile) * ngrp + grp) * TR * VA;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = int(threadIdx.x) + k * TB2_T;
    float v = DA[0][i];
#pragma unroll
    for (int w = 1; w < TB2_W; ++w) v += DA[w][i];
    st_sc1(slot + i, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t k = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = k == uint32_t(ngrp - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (flag == 0u) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float* base = ws + int64_t(tile) * ngrp * TR * VA;
  constexpr int MAXG = MAXD / TB2_COLS;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = int(threadIdx.x) + k * TB2_T;
    float v[MAXG];
#pragma unroll
    for (int q = 0; q < MAXG; ++q)
      v[q] = __hip_atomic_load(base + int64_t(q < ngrp ? q : 0) * TR * VA + i, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < MAXG; ++q) s += q < ngrp ? v[q] : 0.f;
    if (i / VA < nrows) dagg[(row0 + i / VA) * VA + i % VA] = s;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

static bool vc_ok(int64_t m, int32_t D) { return m > 0 && m <= 256 && (D == 256 || D == 512 || D == 1024); }

extern "C" int32_t gasfm_view_chain_ok(int64_t m, int32_t D) { return vc_ok(m, D) ? 1 : 0; }

extern "C" int64_t gasfm_view_chain_scratch_floats(int64_t m, int32_t D) {
  const int64_t T = (m + TR - 1) / TR, ncb = D / CW;
  return m * ncb * 4 + T * ncb * TR * VA + 64;  // RSUM (float4 / float2 per (row, block)), d agg partials
}

extern "C" int32_t gasfm_view_chain_counters(int64_t m) { return int32_t((m + TR - 1) / TR); }

namespace {
template <int KU, int KQ>
void launch_hub_bwd1(dim3 g1, hipStream_t st, const float* v, const float2* rsv, int64_t m, const float* gC,
                     const float* bC, const float* Wv, const float* gA, const float* bA, const float* Wa,
                     const float* t, const float* Wr, const float* Wl, const float* dsv, const float* dxr,
                     const float* dxl, const float* dres, float* dacc, float* dWl, float4* RSUM, float* part) {
  hipLaunchKernelGGL((vc_hub_bwd1_kernel<KU, KQ>), g1, dim3(NT), 0, st, v, rsv, m, gC, bC, Wv, gA, bA, Wa, t, Wr,
                     Wl, dsv, dxr, dxl, dres, dacc, dWl, RSUM, part);
}
template <int KU, int KQ>
void launch_tail_bwd1(dim3 g1, hipStream_t st, const float* dv, const float* x, const float* h, const float2* rsx,
                      int64_t m, const float* ln_w, const float* ln_b, const float* Wm, float* dh, float* dWm,
                      float2* RSUMT, float* part) {
  hipLaunchKernelGGL((vc_tail_bwd1_kernel<KU, KQ>), g1, dim3(NT), 0, st, dv, x, h, rsx, m, ln_w, ln_b, Wm, dh, dWm,
                     RSUMT, part);
}
template <int KU>
void kq_hub_bwd1(int64_t m, dim3 g1, hipStream_t st, const float* v, const float2* rsv, const float* gC,
                 const float* bC, const float* Wv, const float* gA, const float* bA, const float* Wa, const float* t,
                 const float* Wr, const float* Wl, const float* dsv, const float* dxr, const float* dxl,
                 const float* dres, float* dacc, float* dWl, float4* RSUM, float* part) {
  if (m <= 64)
    launch_hub_bwd1<KU, 4>(g1, st, v, rsv, m, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl, RSUM,
                           part);
  else if (m <= 128)
    launch_hub_bwd1<KU, 8>(g1, st, v, rsv, m, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl, RSUM,
                           part);
  else
    launch_hub_bwd1<KU, 16>(g1, st, v, rsv, m, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl,
                            RSUM, part);
}
template <int KU>
void kq_tail_bwd1(int64_t m, dim3 g1, hipStream_t st, const float* dv, const float* x, const float* h,
                  const float2* rsx, const float* ln_w, const float* ln_b, const float* Wm, float* dh, float* dWm,
                  float2* RSUMT, float* part) {
  if (m <= 64)
    launch_tail_bwd1<KU, 4>(g1, st, dv, x, h, rsx, m, ln_w, ln_b, Wm, dh, dWm, RSUMT, part);
  else if (m <= 128)
    launch_tail_bwd1<KU, 8>(g1, st, dv, x, h, rsx, m, ln_w, ln_b, Wm, dh, dWm, RSUMT, part);
  else
    launch_tail_bwd1<KU, 16>(g1, st, dv, x, h, rsx, m, ln_w, ln_b, Wm, dh, dWm, RSUMT, part);
}
}  // namespace

extern "C" int gasfm_view_chain_tail_fwd(const float* prev, const float* agg, int64_t m, int32_t D, const float* Wp,
                                         const float* bp, const float* ln_w, const float* ln_b, float eps,
                                         const float* Wm, const float* bm, float* view, float* x, float* h, float* rs,
                                         void* stream) {
  GASFM_REQUIRE(vc_ok(m, D), "gasfm_view_chain_tail_fwd: m=%lld D=%d", (long long)m, D);
  GASFM_REQUIRE(agg && Wp && bp && ln_w && ln_b && Wm && bm && view && x && h && rs,
                "gasfm_view_chain_tail_fwd: null pointer");
  GASFM_REQUIRE(aligned16(agg) && aligned16(Wp) && aligned16(Wm) && (!prev || aligned16(prev)),
                "gasfm_view_chain_tail_fwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(unsigned(((m + TR - 1) / TR) * (D / CW)));
  float2* rso = reinterpret_cast<float2*>(rs);
#define GASFM_VC_TAIL(KU_, P_)                                                                                  \
  hipLaunchKernelGGL((vc_tail_fwd_kernel<KU_, P_>), grid, dim3(NT), 0, st, prev, agg, m, Wp, bp, ln_w, ln_b, eps, Wm, \
                     bm, view, x, h, rso)
  if (prev) {
    if (D == 256) GASFM_VC_TAIL(2, true);
    else if (D == 512) GASFM_VC_TAIL(4, true);
    else GASFM_VC_TAIL(8, true);
  } else {
    if (D == 256) GASFM_VC_TAIL(2, false);
    else if (D == 512) GASFM_VC_TAIL(4, false);
    else GASFM_VC_TAIL(8, false);
  }
#undef GASFM_VC_TAIL
  return launch_status("gasfm_view_chain_tail_fwd");
}

extern "C" int gasfm_view_chain_hub_fwd(const float* v, int64_t m, int32_t D, float eps, const float* Wl,
                                        const float* bl, const float* gC, const float* bC, const float* Wv,
                                        const float* gA, const float* bA, const float* Wa, const float* ba,
                                        const float* Wr, const float* br, float* XL, float* sv, float* t, float* xr,
                                        int32_t ldo, float* rs, void* stream) {
  GASFM_REQUIRE(vc_ok(m, D), "gasfm_view_chain_hub_fwd: m=%lld D=%d", (long long)m, D);
  GASFM_REQUIRE(v && Wl && bl && gC && bC && Wv && gA && bA && Wa && ba && Wr && br && XL && sv && t && xr && rs,
                "gasfm_view_chain_hub_fwd: null pointer");
  GASFM_REQUIRE(aligned16(v) && aligned16(Wl) && aligned16(Wv) && aligned16(Wa) && ldo >= VA,
                "gasfm_view_chain_hub_fwd: alignment / ldo");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int T = int((m + TR - 1) / TR);
  const dim3 grid(unsigned(T * (D / CW) + 2 * T));
#define GASFM_VC_HUB(KU_)                                                                                       \
  hipLaunchKernelGGL((vc_hub_fwd_kernel<KU_>), grid, dim3(NT), 0, st, v, m, eps, Wl, bl, gC, bC, Wv, gA, bA, Wa, ba, \
                     Wr, br, XL, sv, t, xr, ldo, reinterpret_cast<float2*>(rs))
  if (D == 256) GASFM_VC_HUB(2);
  else if (D == 512) GASFM_VC_HUB(4);
  else GASFM_VC_HUB(8);
#undef GASFM_VC_HUB
  return launch_status("gasfm_view_chain_hub_fwd");
}

extern "C" int gasfm_view_chain_hub_bwd(const float* v, const float* rs, int64_t m, int32_t D, const float* gC,
                                        const float* bC, const float* Wv, const float* gA, const float* bA,
                                        const float* Wa, const float* t, const float* Wr, const float* Wl,
                                        const float* dsv, const float* dxr, const float* dxl, const float* dres,
                                        float* dacc, float* dWl, float* part, float* scratch, void* stream) {
  GASFM_REQUIRE(vc_ok(m, D), "gasfm_view_chain_hub_bwd: m=%lld D=%d", (long long)m, D);
  GASFM_REQUIRE(v && rs && gC && bC && Wv && gA && bA && Wa && t && Wr && Wl && dsv && dxr && dxl && dacc && dWl &&
                    part && scratch,
                "gasfm_view_chain_hub_bwd: null pointer");
  GASFM_REQUIRE(aligned16(dxl) && aligned16(scratch), "gasfm_view_chain_hub_bwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int T = int((m + TR - 1) / TR);
  float4* RSUM = reinterpret_cast<float4*>(scratch);
  const float2* rsv = reinterpret_cast<const float2*>(rs);
  const dim3 g1(unsigned(T * (D / CW) + T * (D / CW / 4) + (D / TR) * (D / WGT)));
  if (D == 256)
    kq_hub_bwd1<2>(m, g1, st, v, rsv, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl, RSUM, part);
  else if (D == 512)
    kq_hub_bwd1<4>(m, g1, st, v, rsv, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl, RSUM, part);
  else
    kq_hub_bwd1<8>(m, g1, st, v, rsv, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl, RSUM, part);
  int s = launch_status("gasfm_view_chain_hub_bwd1");
  if (s != GASFM_OK) return s;
#define GASFM_VC_HB2(KU_)                                                                                        \
  hipLaunchKernelGGL((vc_hub_bwd2_kernel<KU_>), dim3(unsigned(T * (D / 64))), dim3(256), 0, st, v, rsv, m, gC, bC, Wv, \
                     gA, bA, Wa, Wr, dsv, dxr, RSUM, dacc)
  if (D == 256) GASFM_VC_HB2(2);
  else if (D == 512) GASFM_VC_HB2(4);
  else GASFM_VC_HB2(8);
#undef GASFM_VC_HB2
  return launch_status("gasfm_view_chain_hub_bwd2");
}

extern "C" int gasfm_view_chain_tail_bwd(const float* dv, const float* x, const float* h, const float* rs,
                                         const float* agg, int64_t m, int32_t D, const float* Wp, const float* ln_w,
                                         const float* ln_b, const float* Wm, float* dh, float* dWm, float* dx,
                                         float* dagg, float* part, float* scratch, uint32_t* counters, void* stream) {
  GASFM_REQUIRE(vc_ok(m, D), "gasfm_view_chain_tail_bwd: m=%lld D=%d", (long long)m, D);
  GASFM_REQUIRE(dv && x && h && rs && agg && Wp && ln_w && ln_b && Wm && dh && dWm && dx && dagg && part && scratch &&
                    counters,
                "gasfm_view_chain_tail_bwd: null pointer");
  GASFM_REQUIRE(aligned16(dv) && aligned16(scratch), "gasfm_view_chain_tail_bwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int T = int((m + TR - 1) / TR), ncb = D / CW;
  float2* RSUMT = reinterpret_cast<float2*>(scratch);
  float* ws = scratch + m * ncb * 4;
  const float2* rsx = reinterpret_cast<const float2*>(rs);
  const dim3 g1(unsigned(T * ncb + (D / TR) * (D / WGT)));
  if (D == 256)
    kq_tail_bwd1<2>(m, g1, st, dv, x, h, rsx, ln_w, ln_b, Wm, dh, dWm, RSUMT, part);
  else if (D == 512)
    kq_tail_bwd1<4>(m, g1, st, dv, x, h, rsx, ln_w, ln_b, Wm, dh, dWm, RSUMT, part);
  else
    kq_tail_bwd1<8>(m, g1, st, dv, x, h, rsx, ln_w, ln_b, Wm, dh, dWm, RSUMT, part);
  int s = launch_status("gasfm_view_chain_tail_bwd1");
  if (s != GASFM_OK) return s;
  hipLaunchKernelGGL(vc_tail_bwd2_kernel, dim3(unsigned(T * (D / TB2_COLS))), dim3(TB2_T), 0, st, dv, dh, x, rsx, agg, m, D, ln_w,
                     ln_b, Wp, RSUMT, dx, dagg, ws, counters, part);
  return launch_status("gasfm_view_chain_tail_bwd2");
}
