// Fused camera-side (view feature rows, m x D, D = n_feat_view, a multiple of 64 <= 1024) chains
// of a GASFM block, gfx950.  Same decomposition as point_block.hip, with the two D x D GEMMs of
// a block left to hipBLASLt (torch.addmm / mm) and everything around them fused:
//
//   tail (Proj2View.forward, code/models/layers.py:345-360):
//     x = prev + W_p agg + b_p           proj_proj2view + state skip           :345-351
//     view = x + W_m relu(LN(x)) + b_m   norm_pre_mlp, ReLU, mlp, skip          :354-360
//     (kernels produce x, x + b_m and h = relu(LN(x)); the GEMM is addmm(x + b_m, h, W_m^T))
//   hub (consumers of view v):
//     sv = W_v relu(LN_c(v))                       lin_view of the projection update (:928-935)
//     XR = W_r (W_a relu(LN_a(v)) + b_a) + b_r     next block's norm_and_proj_view2proj (:331)
//                                                   and its GATv2 lin_r (target rows)
//     XL = W_l v + b_l                             graph_conv_view2global.lin_l (addmm, :551-556)
//
// m is ~1000 cameras, so a 16-row tile per workgroup would occupy 63 CUs.  Every kernel here
// runs ONE wave per (16-row tile, 64-column block): ceil(m/16) x D/64 = 1008 waves at config 4.
// Quantities that need whole rows cross column blocks through small global buffers, always
// combined in block order (deterministic):
//   row statistics   per-block (mean, M2) pairs, merged with Chan's formula;
//   row sums         per-block partials of the LayerNorm-backward sums;
//   32-wide outputs  per-block partial products of the K = D projections.
// Weight / bias / LayerNorm-affine gradients leave as one partial row per tile (each column
// block writes its own columns) for gasfm_colsum.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

using namespace tile;

constexpr int VA = 32;  // aggregation / projection width
constexpr int CB = 64;  // columns per wave
constexpr int L66 = 66, L34 = 34;

struct Slice {
  int64_t row0;
  int nrows, tile, cb, col0, ncb;
};
__device__ __forceinline__ Slice slice_of(int64_t m, int D) {
  Slice s;
  s.tile = blockIdx.x;
  s.cb = blockIdx.y;
  s.ncb = D / CB;
  s.col0 = CB * s.cb;
  s.row0 = int64_t(s.tile) * TR;
  s.nrows = int(m - s.row0 < TR ? m - s.row0 : TR);
  return s;
}

// 16 x 64 slice (rows row0.., columns col0..) of a [m x D] matrix in row layout: lane group g
// holds rows g + 4u (u < 4), lane c = l & 15 the columns col0 + 4c .. +3; rows past nrows are 0
__device__ __forceinline__ void slice_load(const float* __restrict__ P, int D, const Slice& s, float4 (&v)[4],
                                           int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = g + 4 * u;
    v[u] = *reinterpret_cast<const float4*>(P + (s.row0 + (r < s.nrows ? r : 0)) * D + s.col0 + 4 * c);
    if (r >= s.nrows) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ __forceinline__ void slice_store(float* __restrict__ P, int D, const Slice& s, const float4 (&v)[4],
                                            int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = g + 4 * u;
    if (r < s.nrows) *reinterpret_cast<float4*>(P + (s.row0 + r) * D + s.col0 + 4 * c) = v[u];
  }
}
__device__ __forceinline__ void slice_to_lds(float* T, const float4 (&v)[4], int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float2* d = reinterpret_cast<float2*>(T + (g + 4 * u) * L66 + 4 * c);
    d[0] = make_float2(v[u].x, v[u].y);
    d[1] = make_float2(v[u].z, v[u].w);
  }
}
__device__ __forceinline__ void slice_from_lds(const float* T, float4 (&v)[4], int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float2* p = reinterpret_cast<const float2*>(T + (g + 4 * u) * L66 + 4 * c);
    const float2 a = p[0], b = p[1];
    v[u] = make_float4(a.x, a.y, b.x, b.y);
  }
}

// per-row (mean, M2) of a row-layout slice -> SP[row][cb] (two floats)
__device__ __forceinline__ void slice_stats_out(const float4 (&v)[4], const Slice& s, float2* __restrict__ SP,
                                                int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = g + 4 * u;
    const float mean = sum16(v[u].x + v[u].y + v[u].z + v[u].w) * (1.f / CB);
    const float q = (v[u].x - mean) * (v[u].x - mean) + (v[u].y - mean) * (v[u].y - mean) +
                    (v[u].z - mean) * (v[u].z - mean) + (v[u].w - mean) * (v[u].w - mean);
    const float m2 = sum16(q);
    if (c == 0 && r < s.nrows) SP[(s.row0 + r) * s.ncb + s.cb] = make_float2(mean, m2);
  }
}

// (mean, rstd) of the tile's 16 rows from the per-block (mean, M2) pairs (Chan's merge, block
// order), into MS / RS (LDS); lanes 0..15 each merge one row.  Rows past nrows get (0, 1).
__device__ __forceinline__ void merge_stats(const float2* __restrict__ SP, const Slice& s, float eps, float* MS,
                                            float* RS, int lane) {
  if (lane < TR) {
    float mean = 0.f, rstd = 1.f;
    if (lane < s.nrows) {
      const float2* p = SP + (s.row0 + lane) * s.ncb;
      float sm = 0.f;
      for (int b = 0; b < s.ncb; ++b) sm += p[b].x;
      mean = sm / s.ncb;
      float m2 = 0.f;
      for (int b = 0; b < s.ncb; ++b) {
        const float d = p[b].x - mean;
        m2 += p[b].y + CB * d * d;
      }
      rstd = rsq_normal(m2 / (s.ncb * CB) + eps);
    }
    MS[lane] = mean;
    RS[lane] = rstd;
  }
  wave_sync();
}

// ----------------------------------------------------------------------------- tail forward
// x = prev + agg W_p^T + b_p, xb = x + b_m; per-block row statistics of x
template <bool PREV>
__global__ __launch_bounds__(kW) void view_tail_x_kernel(const float* __restrict__ prev,
                                                         const float* __restrict__ agg, int64_t m, int D,
                                                         const float* __restrict__ Wp, const float* __restrict__ bp,
                                                         const float* __restrict__ bm, float* __restrict__ xo,
                                                         float* __restrict__ xbo, float2* __restrict__ SP) {
  __shared__ float Ag[TR * L34];
  __shared__ float Xs[TR * L66];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  {
    float4 va[2];
    rows_load<VA>(agg, VA, s.row0, s.nrows, va, lane);
    rows_to_lds<VA, L34>(Ag, va, lane);
  }
  if (PREV) {
    float4 vp[4];
    slice_load(prev, D, s, vp, lane);
    slice_to_lds(Xs, vp, lane);
  }
  float wb[VA / 4][4];  // B[k = 4s+g][n] = W_p[col0 + n][k]
#pragma unroll
  for (int q = 0; q < VA / 4; ++q)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) wb[q][nt] = Wp[(s.col0 + nt * 16 + c) * VA + 4 * q + g];
  float bpv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bpv[nt] = bp[s.col0 + nt * 16 + c];
  wave_sync();
  f32x4 xa[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = Ag[c * L34 + 4 * q + g];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) xa[nt] = mfma16(a, wb[q][nt], xa[nt]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float* d = Xs + (4 * g + r) * L66 + nt * 16 + c;
      *d = xa[nt][r] + bpv[nt] + (PREV ? *d : 0.f);
    }
  wave_sync();
  float4 vx[4];
  slice_from_lds(Xs, vx, lane);
  slice_stats_out(vx, s, SP, lane);
  slice_store(xo, D, s, vx, lane);
  const float4 b4 = *reinterpret_cast<const float4*>(bm + s.col0 + 4 * c);
#pragma unroll
  for (int u = 0; u < 4; ++u) vx[u] = make_float4(vx[u].x + b4.x, vx[u].y + b4.y, vx[u].z + b4.z, vx[u].w + b4.w);
  slice_store(xbo, D, s, vx, lane);
}

// h = relu(LN(x)); block 0 also stores the row (mean, rstd) for the backward pass
__global__ __launch_bounds__(kW) void view_tail_h_kernel(const float* __restrict__ x, int64_t m, int D,
                                                         const float2* __restrict__ SP,
                                                         const float* __restrict__ gam, const float* __restrict__ bet,
                                                         float eps, float* __restrict__ ho,
                                                         float2* __restrict__ RSo) {
  __shared__ float MS[TR], RS[TR];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  float4 vx[4];
  slice_load(x, D, s, vx, lane);
  merge_stats(SP, s, eps, MS, RS, lane);
  if (s.cb == 0 && lane < s.nrows) RSo[s.row0 + lane] = make_float2(MS[lane], RS[lane]);
  const float4 g4 = *reinterpret_cast<const float4*>(gam + s.col0 + 4 * c);
  const float4 b4 = *reinterpret_cast<const float4*>(bet + s.col0 + 4 * c);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float mu = MS[g + 4 * u], rs = RS[g + 4 * u];
    vx[u] = make_float4(fmaxf(fmaf((vx[u].x - mu) * rs, g4.x, b4.x), 0.f),
                        fmaxf(fmaf((vx[u].y - mu) * rs, g4.y, b4.y), 0.f),
                        fmaxf(fmaf((vx[u].z - mu) * rs, g4.z, b4.z), 0.f),
                        fmaxf(fmaf((vx[u].w - mu) * rs, g4.w, b4.w), 0.f));
  }
  slice_store(ho, D, s, vx, lane);
}

// ----------------------------------------------------------------------------- tail backward
// pass 1: per-block partials of the LayerNorm-backward row sums (sum gv, sum gv x_hat) with
// gv = mask * dh * gamma; the tile's dgamma / dbeta / db_m column partials
__global__ __launch_bounds__(kW) void view_tail_b1_kernel(const float* __restrict__ dv,
                                                          const float* __restrict__ dh,
                                                          const float* __restrict__ x, int64_t m, int D,
                                                          const float2* __restrict__ RSx,
                                                          const float* __restrict__ gam,
                                                          const float* __restrict__ bet, float2* __restrict__ RSUM,
                                                          float* __restrict__ part) {
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  float4 vx[4], vh[4], vd[4];
  slice_load(x, D, s, vx, lane);
  slice_load(dh, D, s, vh, lane);
  slice_load(dv, D, s, vd, lane);
  const float4 g4 = *reinterpret_cast<const float4*>(gam + s.col0 + 4 * c);
  const float4 b4 = *reinterpret_cast<const float4*>(bet + s.col0 + 4 * c);
  const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
  float dgp[4] = {0.f, 0.f, 0.f, 0.f}, dbp[4] = {0.f, 0.f, 0.f, 0.f}, dmp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = g + 4 * u;
    const float2 st = RSx[s.row0 + (r < s.nrows ? r : 0)];
    const float xs[4] = {vx[u].x, vx[u].y, vx[u].z, vx[u].w}, hs[4] = {vh[u].x, vh[u].y, vh[u].z, vh[u].w},
                ds[4] = {vd[u].x, vd[u].y, vd[u].z, vd[u].w};
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (xs[k] - st.x) * st.y;
      const float dy = fmaf(xh, gg[k], bb[k]) > 0.f ? hs[k] : 0.f;  // rows past nrows: dh = 0
      dgp[k] = fmaf(dy, xh, dgp[k]);
      dbp[k] += dy;
      dmp[k] += ds[k];
      s1 = fmaf(dy, gg[k], s1);
      s2 = fmaf(dy * gg[k], xh, s2);
    }
    s1 = sum16(s1);
    s2 = sum16(s2);
    if (c == 0 && r < s.nrows) RSUM[(s.row0 + r) * s.ncb + s.cb] = make_float2(s1, s2);
  }
  // columns 4c..4c+3: sum over the four lane groups
  float* out = part + int64_t(s.tile) * (D * VA + 4 * D) + D * VA;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = sum_groups(dgp[k]), b = sum_groups(dbp[k]), e = sum_groups(dmp[k]);
    if (g == 0) {
      out[D + s.col0 + 4 * c + k] = a;
      out[2 * D + s.col0 + 4 * c + k] = b;
      out[3 * D + s.col0 + 4 * c + k] = e;
    }
  }
}

// pass 2: dx = dv + rstd (gv - mean(gv) - x_hat mean(gv x_hat)); dW_p and db_p column partials;
// this block's share of dagg = dx W_p (partial products, finished by view_rows32_sum)
__global__ __launch_bounds__(kW) void view_tail_b2_kernel(const float* __restrict__ dv,
                                                          const float* __restrict__ dh,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ agg, int64_t m, int D,
                                                          const float2* __restrict__ RSx,
                                                          const float2* __restrict__ RSUM,
                                                          const float* __restrict__ Wp,
                                                          const float* __restrict__ gam,
                                                          const float* __restrict__ bet, float* __restrict__ dx,
                                                          float* __restrict__ DA, float* __restrict__ part) {
  __shared__ float Ag[TR * L34];
  __shared__ float DXs[TR * L66];
  __shared__ float S1[TR], S2[TR];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  {
    float4 va[2];
    rows_load<VA>(agg, VA, s.row0, s.nrows, va, lane);
    rows_to_lds<VA, L34>(Ag, va, lane);
  }
  float4 vx[4], vh[4], vd[4];
  slice_load(x, D, s, vx, lane);
  slice_load(dh, D, s, vh, lane);
  slice_load(dv, D, s, vd, lane);
  if (lane < TR) {
    float a = 0.f, b = 0.f;
    if (lane < s.nrows) {
      const float2* p = RSUM + (s.row0 + lane) * s.ncb;
      for (int q = 0; q < s.ncb; ++q) {
        a += p[q].x;
        b += p[q].y;
      }
    }
    S1[lane] = a / D;
    S2[lane] = b / D;
  }
  wave_sync();
  const float4 g4 = *reinterpret_cast<const float4*>(gam + s.col0 + 4 * c);
  const float4 b4 = *reinterpret_cast<const float4*>(bet + s.col0 + 4 * c);
  const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
  float dbp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = g + 4 * u;
    const float2 st = RSx[s.row0 + (r < s.nrows ? r : 0)];
    const float xs[4] = {vx[u].x, vx[u].y, vx[u].z, vx[u].w}, hs[4] = {vh[u].x, vh[u].y, vh[u].z, vh[u].w},
                ds[4] = {vd[u].x, vd[u].y, vd[u].z, vd[u].w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (xs[k] - st.x) * st.y;
      const float gv = (fmaf(xh, gg[k], bb[k]) > 0.f ? hs[k] : 0.f) * gg[k];
      o[k] = r < s.nrows ? ds[k] + st.y * (gv - S1[r] - xh * S2[r]) : 0.f;
      dbp[k] += o[k];
    }
    vd[u] = make_float4(o[0], o[1], o[2], o[3]);
  }
  slice_store(dx, D, s, vd, lane);
  slice_to_lds(DXs, vd, lane);
  float* out = part + int64_t(s.tile) * (D * VA + 4 * D);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = sum_groups(dbp[k]);
    if (g == 0) out[D * VA + s.col0 + 4 * c + k] = a;
  }
  wave_sync();
  // dW_p[col][j] over the tile's rows: A[i = col][kk = row] = dx, B[kk = row][j] = agg
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    f32x4 w2[2] = {zero4(), zero4()};
#pragma unroll
    for (int q = 0; q < TR / 4; ++q) {
      const float a = DXs[(4 * q + g) * L66 + mt * 16 + c];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) w2[nt] = mfma16(a, Ag[(4 * q + g) * L34 + nt * 16 + c], w2[nt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) out[(s.col0 + mt * 16 + 4 * g + r) * VA + nt * 16 + c] = w2[nt][r];
  }
  // dagg partial: A[i = row][k = col] = dx, B[k = col][j] = W_p[col][j]
  f32x4 da[2] = {zero4(), zero4()};
#pragma unroll
  for (int q = 0; q < CB / 4; ++q) {
    const float a = DXs[c * L66 + 4 * q + g];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) da[nt] = mfma16(a, Wp[(s.col0 + 4 * q + g) * VA + nt * 16 + c], da[nt]);
  }
  float* dst = DA + (int64_t(s.tile) * s.ncb + s.cb) * TR * VA;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) dst[(4 * g + r) * VA + nt * 16 + c] = da[nt][r];
}

// out[16 x 32 tile] = sum over column blocks of the partial products (block order); one
// 256-thread workgroup per tile, 2 outputs per thread, the block loads in flight together
constexpr int kSumThreads = 256;
__global__ __launch_bounds__(kSumThreads) void view_rows32_sum_kernel(const float* __restrict__ PPt, int64_t m,
                                                                      int ncb, float* __restrict__ out) {
  const int64_t row0 = int64_t(blockIdx.x) * TR;
  const int nrows = int(m - row0 < TR ? m - row0 : TR);
  const float* src = PPt + int64_t(blockIdx.x) * ncb * TR * VA;
  for (int i = threadIdx.x; i < TR * VA; i += kSumThreads) {
    float s = 0.f;
#pragma unroll 8
    for (int b = 0; b < ncb; ++b) s += src[b * TR * VA + i];
    if (i / VA < nrows) out[(row0 + i / VA) * VA + i % VA] = s;
  }
}

// ----------------------------------------------------------------------------- hub forward
__global__ __launch_bounds__(kW) void view_stats_kernel(const float* __restrict__ v, int64_t m, int D,
                                                        float2* __restrict__ SP) {
  const Slice s = slice_of(m, D);
  float4 vx[4];
  slice_load(v, D, s, vx, threadIdx.x);
  slice_stats_out(vx, s, SP, threadIdx.x);
}

// partial products of this column block: [S | T] = relu(LN_c v) W_v^T, relu(LN_a v) W_a^T over
// its 64 columns; block 0 also stores the row (mean, rstd)
__global__ __launch_bounds__(kW) void view_hub_proj_kernel(
    const float* __restrict__ v, int64_t m, int D, float eps, const float2* __restrict__ SP,
    const float* __restrict__ gC, const float* __restrict__ bC, const float* __restrict__ Wv,
    const float* __restrict__ gA, const float* __restrict__ bA, const float* __restrict__ Wa,
    float* __restrict__ PP, float2* __restrict__ RSo) {
  __shared__ float Vs[TR * L66];
  __shared__ float G[4 * CB];
  __shared__ float MS[TR], RS[TR];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  float4 vx[4];
  slice_load(v, D, s, vx, lane);
  float wv[16][2], wa[16][2];  // B[k = col0 + 4q+g][n] = W[n][k]
#pragma unroll
  for (int q = 0; q < 16; ++q)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      wv[q][nt] = Wv[(nt * 16 + c) * D + s.col0 + 4 * q + g];
      wa[q][nt] = Wa[(nt * 16 + c) * D + s.col0 + 4 * q + g];
    }
  G[lane] = gC[s.col0 + lane];
  G[CB + lane] = bC[s.col0 + lane];
  G[2 * CB + lane] = gA[s.col0 + lane];
  G[3 * CB + lane] = bA[s.col0 + lane];
  slice_to_lds(Vs, vx, lane);
  merge_stats(SP, s, eps, MS, RS, lane);
  if (s.cb == 0 && lane < s.nrows) RSo[s.row0 + lane] = make_float2(MS[lane], RS[lane]);
  const float mi = MS[c], ri = RS[c];
  f32x4 accS[2] = {zero4(), zero4()}, accT[2] = {zero4(), zero4()};
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = 4 * q + g;
    const float xh = (Vs[c * L66 + k] - mi) * ri;
    const float hc = fmaxf(fmaf(xh, G[k], G[CB + k]), 0.f);
    const float ha = fmaxf(fmaf(xh, G[2 * CB + k], G[3 * CB + k]), 0.f);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      accS[nt] = mfma16(hc, wv[q][nt], accS[nt]);
      accT[nt] = mfma16(ha, wa[q][nt], accT[nt]);
    }
  }
  float* dst = PP + (int64_t(s.tile) * s.ncb + s.cb) * 2 * TR * VA;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      dst[(4 * g + r) * VA + nt * 16 + c] = accS[nt][r];
      dst[TR * VA + (4 * g + r) * VA + nt * 16 + c] = accT[nt][r];
    }
}

// sv = sum_b S_b, t = sum_b T_b + b_a (block order), XR = t W_r^T + b_r; one 256-thread
// workgroup per tile (4 outputs per thread), wave 0 runs the W_r product
__global__ __launch_bounds__(kSumThreads) void view_hub_fin_kernel(const float* __restrict__ PP, int64_t m, int ncb,
                                                                   const float* __restrict__ ba,
                                                                   const float* __restrict__ Wr,
                                                                   const float* __restrict__ br,
                                                                   float* __restrict__ sv, float* __restrict__ to,
                                                                   float* __restrict__ xr, int ldo) {
  __shared__ float Tt[TR * L34];
  const int64_t row0 = int64_t(blockIdx.x) * TR;
  const int nrows = int(m - row0 < TR ? m - row0 : TR);
  const float* src = PP + int64_t(blockIdx.x) * ncb * 2 * TR * VA;
  for (int i = threadIdx.x; i < 2 * TR * VA; i += kSumThreads) {
    const int which = i / (TR * VA), j = i % (TR * VA), e = j / VA, n = j % VA;
    float s = 0.f;
#pragma unroll 8
    for (int b = 0; b < ncb; ++b) s += src[(b * 2 + which) * TR * VA + j];
    if (which) {
      s += ba[n];
      Tt[e * L34 + n] = s;
      if (e < nrows) to[(row0 + e) * VA + n] = s;
    } else if (e < nrows) {
      sv[(row0 + e) * ldo + n] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x >= kW) return;
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  f32x4 accR[2] = {zero4(), zero4()};
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = Tt[c * L34 + 4 * q + g];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) accR[nt] = mfma16(a, Wr[(nt * 16 + c) * VA + 4 * q + g], accR[nt]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = 4 * g + r;
    if (e < nrows) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) xr[(row0 + e) * ldo + nt * 16 + c] = accR[nt][r] + br[nt * 16 + c];
    }
  }
}

// ----------------------------------------------------------------------------- hub backward
// hub partial-row layout (per tile)
struct HubPart {
  int64_t WV, WA, GC, BC, GA, BA, BL, WR, BAB, BR, cols;
  __device__ __host__ explicit HubPart(int D)
      : WV(0), WA(int64_t(VA) * D), GC(2 * int64_t(VA) * D), BC(GC + D), GA(BC + D), BA(GA + D), BL(BA + D),
        WR(BL + D), BAB(WR + VA * VA), BR(BAB + VA), cols(BR + VA) {}
};

// dt = dxr W_r (-> DT), dW_r = dxr^T t, db_r = sum dxr, db_a = sum dt; one wave per tile
__global__ __launch_bounds__(kW) void view_hub_b0_kernel(const float* __restrict__ dxr,
                                                         const float* __restrict__ t, int64_t m, int D,
                                                         const float* __restrict__ Wr, float* __restrict__ DT,
                                                         float* __restrict__ part) {
  __shared__ float Xr[TR * L34], Tt[TR * L34], Dt[TR * L34];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const int64_t row0 = int64_t(blockIdx.x) * TR;
  const int nrows = int(m - row0 < TR ? m - row0 : TR);
  const HubPart P(D);
  float* out = part + int64_t(blockIdx.x) * P.cols;
  {
    float4 a[2], b[2];
    rows_load<VA>(dxr, VA, row0, nrows, a, lane);
    rows_load<VA>(t, VA, row0, nrows, b, lane);
    rows_to_lds<VA, L34>(Xr, a, lane);
    rows_to_lds<VA, L34>(Tt, b, lane);
  }
  wave_sync();
  f32x4 d2[2] = {zero4(), zero4()};
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = Xr[c * L34 + 4 * q + g];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) d2[nt] = mfma16(a, Wr[(4 * q + g) * VA + nt * 16 + c], d2[nt]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) Dt[(4 * g + r) * L34 + nt * 16 + c] = d2[nt][r];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x4 w2[2] = {zero4(), zero4()};
#pragma unroll
    for (int q = 0; q < TR / 4; ++q) {
      const float a = Xr[(4 * q + g) * L34 + mt * 16 + c];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) w2[nt] = mfma16(a, Tt[(4 * q + g) * L34 + nt * 16 + c], w2[nt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) out[P.WR + (mt * 16 + 4 * g + r) * VA + nt * 16 + c] = w2[nt][r];
  }
  wave_sync();
  {
    float4 vd[2];
    rows_from_lds<VA, L34>(Dt, vd, lane);
    rows_store<VA>(DT, VA, row0, nrows, vd, lane);
  }
  if (lane < VA) {
    float sr = 0.f, sa = 0.f;
    for (int e = 0; e < TR; ++e) {  // rows past nrows are zero in Xr and hence in Dt
      sr += Xr[e * L34 + lane];
      sa += Dt[e * L34 + lane];
    }
    out[P.BR + lane] = sr;
    out[P.BAB + lane] = sa;
  }
}

// d relu-outs of both LayerNorm branches for this column block (C layout)
__device__ __forceinline__ void hub_dh(const float* Sd, const float* Dt, const float* __restrict__ Wv,
                                       const float* __restrict__ Wa, int D, int col0, int c, int g, f32x4 (&dhc)[4],
                                       f32x4 (&dha)[4]) {
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) dhc[nt] = dha[nt] = zero4();
#pragma unroll
  for (int q = 0; q < VA / 4; ++q) {
    const float a = Sd[c * L34 + 4 * q + g], b = Dt[c * L34 + 4 * q + g];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = col0 + nt * 16 + c;
      dhc[nt] = mfma16(a, Wv[(4 * q + g) * D + col], dhc[nt]);
      dha[nt] = mfma16(b, Wa[(4 * q + g) * D + col], dha[nt]);
    }
  }
}

// pass 1: LayerNorm-backward row-sum partials of both branches, dgamma / dbeta, db_l and the
// dW_v / dW_a column-block partials of the tile
__global__ __launch_bounds__(kW) void view_hub_b1_kernel(
    const float* __restrict__ v, int64_t m, int D, const float2* __restrict__ RSv, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ Wv, const float* __restrict__ gA,
    const float* __restrict__ bA, const float* __restrict__ Wa, const float* __restrict__ dsv,
    const float* __restrict__ DT, const float* __restrict__ dxl, float4* __restrict__ RSUM,
    float* __restrict__ part) {
  __shared__ float Vs[TR * L66];
  __shared__ float Sd[TR * L34], Dt[TR * L34];
  __shared__ float MS[TR], RS[TR];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  const HubPart P(D);
  float* out = part + int64_t(s.tile) * P.cols;
  {
    float4 a[2], b[2], vx[4], vl[4];
    rows_load<VA>(dsv, VA, s.row0, s.nrows, a, lane);
    rows_load<VA>(DT, VA, s.row0, s.nrows, b, lane);
    slice_load(v, D, s, vx, lane);
    slice_load(dxl, D, s, vl, lane);
    rows_to_lds<VA, L34>(Sd, a, lane);
    rows_to_lds<VA, L34>(Dt, b, lane);
    slice_to_lds(Vs, vx, lane);
    // db_l: column sums of dXL over the tile
    float4 sl = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sl.x += vl[u].x;
      sl.y += vl[u].y;
      sl.z += vl[u].z;
      sl.w += vl[u].w;
    }
    sl = make_float4(sum_groups(sl.x), sum_groups(sl.y), sum_groups(sl.z), sum_groups(sl.w));
    if (g == 0) {
      float* o = out + P.BL + s.col0 + 4 * c;
      o[0] = sl.x;
      o[1] = sl.y;
      o[2] = sl.z;
      o[3] = sl.w;
    }
    if (lane < TR) {
      const float2 st = RSv[s.row0 + (lane < s.nrows ? lane : 0)];
      MS[lane] = st.x;
      RS[lane] = st.y;
    }
  }
  wave_sync();
  f32x4 dhc[4], dha[4];
  hub_dh(Sd, Dt, Wv, Wa, D, s.col0, c, g, dhc, dha);
  float gc[4], bc[4], ga[4], bav[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = s.col0 + nt * 16 + c;
    gc[nt] = gC[col];
    bc[nt] = bC[col];
    ga[nt] = gA[col];
    bav[nt] = bA[col];
  }
  float dgc[4] = {0.f, 0.f, 0.f, 0.f}, dbcp[4] = {0.f, 0.f, 0.f, 0.f}, dgap[4] = {0.f, 0.f, 0.f, 0.f},
        dbap[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = 4 * g + r;
    const float me = MS[e], re = RS[e];
    float s1c = 0.f, s2c = 0.f, s1a = 0.f, s2a = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float xh = (Vs[e * L66 + nt * 16 + c] - me) * re;
      const float dyc = fmaf(xh, gc[nt], bc[nt]) > 0.f ? dhc[nt][r] : 0.f;  // rows past nrows: 0
      const float dya = fmaf(xh, ga[nt], bav[nt]) > 0.f ? dha[nt][r] : 0.f;
      dgc[nt] = fmaf(dyc, xh, dgc[nt]);
      dbcp[nt] += dyc;
      dgap[nt] = fmaf(dya, xh, dgap[nt]);
      dbap[nt] += dya;
      s1c = fmaf(dyc, gc[nt], s1c);
      s2c = fmaf(dyc * gc[nt], xh, s2c);
      s1a = fmaf(dya, ga[nt], s1a);
      s2a = fmaf(dya * ga[nt], xh, s2a);
    }
    s1c = sum16(s1c);
    s2c = sum16(s2c);
    s1a = sum16(s1a);
    s2a = sum16(s2a);
    if (c == 0 && e < s.nrows) RSUM[(s.row0 + e) * s.ncb + s.cb] = make_float4(s1c, s2c, s1a, s2a);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const float a0 = sum_groups(dgc[nt]), a1 = sum_groups(dbcp[nt]), a2 = sum_groups(dgap[nt]),
                a3 = sum_groups(dbap[nt]);
    if (g == 0) {
      const int col = s.col0 + nt * 16 + c;
      out[P.GC + col] = a0;
      out[P.BC + col] = a1;
      out[P.GA + col] = a2;
      out[P.BA + col] = a3;
    }
  }
  // dW_v = dsv^T relu(LN_c v), dW_a = dt^T relu(LN_a v) over the tile's rows
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x4 wc[4] = {zero4(), zero4(), zero4(), zero4()}, wa2[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int q = 0; q < TR / 4; ++q) {
      const int row = 4 * q + g;
      const float a = Sd[row * L34 + mt * 16 + c], b = Dt[row * L34 + mt * 16 + c];
      const float mr = MS[row], rr = RS[row];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float xr = (Vs[row * L66 + nt * 16 + c] - mr) * rr;
        wc[nt] = mfma16(a, fmaxf(fmaf(xr, gc[nt], bc[nt]), 0.f), wc[nt]);
        wa2[nt] = mfma16(b, fmaxf(fmaf(xr, ga[nt], bav[nt]), 0.f), wa2[nt]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int64_t o = int64_t(mt * 16 + 4 * g + r) * D + s.col0 + nt * 16 + c;
        out[P.WV + o] = wc[nt][r];
        out[P.WA + o] = wa2[nt][r];
      }
  }
}

// pass 2: dacc += rstd (gv_c - mean gv_c - x_hat mean(gv_c x_hat)) + (same for branch a)
__global__ __launch_bounds__(kW) void view_hub_b2_kernel(
    const float* __restrict__ v, int64_t m, int D, const float2* __restrict__ RSv, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ Wv, const float* __restrict__ gA,
    const float* __restrict__ bA, const float* __restrict__ Wa, const float* __restrict__ dsv,
    const float* __restrict__ DT, const float4* __restrict__ RSUM, const float* __restrict__ dres,
    float* __restrict__ dacc) {
  __shared__ float Vs[TR * L66];
  __shared__ float Sd[TR * L34], Dt[TR * L34];
  __shared__ float MS[TR], RS[TR];
  __shared__ float4 SM[TR];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const Slice s = slice_of(m, D);
  {
    float4 a[2], b[2], vx[4];
    rows_load<VA>(dsv, VA, s.row0, s.nrows, a, lane);
    rows_load<VA>(DT, VA, s.row0, s.nrows, b, lane);
    slice_load(v, D, s, vx, lane);
    rows_to_lds<VA, L34>(Sd, a, lane);
    rows_to_lds<VA, L34>(Dt, b, lane);
    slice_to_lds(Vs, vx, lane);
    if (lane < TR) {
      const int rr = lane < s.nrows ? lane : 0;
      const float2 st = RSv[s.row0 + rr];
      MS[lane] = st.x;
      RS[lane] = st.y;
      float4 a4 = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int q = 0; q < s.ncb; ++q) {
        const float4 p = RSUM[(s.row0 + rr) * s.ncb + q];
        a4.x += p.x;
        a4.y += p.y;
        a4.z += p.z;
        a4.w += p.w;
      }
      SM[lane] = make_float4(a4.x / D, a4.y / D, a4.z / D, a4.w / D);
    }
  }
  wave_sync();
  f32x4 dhc[4], dha[4];
  hub_dh(Sd, Dt, Wv, Wa, D, s.col0, c, g, dhc, dha);
  float gc[4], bc[4], ga[4], bav[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = s.col0 + nt * 16 + c;
    gc[nt] = gC[col];
    bc[nt] = bC[col];
    ga[nt] = gA[col];
    bav[nt] = bA[col];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = 4 * g + r;
    const float me = MS[e], re = RS[e];
    const float4 sm = SM[e];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float xh = (Vs[e * L66 + nt * 16 + c] - me) * re;
      const float gvc = (fmaf(xh, gc[nt], bc[nt]) > 0.f ? dhc[nt][r] : 0.f) * gc[nt];
      const float gva = (fmaf(xh, ga[nt], bav[nt]) > 0.f ? dha[nt][r] : 0.f) * ga[nt];
      if (e < s.nrows) {
        const int64_t o = (s.row0 + e) * D + s.col0 + nt * 16 + c;
        dacc[o] += re * (gvc - sm.x - xh * sm.y) + re * (gva - sm.z - xh * sm.w) + (dres ? dres[o] : 0.f);
      }
    }
  }
}

bool width_ok(int32_t D) { return D > 0 && D % CB == 0 && D <= 1024; }

dim3 grid2(int64_t m, int D) { return dim3(unsigned((m + TR - 1) / TR), unsigned(D / CB)); }
dim3 grid1(int64_t m) { return dim3(unsigned((m + TR - 1) / TR)); }

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int32_t gasfm_view_tail_part_cols(int32_t D) { return D * VA + 4 * D; }
extern "C" int32_t gasfm_view_hub_part_cols(int32_t D) { return int32_t(HubPart(D).cols); }
extern "C" int64_t gasfm_view_scratch_floats(int64_t m, int32_t D) {
  const int64_t tiles = (m + TR - 1) / TR, ncb = D / CB;
  // per-(row, block) statistics / sums (<= 4 floats) + per-(tile, block) partial products
  return m * ncb * 4 + tiles * ncb * 2 * TR * VA + m * VA;
}

extern "C" int gasfm_view_tail_fwd(const float* prev, const float* agg, int64_t m, int32_t D, const float* Wp,
                                   const float* bp, const float* ln_w, const float* ln_b, float eps, const float* bm,
                                   float* x, float* xb, float* h, float* rs, float* scratch, void* stream) {
  GASFM_REQUIRE(m >= 0 && width_ok(D), "gasfm_view_tail_fwd: m=%lld D=%d", (long long)m, D);
  if (m == 0) return GASFM_OK;
  GASFM_REQUIRE(agg && Wp && bp && ln_w && ln_b && bm && x && xb && h && rs && scratch,
                "gasfm_view_tail_fwd: null pointer");
  GASFM_REQUIRE(aligned16(agg) && aligned16(x) && aligned16(xb) && aligned16(h) && aligned16(bm) &&
                    aligned16(ln_w) && aligned16(ln_b) && (!prev || aligned16(prev)),
                "gasfm_view_tail_fwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float2* SP = reinterpret_cast<float2*>(scratch);
  if (prev)
    hipLaunchKernelGGL(view_tail_x_kernel<true>, grid2(m, D), dim3(kW), 0, st, prev, agg, m, D, Wp, bp, bm, x, xb, SP);
  else
    hipLaunchKernelGGL(view_tail_x_kernel<false>, grid2(m, D), dim3(kW), 0, st, prev, agg, m, D, Wp, bp, bm, x, xb,
                       SP);
  hipLaunchKernelGGL(view_tail_h_kernel, grid2(m, D), dim3(kW), 0, st, x, m, D, SP, ln_w, ln_b, eps, h,
                     reinterpret_cast<float2*>(rs));
  return launch_status("gasfm_view_tail_fwd");
}

extern "C" int gasfm_view_tail_bwd(const float* dv, const float* dh, const float* x, const float* rs,
                                   const float* agg, int64_t m, int32_t D, const float* Wp, const float* ln_w,
                                   const float* ln_b, float* dx, float* dagg, float* part, float* scratch,
                                   void* stream) {
  GASFM_REQUIRE(m >= 0 && width_ok(D), "gasfm_view_tail_bwd: m=%lld D=%d", (long long)m, D);
  if (m == 0) return GASFM_OK;
  GASFM_REQUIRE(dv && dh && x && rs && agg && Wp && ln_w && ln_b && dx && dagg && part && scratch,
                "gasfm_view_tail_bwd: null pointer");
  GASFM_REQUIRE(aligned16(dv) && aligned16(dh) && aligned16(x) && aligned16(agg) && aligned16(dx) &&
                    aligned16(ln_w) && aligned16(ln_b),
                "gasfm_view_tail_bwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t ncb = D / CB;
  float2* RSUM = reinterpret_cast<float2*>(scratch);
  float* DA = scratch + m * ncb * 4;
  const float2* RSx = reinterpret_cast<const float2*>(rs);
  hipLaunchKernelGGL(view_tail_b1_kernel, grid2(m, D), dim3(kW), 0, st, dv, dh, x, m, D, RSx, ln_w, ln_b, RSUM, part);
  hipLaunchKernelGGL(view_tail_b2_kernel, grid2(m, D), dim3(kW), 0, st, dv, dh, x, agg, m, D, RSx, RSUM, Wp, ln_w,
                     ln_b, dx, DA, part);
  hipLaunchKernelGGL(view_rows32_sum_kernel, grid1(m), dim3(kSumThreads), 0, st, DA, m, int(ncb), dagg);
  return launch_status("gasfm_view_tail_bwd");
}

extern "C" int gasfm_view_hub_fwd(const float* v, int64_t m, int32_t D, float eps, const float* gC, const float* bC,
                                  const float* Wv, const float* gA, const float* bA, const float* Wa,
                                  const float* ba, const float* Wr, const float* br, float* sv, float* t, float* xr,
                                  int32_t ldo, float* rs, float* scratch, void* stream) {
  GASFM_REQUIRE(m >= 0 && width_ok(D), "gasfm_view_hub_fwd: m=%lld D=%d", (long long)m, D);
  if (m == 0) return GASFM_OK;
  GASFM_REQUIRE(v && gC && bC && Wv && gA && bA && Wa && ba && Wr && br && sv && t && xr && rs && scratch,
                "gasfm_view_hub_fwd: null pointer");
  GASFM_REQUIRE(aligned16(v) && ldo >= VA, "gasfm_view_hub_fwd: alignment / ldo=%d", ldo);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t ncb = D / CB;
  float2* SP = reinterpret_cast<float2*>(scratch);
  float* PP = scratch + m * ncb * 4;
  hipLaunchKernelGGL(view_stats_kernel, grid2(m, D), dim3(kW), 0, st, v, m, D, SP);
  hipLaunchKernelGGL(view_hub_proj_kernel, grid2(m, D), dim3(kW), 0, st, v, m, D, eps, SP, gC, bC, Wv, gA, bA, Wa,
                     PP, reinterpret_cast<float2*>(rs));
  hipLaunchKernelGGL(view_hub_fin_kernel, grid1(m), dim3(kSumThreads), 0, st, PP, m, int(ncb), ba, Wr, br, sv, t, xr, ldo);
  return launch_status("gasfm_view_hub_fwd");
}

extern "C" int gasfm_view_hub_bwd(const float* v, const float* rs, int64_t m, int32_t D, const float* gC,
                                  const float* bC, const float* Wv, const float* gA, const float* bA, const float* Wa,
                                  const float* t, const float* Wr, const float* dsv, const float* dxr,
                                  const float* dxl, const float* dres, float* dacc, float* part, float* scratch,
                                  void* stream) {
  GASFM_REQUIRE(m >= 0 && width_ok(D), "gasfm_view_hub_bwd: m=%lld D=%d", (long long)m, D);
  if (m == 0) return GASFM_OK;
  GASFM_REQUIRE(v && rs && gC && bC && Wv && gA && bA && Wa && t && Wr && dsv && dxr && dxl && dacc && part &&
                    scratch,
                "gasfm_view_hub_bwd: null pointer");
  GASFM_REQUIRE(aligned16(v) && aligned16(dsv) && aligned16(dxr) && aligned16(t) && aligned16(dxl),
                "gasfm_view_hub_bwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t ncb = D / CB;
  float4* RSUM = reinterpret_cast<float4*>(scratch);
  float* DT = scratch + m * ncb * 4;  // m x 32 inside the partial-product area
  const float2* RSv = reinterpret_cast<const float2*>(rs);
  hipLaunchKernelGGL(view_hub_b0_kernel, grid1(m), dim3(kW), 0, st, dxr, t, m, D, Wr, DT, part);
  hipLaunchKernelGGL(view_hub_b1_kernel, grid2(m, D), dim3(kW), 0, st, v, m, D, RSv, gC, bC, Wv, gA, bA, Wa, dsv, DT,
                     dxl, RSUM, part);
  hipLaunchKernelGGL(view_hub_b2_kernel, grid2(m, D), dim3(kW), 0, st, v, m, D, RSv, gC, bC, Wv, gA, bA, Wa, dsv, DT,
                     RSUM, dres, dacc);
  return launch_status("gasfm_view_hub_bwd");
}
