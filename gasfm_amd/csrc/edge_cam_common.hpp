// Shared helpers of the camera-item edge kernels (edge_cam.hip, edge_seam.hip): constants, LayerNorm
// and MFMA slab helpers on the T layout.  Device-only, included by both translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

using namespace tile;

constexpr int F = 32;       // projection features (n_feat_proj) = HC of both convs (H = 4, C = 8)
constexpr int H = 4;
constexpr int NX = 64;      // [point | camera] lin_l outputs
constexpr int LD34 = 34;    // LDS row stride of the P_hat tile
constexpr int LDA = 36;     // LDS row stride of staged weights W[out][in] (A operand, 2-way banks)
constexpr int PART = F + 2 * H;  // packed partial row

// leaky_relu for 0 <= slope <= 1 (the launchers require it; GATv2's 0.2): max(z, slope z) is
// two VALU instead of a compare, a multiply and a select
__device__ __forceinline__ float leaky(float z, float slope) { return fmaxf(z, z * slope); }

// max over the 16 lanes of a row (DPP, as lanes.hpp's sums)
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, xor_lane<1>(v));
  v = fmaxf(v, xor_lane<2>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));  // row_half_mirror: quad 0 <-> quad 1 of each half-row
  v = fmaxf(v, xor_lane<8>(v));
  return v;
}

// a work item in scalar registers (its fields are wave-uniform)
__device__ __forceinline__ gasfm_work_item uniform_item(const gasfm_work_item& w) {
  return gasfm_work_item{__builtin_amdgcn_readfirstlane(w.seg), __builtin_amdgcn_readfirstlane(w.begin),
                         __builtin_amdgcn_readfirstlane(w.end), __builtin_amdgcn_readfirstlane(w.slot)};
}

// Rows of a 16 x 32 tile in row layout: lane l holds row (l >> 3) + 8u (u = 0, 1), columns
// 4 (l & 7) .. + 3.  Rows >= nrows re-read row 0 (always valid); phat_to_lds writes zeros for
// them.  No select on the loaded registers here: these loads are the next tile's prefetch, and
// a select right after them would make the wave wait for them at once.
__device__ __forceinline__ void load_rows(const float* __restrict__ X, int64_t ld, int64_t row0, int nrows,
                                          float4 (&v)[2], int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (lane >> 3) + 8 * u;
    v[u] = *reinterpret_cast<const float4*>(X + (row0 + (r < nrows ? r : 0)) * ld + (lane & 7) * 4);
  }
}

// relu(LN(P)) of the row-layout registers into the wave's LDS tile (row stride 34); rows >= nrows
// are zeros.  LN == false: the raw rows (the final update, graph_attn_sfm.py:141-148).
template <bool LN>
__device__ __forceinline__ void phat_to_lds(const float4 (&v)[2], int nrows, float4 g4, float4 b4, float eps,
                                            float* T, int lane) {
  const int cc = (lane & 7) * 4;
  const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (lane >> 3) + 8 * u;
    const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    float mean = 0.f, rstd = 1.f;
    if (LN) {
      mean = group_sum<8>(x[0] + x[1] + x[2] + x[3]) * (1.f / F);
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) q = fmaf(x[k] - mean, x[k] - mean, q);
      rstd = rsq_normal(group_sum<8>(q) * (1.f / F) + eps);
    }
    float ph[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = LN ? (x[k] - mean) * rstd : x[k];
      ph[k] = (r < nrows) ? (LN ? fmaxf(fmaf(xh, gg[k], bb[k]), 0.f) : xh) : 0.f;
    }
    float2* d = reinterpret_cast<float2*>(T + r * LD34 + cc);
    d[0] = make_float2(ph[0], ph[1]);
    d[1] = make_float2(ph[2], ph[3]);
  }
}

// acc[ot] += W[16 ot + c][k] P_hat[edge c][k] over k < 32: A = W rows (LDS, stride LDA), B = P_hat^T
template <int OT>
__device__ __forceinline__ void xl_t(const float* Wl, const float* T, f32x4 (&acc)[OT], int c, int g) {
#pragma unroll
  for (int s = 0; s < F / 4; ++s) {
    const float b = T[c * LD34 + 4 * s + g];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(Wl[(16 * ot + c) * LDA + 4 * s + g], b, acc[ot]);
  }
}

// ---- register-resident front end (GASFM_EDGE_CAM_R, default): no P_hat tile in LDS.
// P rows are loaded straight into the B-operand layout of the transposed product ("slabs": lane
// (g, c) holds P[edge c][16 u + 4 g + j], j < 4, u = 0, 1 -- the k index of MFMA step (u, j) is
// 16 u + 4 g + j), the LayerNorm runs on those registers (a row's 32 features: 8 per lane, then
// the 4 lane groups), and the weights are staged once per workgroup as float4 slabs in the same
// k order (one ds_read_b128 per 4 MFMAs; was a ds_read_b32 per MFMA operand and a 16 x 34 LDS
// tile write + read per 16 edges).  The accumulators come out exactly as xl_t's (lane (g, c):
// features 16 ot + 4 g + r of edge c).
#ifndef GASFM_EDGE_CAM_R
#define GASFM_EDGE_CAM_R 1
#endif
constexpr bool kCamR = GASFM_EDGE_CAM_R != 0;
#ifndef GASFM_CAM_MINW
#define GASFM_CAM_MINW 3  // minimum waves per SIMD (168 VGPRs): fwd 282 -> 251 us, bwd 270 -> 236 us vs 2 (tools/edge_bench.py)
#endif

// W [O x 32] rows (o < O) -> slabs Q[(ot * 2 + u) * 64 + 16 g + c] = (W[16 ot + c][16 u + 4 g + j], j < 4)
template <int O, int NT, class Src>
__device__ __forceinline__ void stage_slabs32(Src src, float* Q) {
  Stage<O * F, NT> st;
  st.load([&](int q) { return src(q); });
  st.store([&](int q, float v) {
    const int o = q / F, k = q % F;
    Q[(((o / 16) * 2 + k / 16) * 64 + ((k % 16) / 4) * 16 + o % 16) * 4 + k % 4] = v;
  });
}

// P rows of edge c (clamped to a valid row; dead rows are computed and never stored)
__device__ __forceinline__ void load_slabs32(const float* __restrict__ X, int64_t row0, int nrows, f32x4 (&v)[2],
                                             int lane) {
  const int c = lane & 15, g = lane >> 4;
  const float* p = X + (row0 + (c < nrows ? c : 0)) * F + 4 * g;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float4 t = *reinterpret_cast<const float4*>(p + 16 * u);
    v[u] = f32x4{t.x, t.y, t.z, t.w};
  }
}

// ---- the LayerNorm of a row held as slabs (lane (g, c): 8 features of row c), in packed fp32 math
// (round 5): v_pk_add / v_pk_mul / v_pk_fma handle two features per instruction (the compiler does
// not pair these on its own), so the statistics and the affine take about half the VALU.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pair(const f32x4& v, int h) { return h ? f32x2{v[2], v[3]} : f32x2{v[0], v[1]}; }
__device__ __forceinline__ void set_pair(f32x4& v, int h, f32x2 x) {
  v[2 * h] = x.x;
  v[2 * h + 1] = x.y;
}
// centres v in place (v - mean over the row's 32 features) and returns rstd
__device__ __forceinline__ float ln_center(f32x4 (&v)[2], float eps) {
  const f32x2 s2 = (pair(v[0], 0) + pair(v[0], 1)) + (pair(v[1], 0) + pair(v[1], 1));
  const float mean = xsum32(xsum16(s2.x + s2.y)) * (1.f / F);
  const f32x2 m2 = {mean, mean};
  f32x2 q2 = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 d = pair(v[u], h) - m2;
      q2 = __builtin_elementwise_fma(d, d, q2);
      set_pair(v[u], h, d);
    }
  return rsq_normal(xsum32(xsum16(q2.x + q2.y)) * (1.f / F) + eps);
}
// out = relu(d rstd gamma + beta) for the centred slabs d (xh = d rstd also returned when asked)
__device__ __forceinline__ void ln_affine(const f32x4 (&d)[2], float rstd, const float (&g8)[2][4],
                                          const float (&b8)[2][4], f32x4 (&out)[2], f32x4* xh = nullptr) {
  const f32x2 r2 = {rstd, rstd};
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 x = pair(d[u], h) * r2;
      const f32x2 y = __builtin_elementwise_fma(x, f32x2{g8[u][2 * h], g8[u][2 * h + 1]},
                                                f32x2{b8[u][2 * h], b8[u][2 * h + 1]});
      if (xh) set_pair(xh[u], h, x);
      out[u][2 * h] = fmaxf(y.x, 0.f);
      out[u][2 * h + 1] = fmaxf(y.y, 0.f);
    }
}

// relu(LN(P)) (LN) or P (the final update) in place on the slabs; g8 / b8: gamma / beta at this
// lane's features 16 u + 4 g + j
template <bool LN>
__device__ __forceinline__ void phat_slabs(f32x4 (&v)[2], const float (&g8)[2][4], const float (&b8)[2][4],
                                           float eps) {
  if (!LN) return;
  const float rstd = ln_center(v, eps);
  ln_affine(v, rstd, g8, b8, v);
}

// acc[ot] += W P_hat^T (A = W slabs, B = P_hat slabs): acc[ot][r] = feature 16 ot + 4 g + r of edge c
template <int OT>
__device__ __forceinline__ void xl_slabs(const float4* __restrict__ Q, const f32x4 (&x)[2], f32x4 (&acc)[OT],
                                         int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float4 w[OT];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) w[ot] = Q[(ot * 2 + u) * 64 + lane];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].x, x[u][0], acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].y, x[u][1], acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].z, x[u][2], acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].w, x[u][3], acc[ot]);
  }
}

}  // namespace
}  // namespace gasfm
