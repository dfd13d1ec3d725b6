// Edge prologue with the CAMERA-direction GATv2 attention fused in, and the camera attention's
// backward recomputing its source rows, gfx950.
//
// A block's edge prologue computes both convs' lin_l on P_hat = relu(LN(P)) (layers.py:232-234;
// PyG's lin_l) -- XL = [XLp | XLc], 32 + 32 features per edge -- and the camera direction's
// attention (Proj2View, layers.py:329-335) then reduces XLc over each camera's edges.  The edges
// are camera-major, so a camera segment is a contiguous run of the prologue's own 16-edge tiles:
//
//   edge_cam_fwd   over the camera plan's work items (one camera, <= max_piece edges each):
//                  XLp is written (in point-segment order through pos, as edge_prologue_fwd does)
//                  and XLc is consumed by an online softmax in registers -- never stored.
//   edge_cam_bwd   the camera attention's backward (gat_attn.hip attn_bwd_*): XLc recomputed from
//                  P (LayerNorm + 16 MFMAs per tile) instead of read back, dXLc written for
//                  gasfm_edge_prologue_bwd (which takes the two halves of dXL separately), dXR per
//                  camera, d att / d bias per workgroup.
// HBM per edge and block: the forward writes 256 B less (XLc) and the camera attention's forward
// read of XLc (128 B) is gone; the backward reads P (128 B) where it read XLc (128 B).
//
// MFMA orientation: the TRANSPOSED products XL^T = W P_hat^T (A = W from LDS, B = P_hat^T from the
// wave's LDS tile) leave lane (g = l >> 4, c = l & 15) holding features 16 ot + 4 g + r (r < 4) of
// EDGE c: one edge per lane column.  A head (8 features) is then 4 of the lane's registers plus
// the same 4 of lane l ^ 16, the per-edge softmax state is one per lane and head, and a lane's
// XLp / dXLc features are one float4 store per 16-feature tile (a row is 8 lanes x 16 B).
//
// Semantics are those of gasfm_gat_attn_fwd / _bwd on the camera plan: complete items write
// out[seg] (finalized with bias, or the raw acc), split items packed partial rows [acc 32 | max 4 |
// sum 4] for gasfm_gat_attn_combine; empty segments give out = bias, max = -inf, sum = 0; d bias
// sums gout over every segment (once, at its first item).
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

__device__ __forceinline__ float leaky(float z, float slope) { return z > 0.f ? z : z * slope; }

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
      rstd = rsqrtf(group_sum<8>(q) * (1.f / F) + eps);
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

// relu(LN(P)) (LN) or P (the final update) in place on the slabs; g8 / b8: gamma / beta at this
// lane's features 16 u + 4 g + j
template <bool LN>
__device__ __forceinline__ void phat_slabs(f32x4 (&v)[2], const float (&g8)[2][4], const float (&b8)[2][4],
                                           float eps) {
  if (!LN) return;
  float sm = (v[0][0] + v[0][1]) + (v[0][2] + v[0][3]) + ((v[1][0] + v[1][1]) + (v[1][2] + v[1][3]));
  sm += __shfl_xor(sm, 16);
  sm += __shfl_xor(sm, 32);
  const float mean = sm * (1.f / F);
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) q = fmaf(v[u][j] - mean, v[u][j] - mean, q);
  q += __shfl_xor(q, 16);
  q += __shfl_xor(q, 32);
  const float rstd = rsqrtf(q * (1.f / F) + eps);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[u][j] = fmaxf(fmaf((v[u][j] - mean) * rstd, g8[u][j], b8[u][j]), 0.f);
}

// phat_slabs that also returns the row statistics (mean, rstd of edge c; 0 / 1 without LN)
template <bool LN>
__device__ __forceinline__ void phat_slabs_st(f32x4 (&v)[2], const float (&g8)[2][4], const float (&b8)[2][4],
                                              float eps, float& mean, float& rstd) {
  mean = 0.f;
  rstd = 1.f;
  if (!LN) return;
  float sm = (v[0][0] + v[0][1]) + (v[0][2] + v[0][3]) + ((v[1][0] + v[1][1]) + (v[1][2] + v[1][3]));
  sm += __shfl_xor(sm, 16);
  sm += __shfl_xor(sm, 32);
  mean = sm * (1.f / F);
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) q = fmaf(v[u][j] - mean, v[u][j] - mean, q);
  q += __shfl_xor(q, 16);
  q += __shfl_xor(q, 32);
  rstd = rsqrtf(q * (1.f / F) + eps);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[u][j] = fmaxf(fmaf((v[u][j] - mean) * rstd, g8[u][j], b8[u][j]), 0.f);
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

// =============================================================================================
// forward
// =============================================================================================
template <bool LN>
__global__ __launch_bounds__(kThreads, GASFM_CAM_MINW) void edge_cam_fwd_kernel(
    const float* __restrict__ P, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ bpt, const float* __restrict__ Wc,
    const float* __restrict__ bc, float* __restrict__ XLp, int64_t ldXLp, const int32_t* __restrict__ pos,
    const float* __restrict__ XR, int64_t ldXR, const float* __restrict__ att, const float* __restrict__ bias,
    float slope, const gasfm_work_item* __restrict__ items, int n_items, int finalize, float* __restrict__ out,
    int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float Wl[kCamR ? NX * F : NX * LDA];  // slabs, or Wl[n][k] = [Wpt; Wc][n][k]
  __shared__ float tiles[kCamR ? 1 : kWaves][TR * LD34];
  if (kCamR) {
    stage_slabs32<NX, kThreads>([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; }, Wl);
  } else {
    Stage<NX * F, kThreads> sw;
    sw.load([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; });
    sw.store([&](int q, float v) { Wl[(q / F) * LDA + q % F] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T = tiles[kCamR ? 0 : wave];
  float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float g8[2][4], b8[2][4];  // gamma / beta at the slab features 16 u + 4 g + j
  if (LN) {
    g4 = *reinterpret_cast<const float4*>(gam + (lane & 7) * 4);
    b4 = *reinterpret_cast<const float4*>(bet + (lane & 7) * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g8[u][j] = gam[16 * u + 4 * g + j];
        b8[u][j] = bet[16 * u + 4 * g + j];
      }
  }
  // this lane's features: point 16 ot + 4 g + r (ot = 0, 1); camera 16 q + 4 g + r (q = 0, 1),
  // head 2 q + (g >> 1)
  float bp[2][4], bcv[2][4], attv[2][4], biasv[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * q + 4 * g + r;
      bp[q][r] = bpt[f];
      bcv[q][r] = bc[f];
      attv[q][r] = att[f];
      biasv[q][r] = finalize ? bias[f] : 0.f;
    }
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;

  float4 np[2];
  f32x4 ns[2];
  int32_t npos = 0;  // point-order row of this lane's edge (column c)
  // branch-free: without pos the index load reads P's first words and is not used (a load under a
  // branch makes the join wait for every load in flight)
  const int32_t* posp = pos ? pos : reinterpret_cast<const int32_t*>(P);
  auto issue = [&](int64_t row0, int nrows) {
    if (kCamR)
      load_slabs32(P, row0, nrows, ns, lane);
    else
      load_rows(P, F, row0, nrows, np, lane);
    npos = posp[row0 + (c < nrows ? c : 0)];
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };

  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) issue(w.begin, rows_at(w, w.begin));
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    float xr[2][4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(XR + seg * ldXR + 16 * q + 4 * g);
      xr[q][0] = v.x, xr[q][1] = v.y, xr[q][2] = v.z, xr[q][3] = v.w;
    }
    float m[2] = {-INFINITY, -INFINITY}, s[2] = {0.f, 0.f};
    float a[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) issue(wn.begin, rows_at(wn, wn.begin));
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 ph[2] = {ns[0], ns[1]};
      if (!kCamR) phat_to_lds<LN>(np, nrows, g4, b4, eps, T, lane);
      const int64_t dst = pos ? int64_t(npos) : row0 + (c < nrows ? c : 0);
      {  // the next tile (this item's, else the next item's first; the last one re-reads itself)
        int64_t r1 = row0;
        int n1 = nrows;
        if (row0 + TR < w.end) {
          r1 = row0 + TR;
          n1 = rows_at(w, r1);
        } else if (more && wn.begin < wn.end) {
          r1 = wn.begin;
          n1 = rows_at(wn, r1);
        }
        issue(r1, n1);
      }
      f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
      if (kCamR) {
        phat_slabs<LN>(ph, g8, b8, eps);
        xl_slabs<4>(reinterpret_cast<const float4*>(Wl), ph, acc, lane);
      } else {
        wave_sync();
        xl_t<4>(Wl, T, acc, c, g);
      }
      const bool valid = c < nrows;
      // point half: this lane's 2 x 4 features of edge c (non-temporal: streamed once by the point
      // attention)
      if (valid) {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int ot = 0; ot < 2; ++ot)
          __builtin_nontemporal_store(v4f{acc[ot][0] + bp[ot][0], acc[ot][1] + bp[ot][1], acc[ot][2] + bp[ot][2],
                                          acc[ot][3] + bp[ot][3]},
                                      reinterpret_cast<v4f*>(XLp + dst * ldXLp + 16 * ot + 4 * g));
      }
      // camera half: logits of edge c, online softmax per head
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float xl[4], p = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = acc[2 + q][r] + bcv[q][r];
          p = fmaf(leaky(xl[r] + xr[q][r], slope), attv[q][r], p);
        }
        p += __shfl_xor(p, 16);  // the head's other 4 features
        if (valid) {
          const float mn = fmaxf(m[q], p);
          const float sc = __expf(m[q] - mn), wt = __expf(p - mn);
          s[q] = fmaf(s[q], sc, wt);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[q][r] = fmaf(a[q][r], sc, wt * xl[r]);
          m[q] = mn;
        }
      }
      if (!kCamR) wave_sync();  // T is rewritten by the next tile
    }
    // merge the 16 edge columns' states
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float M = row_max16(m[q]);
      const float f = (m[q] > -INFINITY) ? __expf(m[q] - M) : 0.f;
      const float S = group_sum<16>(s[q] * f);
      float A[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) A[r] = group_sum<16>(a[q][r] * f);
      if (c == 0) {
        const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
        if (w.slot < 0) {
          const float inv = 1.f / (S + 1e-16f);
          float4 o;
          if (finalize)
            o = make_float4(fmaf(A[0], inv, biasv[q][0]), fmaf(A[1], inv, biasv[q][1]), fmaf(A[2], inv, biasv[q][2]),
                            fmaf(A[3], inv, biasv[q][3]));
          else
            o = make_float4(A[0], A[1], A[2], A[3]);
          *reinterpret_cast<float4*>(out + seg * ldOut + f0) = o;
          if ((g & 1) == 0) {
            seg_max[seg * ldStat + h] = M;
            seg_sum[seg * ldStat + h] = S;
          }
        } else {
          float* pr = part + int64_t(w.slot) * PART;
          *reinterpret_cast<float4*>(pr + f0) = make_float4(A[0], A[1], A[2], A[3]);
          if ((g & 1) == 0) {
            pr[F + h] = M;
            pr[F + H + h] = S;
          }
        }
      }
    }
    w = wn;
  }
}

// =============================================================================================
// forward seam: block b's edge epilogue + block b+1's prologue and camera attention in one pass
// (gasfm_edge_seam_fwd).  Per 16-edge tile of the camera plan's items (edge c on lane column c):
//   P_hat_b = relu(LN_b(P_b)),  Y = Wp_b[:, :32] P_hat_b^T                      (T layout, MFMA)
//   P' = P_b + scale (Y + bp + Sg + Wp_b[:, 32:34] P0 + Sp[pt] + Sv[cam])       stored
//   then exactly edge_cam_fwd on P' (LN_{b+1}, XL, point half stored, camera softmax).
// Replaces edge_epilogue_fwd + edge_cam_fwd: P' is never read back (128 B per edge), and the
// camera of a camera item is fixed, so Sv[cam] is one row per item.  Per-feature vectors live in
// LDS (read as float4 at the lane's features 16 q + 4 g .. + 3).
// =============================================================================================
struct SeamEpi {
  const float* P;     // P_b [E, 32]
  const float* P0;    // [E, 2] or null
  const int32_t* pt;  // point of each edge
  const float* gam;   // LN_b
  const float* bet;
  float eps;
  const float* Wp;    // [32 x ldWp]
  int ldWp;
  const float* bp;
  const float* Sp;    // [n, 32]
  const float* Sv;    // [m, ldSv]
  int64_t ldSv;
  const float* Sg;    // [32]
  float scale;
  float* Pout;        // P' [E, 32]
  // block 0's epilogue (EP0): P [E, 2], gam / bet = LN_a, Wp [32 x 2], and
  const float* gb;    // LN_b [2]
  const float* bb;
  const float* Wsk;   // skip projection [32 x 2]
  const float* bsk;   // [32]
  float* XLc;         // (XS, round 4 experiment) block b+1's XLc [E, 32] in edge order, or null
};

#ifndef GASFM_SEAM_MINW
#define GASFM_SEAM_MINW 2
#endif
// 1: no per-tile branches.  A lane past the item's end computes the item's first edge (its loads
// read that row), so its P' / XL stores go to that edge's rows with the same values (duplicate,
// identical writes), and its softmax update is a select.  0 (default): guarded stores and update.
// tools/edge_bench.py, same box: 468-472 us with 1 vs 454-459 with 0 (the branch-free form of
// edge_cam_pbwd, GASFM_PBWD_V2, gained 5 %: 645-649 vs 683-692 us).
#ifndef GASFM_SEAM_V2
#define GASFM_SEAM_V2 0
#endif
// 1: the Sp[pt] rows of the next tile are gathered half a tile ahead (issued after this tile's P'
// store, from the next tile's point indices, which are loaded first of the next tile's requests);
// 0: gathered at the start of their own tile, hidden only behind LN_b and the epilogue product.
#ifndef GASFM_SEAM_SPPF
#define GASFM_SEAM_SPPF 1
#endif
// 1: the P' and XL stores are unconditional (a lane past the item's end rewrites its clamped row
// with that row's own values, as in GASFM_SEAM_V2), so no store sits under a branch and the
// compiler's vmcnt bookkeeping stays exact (a store under a branch makes every later wait assume
// the store-free path, i.e. wait for younger loads too)
#ifndef GASFM_SEAM_UST
#define GASFM_SEAM_UST 1
#endif
// EP0: block 0's epilogue (edge0_epilogue_fwd, 2-wide P) as the seam's first half:
//   P' = Wsk relu(LN_b(P)) + bsk + scale (Wp relu(LN_a(P)) + bp + Sg + Sp[pt] + Sv[cam])
// computed per lane on its 8 features (2-wide products: no MFMA), in edge0_epilogue_fwd's order.
// 1: the seam's work items dealt so that the workgroups of one XCD (blocks b = x mod 8) take
// contiguous item ranges: at any time an XCD's resident waves cover ~16 consecutive cameras, so its
// L2 holds their point windows' Sp rows instead of those of ~130 cameras spread over all 8 XCDs
// (round 4; the Sp[pt] gathers in camera order are the seam's 1.15x traffic).  The items and their
// outputs are the same either way.
#ifndef GASFM_SEAM_XCD
#define GASFM_SEAM_XCD 0
#endif
#ifndef GASFM_SEAM_PRIO
#define GASFM_SEAM_PRIO 0
#endif
template <bool LN, bool EP0, bool XS = false>
__global__ __launch_bounds__(kThreads, GASFM_SEAM_MINW) void edge_seam_fwd_kernel(
    SeamEpi ep, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ bpt, const float* __restrict__ Wc,
    const float* __restrict__ bc, float* __restrict__ XLp, int64_t ldXLp, const int32_t* __restrict__ pos,
    const float* __restrict__ XR, int64_t ldXR, const float* __restrict__ att, const float* __restrict__ bias,
    float slope, const gasfm_work_item* __restrict__ items, int n_items, int finalize, float* __restrict__ out,
    int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  // vector table (32 floats each): 0 gamma_b 1 beta_b 2 bp+Sg 3 Wp[:,32] 4 Wp[:,33] 5 gamma 6 beta
  // 7 bpt 8 bc 9 att 10 bias; EP0: 0 Wsk[:,0] 1 Wsk[:,1] 2 bp+Sg 3 Wp[:,0] 4 Wp[:,1] 11 bsk
  __shared__ __attribute__((aligned(16))) float Wl[NX * F];   // [Wpt; Wc] slabs
  __shared__ __attribute__((aligned(16))) float WpQ[EP0 ? 4 : F * F];  // Wp_b[:, :32] slabs
  __shared__ __attribute__((aligned(16))) float V[12 * F];
  stage_slabs32<NX, kThreads>([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; }, Wl);
  if (!EP0) stage_slabs32<F, kThreads>([&](int q) { return ep.Wp[(q / F) * ep.ldWp + q % F]; }, WpQ);
  if (threadIdx.x < F) {
    const int f = threadIdx.x;
    V[f] = EP0 ? ep.Wsk[2 * f] : ep.gam[f];
    V[F + f] = EP0 ? ep.Wsk[2 * f + 1] : ep.bet[f];
    V[2 * F + f] = ep.bp[f] + ep.Sg[f];
    V[3 * F + f] = EP0 ? ep.Wp[2 * f] : (ep.P0 ? ep.Wp[f * ep.ldWp + 32] : 0.f);
    V[4 * F + f] = EP0 ? ep.Wp[2 * f + 1] : (ep.P0 ? ep.Wp[f * ep.ldWp + 33] : 0.f);
    V[11 * F + f] = EP0 ? ep.bsk[f] : 0.f;
    V[5 * F + f] = LN ? gam[f] : 1.f;
    V[6 * F + f] = LN ? bet[f] : 0.f;
    V[7 * F + f] = bpt[f];
    V[8 * F + f] = bc[f];
    V[9 * F + f] = att[f];
    V[10 * F + f] = finalize ? bias[f] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  // (EP0) LN_a and LN_b over the 2 input features
  const float ga0 = EP0 ? ep.gam[0] : 0.f, ga1 = EP0 ? ep.gam[1] : 0.f, ba0 = EP0 ? ep.bet[0] : 0.f,
              ba1 = EP0 ? ep.bet[1] : 0.f, gb0 = EP0 ? ep.gb[0] : 0.f, gb1 = EP0 ? ep.gb[1] : 0.f,
              bb0 = EP0 ? ep.bb[0] : 0.f, bb1 = EP0 ? ep.bb[1] : 0.f;
  auto vec = [&](int which, int q) {
    const float4 t = *reinterpret_cast<const float4*>(V + which * F + 16 * q + 4 * g);
    return f32x4{t.x, t.y, t.z, t.w};
  };
  const int bx = (GASFM_SEAM_XCD && gridDim.x % 8 == 0)
                     ? int(blockIdx.x % 8) * int(gridDim.x / 8) + int(blockIdx.x / 8) : int(blockIdx.x);
  const int gw = bx * kWaves + wave, nw = gridDim.x * kWaves;
  if (GASFM_SEAM_PRIO && blockIdx.x >= gridDim.x / 2) __builtin_amdgcn_s_setprio(1);  // as GASFM_PBWD_PRIO
  // next tile: P_b slabs, the edge's point and P0 pair, its point-order row (all branch-free)
  f32x4 ns[2];
  int32_t npos = 0, npt = 0;
  float2 nq = make_float2(0.f, 0.f);
  const int32_t* posp = pos ? pos : reinterpret_cast<const int32_t*>(ep.P);
  const float* p0p = EP0 ? ep.P : (ep.P0 ? ep.P0 : ep.P);  // EP0: the 2-wide P row itself
  f32x4 nsp[2];  // GASFM_SEAM_SPPF: Sp[pt] of the next tile
  auto issue = [&](int64_t row0, int nrows) {
    const int64_t e = row0 + (c < nrows ? c : 0);
    if (GASFM_SEAM_SPPF) npt = ep.pt[e];  // first: waiting for it does not wait for the P rows
    if (!EP0) load_slabs32(ep.P, row0, nrows, ns, lane);
    npos = posp[e];
    if (!GASFM_SEAM_SPPF) npt = ep.pt[e];
    nq = *reinterpret_cast<const float2*>(p0p + e * 2);
  };
  auto issue_sp = [&]() {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 t = *reinterpret_cast<const float4*>(ep.Sp + int64_t(npt) * F + 16 * q + 4 * g);
      nsp[q] = f32x4{t.x, t.y, t.z, t.w};
    }
  };
  // an item's first tile outside the tile loop: the Sp rows before the P rows, so that (as on the
  // loop's own path, where the tile's stores follow them) younger requests follow the Sp rows when
  // the loop is entered -- the compiler's wait counts are the minimum over the entering paths
  auto issue_first = [&](int64_t row0, int nrows) {
    if (GASFM_SEAM_SPPF) {
      npt = ep.pt[row0 + (c < nrows ? c : 0)];
      issue_sp();
    }
    issue(row0, nrows);
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };

  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) {
      issue_first(w.begin, rows_at(w, w.begin));
    }
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    f32x4 xr[2], sv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(XR + seg * ldXR + 16 * q + 4 * g);
      xr[q] = f32x4{v.x, v.y, v.z, v.w};
      const float4 t = *reinterpret_cast<const float4*>(ep.Sv + seg * ep.ldSv + 16 * q + 4 * g);
      sv[q] = f32x4{t.x, t.y, t.z, t.w};
    }
    float m[2] = {-INFINITY, -INFINITY}, s[2] = {0.f, 0.f};
    f32x4 a[2] = {zero4(), zero4()};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) {
      issue_first(wn.begin, rows_at(wn, wn.begin));
    }
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 pb[2] = {ns[0], ns[1]};
      f32x4 sp[2];
      if (GASFM_SEAM_SPPF) {
        sp[0] = nsp[0];
        sp[1] = nsp[1];
      }
      // lanes past the item's end hold row0's values (clamped loads) and store them to row0's own
      // row: with pos == nullptr, row0 + c would belong to the next item (another wave's rows)
      const int64_t dst = pos ? int64_t(npos) : row0 + (c < nrows ? c : 0);
      const int32_t ptc = npt;
      const float2 q0 = nq;
      {  // the next tile (this item's, else the next item's first; the last one re-reads itself)
        int64_t r1 = row0;
        int n1 = nrows;
        if (row0 + TR < w.end) {
          r1 = row0 + TR;
          n1 = rows_at(w, r1);
        } else if (more && wn.begin < wn.end) {
          r1 = wn.begin;
          n1 = rows_at(wn, r1);
        }
        issue(r1, n1);
      }
      if (!GASFM_SEAM_SPPF) {  // Sp[pt] of edge c: its latency overlaps LN_b and the epilogue product
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float4 t = *reinterpret_cast<const float4*>(ep.Sp + int64_t(ptc) * F + 16 * q + 4 * g);
          sp[q] = f32x4{t.x, t.y, t.z, t.w};
        }
      }
      const bool valid = c < nrows;
      // ---- epilogue of block b (T layout)
      f32x4 pn[2];  // P' (this block's output, the next block's input)
      if (EP0) {
        // block 0: 2-wide P (q0), LN_a / LN_b over its 2 features (edge0_epilogue_fwd's order)
        const float mean = 0.5f * (q0.x + q0.y);
        const float d0 = q0.x - mean, d1 = q0.y - mean;
        const float rs = rsqrtf(0.5f * (d0 * d0 + d1 * d1) + ep.eps);
        const float xh0 = d0 * rs, xh1 = d1 * rs;
        const float ha0 = fmaxf(fmaf(xh0, ga0, ba0), 0.f), ha1 = fmaxf(fmaf(xh1, ga1, ba1), 0.f);
        const float hb0 = fmaxf(fmaf(xh0, gb0, bb0), 0.f), hb1 = fmaxf(fmaf(xh1, gb1, bb1), 0.f);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 ka = vec(0, q), kb = vec(1, q), cs = vec(2, q), wa = vec(3, q), wb = vec(4, q), bs = vec(11, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = fmaf(wa[r], ha0, fmaf(wb[r], ha1, cs[r])) + sp[q][r] + sv[q][r];
            pn[q][r] = fmaf(d, ep.scale, fmaf(ka[r], hb0, fmaf(kb[r], hb1, bs[r])));
          }
        }
      } else {
        f32x4 ph[2] = {pb[0], pb[1]};
        {
          float gs[2][4], bs[2][4];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x4 ga = vec(0, q), be = vec(1, q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              gs[q][r] = ga[r];
              bs[q][r] = be[r];
            }
          }
          phat_slabs<true>(ph, gs, bs, ep.eps);
        }
        f32x4 y[2] = {zero4(), zero4()};
        xl_slabs<2>(reinterpret_cast<const float4*>(WpQ), ph, y, lane);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 cs = vec(2, q), w32 = vec(3, q), w33 = vec(4, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float d = y[q][r] + cs[r];
            d = fmaf(w32[r], q0.x, fmaf(w33[r], q0.y, d));
            // (d + Sv) + Sp: the gathered Sp row is consumed last (not hoisted to the tile's top)
            d = GASFM_SEAM_SPPF ? (d + sv[q][r]) + sp[q][r] : d + (sp[q][r] + sv[q][r]);
            pn[q][r] = fmaf(d, ep.scale, pb[q][r]);
          }
        }
      }
      if (GASFM_SEAM_SPPF) {
        // not hoisted towards the point-index load it waits for: the address is formed from npt
        // only once P' exists
        asm volatile("" : "+v"(npt) : "v"(pn[0][0]), "v"(pn[1][3]));
        issue_sp();
      }
      if (GASFM_SEAM_V2 || GASFM_SEAM_UST || valid) {
        const int64_t prow = row0 + (valid ? c : 0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
          *reinterpret_cast<float4*>(ep.Pout + prow * F + 16 * q + 4 * g) =
              make_float4(pn[q][0], pn[q][1], pn[q][2], pn[q][3]);
      }
      // ---- prologue + camera attention of block b+1 on P' (edge_cam_fwd_kernel)
      {
        float gs[2][4], bs[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 ga = vec(5, q), be = vec(6, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gs[q][r] = ga[r];
            bs[q][r] = be[r];
          }
        }
        phat_slabs<LN>(pn, gs, bs, eps);
      }
      f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
      xl_slabs<4>(reinterpret_cast<const float4*>(Wl), pn, acc, lane);
      if (GASFM_SEAM_V2 || GASFM_SEAM_UST || valid) {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
          const f32x4 b = vec(7, ot);
          __builtin_nontemporal_store(v4f{acc[ot][0] + b[0], acc[ot][1] + b[1], acc[ot][2] + b[2], acc[ot][3] + b[3]},
                                      reinterpret_cast<v4f*>(XLp + dst * ldXLp + 16 * ot + 4 * g));
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 bcq = vec(8, q), atq = vec(9, q);
        float xl[4], p = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = acc[2 + q][r] + bcq[r];
          p = fmaf(leaky(xl[r] + xr[q][r], slope), atq[r], p);
        }
        if (XS) {  // XLc kept for edge_cam_pbwd (lanes past the item's end rewrite row0's own values)
          const int64_t xrow = row0 + (valid ? c : 0);
          *reinterpret_cast<float4*>(ep.XLc + xrow * F + 16 * q + 4 * g) = make_float4(xl[0], xl[1], xl[2], xl[3]);
        }
        p += __shfl_xor(p, 16);  // the head's other 4 features
        if (GASFM_SEAM_V2) {
          const float mn = valid ? fmaxf(m[q], p) : m[q];
          const float sc = valid ? __expf(m[q] - mn) : 1.f, wt = valid ? __expf(p - mn) : 0.f;
          s[q] = fmaf(s[q], sc, wt);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[q][r] = fmaf(a[q][r], sc, wt * xl[r]);
          m[q] = mn;
        } else if (valid) {
          const float mn = fmaxf(m[q], p);
          const float sc = __expf(m[q] - mn), wt = __expf(p - mn);
          s[q] = fmaf(s[q], sc, wt);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[q][r] = fmaf(a[q][r], sc, wt * xl[r]);
          m[q] = mn;
        }
      }
    }
    // merge the 16 edge columns' states (edge_cam_fwd_kernel)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float M = row_max16(m[q]);
      const float f = (m[q] > -INFINITY) ? __expf(m[q] - M) : 0.f;
      const float S = group_sum<16>(s[q] * f);
      float A[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) A[r] = group_sum<16>(a[q][r] * f);
      if (c == 0) {
        const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
        if (w.slot < 0) {
          const float inv = 1.f / (S + 1e-16f);
          float4 o;
          if (finalize) {
            const f32x4 bq = vec(10, q);
            o = make_float4(fmaf(A[0], inv, bq[0]), fmaf(A[1], inv, bq[1]), fmaf(A[2], inv, bq[2]),
                            fmaf(A[3], inv, bq[3]));
          } else {
            o = make_float4(A[0], A[1], A[2], A[3]);
          }
          *reinterpret_cast<float4*>(out + seg * ldOut + f0) = o;
          if ((g & 1) == 0) {
            seg_max[seg * ldStat + h] = M;
            seg_sum[seg * ldStat + h] = S;
          }
        } else {
          float* pr = part + int64_t(w.slot) * PART;
          *reinterpret_cast<float4*>(pr + f0) = make_float4(A[0], A[1], A[2], A[3]);
          if ((g & 1) == 0) {
            pr[F + h] = M;
            pr[F + H + h] = S;
          }
        }
      }
    }
    w = wn;
  }
}

// =============================================================================================
// the forward seam with its inputs staged through LDS, two tiles ahead (round 4, GASFM_SEAM_LDS /
// gasfm_tuning_set(GASFM_TUNE_SEAM_LDS);
// blocks 1-11, not block 0's EP0 form).  edge_seam_fwd_kernel holds the next tile's P slabs and
// Sp rows in registers, one tile ahead: ~4 KB in flight per wave at 2 waves / SIMD, about what a
// CU needs for half the HBM rate at the loaded latency, and its memory and MFMA/VALU phases
// add up (453 us for 1.6 GB + 48 MFMA per tile).  Here the loads are direct-to-LDS
// (global_load_lds: no VGPRs held while they fly) in a per-wave ring, in three stages per tile t:
//   I(t+3)  edge indices: pt, pos, P0 pairs (one 4-B load per lane), the item's XR / Sv rows (one)
//   B(t+2)  the Sp[pt] rows of tile t+2 (pt from its I slot, loaded an iteration earlier)
//   A(t+2)  the P rows of tile t+2
// so a tile's P and Sp rows are requested two iterations before use (~8 KB in flight per wave).
// P / Sp rows sit row-major in the slot with their 16-B chunks swizzled (chunk k of row r at
// position k ^ (r & 7)), so the T-layout reads (lane (g, c): row c, chunk 4 u + g) spread over the
// banks.  Every stage issues a fixed number of requests (clamped re-reads past the wave's last
// tile), and the only vector-memory requests in the loop are these and the tile's 4 stores, so
// one s_waitcnt vmcnt(8) at the top of a tile (vmcnt(4) for the first) covers the tile's slots
// and the I slot the B stage reads next; the work items are scalar loads (lgkmcnt).
// The arithmetic is edge_seam_fwd_kernel's, line for line (outputs bitwise equal).
// =============================================================================================
constexpr int SL_PS = 3;                    // P / Sp ring slots per wave
constexpr int SL_IX = 4;                    // index ring slots per wave
constexpr int SL_PSF = 2 * TR * F;          // floats per P / Sp slot (P rows, then Sp rows)
constexpr int SL_IXF = 128;                 // dwords per index slot
constexpr int SL_WAVE = SL_PS * SL_PSF + SL_IX * SL_IXF;  // floats per wave
constexpr size_t SL_DYN = size_t(kWaves) * SL_WAVE * sizeof(float);

__device__ __forceinline__ gasfm_work_item item_s(const gasfm_work_item* __restrict__ items, int it) {
  // wave-uniform index -> scalar loads
  const gasfm_work_item w = items[__builtin_amdgcn_readfirstlane(it)];
  return uniform_item(w);
}

// LDS reads of the seam's DMA ring through inline asm: the compiler waits for every LDS-DMA
// request before a read it sees of the same LDS object (it cannot tell the ring's slots apart),
// which would drain the two-tile prefetch each tile; these reads are ordered by the kernel's own
// s_waitcnt vmcnt instead, and wait for themselves (lgkmcnt(0)) before their results are used
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}
__device__ __forceinline__ void lds_tile_reads(const float* pa, const float* pb, const float* sa, const float* sb,
                                               const float* q, const float* ps, f32x4& P0, f32x4& P1, f32x4& S0,
                                               f32x4& S1, f32x2v& Q, int& pos) {
  asm volatile(
      "ds_read_b128 %0, %6\n"
      "ds_read_b128 %1, %7\n"
      "ds_read_b128 %2, %8\n"
      "ds_read_b128 %3, %9\n"
      "ds_read_b64 %4, %10\n"
      "ds_read_b32 %5, %11\n"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(P0), "=&v"(P1), "=&v"(S0), "=&v"(S1), "=&v"(Q), "=&v"(pos)
      : "v"(lds_off(pa)), "v"(lds_off(pb)), "v"(lds_off(sa)), "v"(lds_off(sb)), "v"(lds_off(q)), "v"(lds_off(ps))
      : "memory");
}
__device__ __forceinline__ void lds_read4x4(const float* a, const float* b, const float* c2, const float* d,
                                            f32x4& A, f32x4& B, f32x4& C, f32x4& D) {
  asm volatile(
      "ds_read_b128 %0, %4\n"
      "ds_read_b128 %1, %5\n"
      "ds_read_b128 %2, %6\n"
      "ds_read_b128 %3, %7\n"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(A), "=&v"(B), "=&v"(C), "=&v"(D)
      : "v"(lds_off(a)), "v"(lds_off(b)), "v"(lds_off(c2)), "v"(lds_off(d))
      : "memory");
}
__device__ __forceinline__ void lds_read2i(const int32_t* a, const int32_t* b, int& A, int& B) {
  asm volatile(
      "ds_read_b32 %0, %2\n"
      "ds_read_b32 %1, %3\n"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(A), "=&v"(B)
      : "v"(lds_off(a)), "v"(lds_off(b))
      : "memory");
}

template <bool LN>
__global__ __launch_bounds__(kThreads, 2) void edge_seam_lds_kernel(
    SeamEpi ep, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ bpt, const float* __restrict__ Wc,
    const float* __restrict__ bc, float* __restrict__ XLp, int64_t ldXLp, const int32_t* __restrict__ pos,
    const float* __restrict__ XR, int64_t ldXR, const float* __restrict__ att, const float* __restrict__ bias,
    float slope, const gasfm_work_item* __restrict__ items, int n_items, int finalize, float* __restrict__ out,
    int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  typedef __attribute__((address_space(3))) void* lds_vp;
  typedef const __attribute__((address_space(1))) void* glb_vp;
  __shared__ __attribute__((aligned(16))) float Wl[NX * F];
  __shared__ __attribute__((aligned(16))) float WpQ[F * F];
  __shared__ __attribute__((aligned(16))) float V[12 * F];
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  stage_slabs32<NX, kThreads>([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; }, Wl);
  stage_slabs32<F, kThreads>([&](int q) { return ep.Wp[(q / F) * ep.ldWp + q % F]; }, WpQ);
  if (threadIdx.x < F) {
    const int f = threadIdx.x;
    V[f] = ep.gam[f];
    V[F + f] = ep.bet[f];
    V[2 * F + f] = ep.bp[f] + ep.Sg[f];
    V[3 * F + f] = ep.P0 ? ep.Wp[f * ep.ldWp + 32] : 0.f;
    V[4 * F + f] = ep.P0 ? ep.Wp[f * ep.ldWp + 33] : 0.f;
    V[5 * F + f] = LN ? gam[f] : 1.f;
    V[6 * F + f] = LN ? bet[f] : 0.f;
    V[7 * F + f] = bpt[f];
    V[8 * F + f] = bc[f];
    V[9 * F + f] = att[f];
    V[10 * F + f] = finalize ? bias[f] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  auto vec = [&](int which, int q) {
    const float4 t = *reinterpret_cast<const float4*>(V + which * F + 16 * q + 4 * g);
    return f32x4{t.x, t.y, t.z, t.w};
  };
  float* ring = dyn + wave * SL_WAVE;         // P / Sp slots
  float* ixr = ring + SL_PS * SL_PSF;         // index slots
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;
  const float* p0src = ep.P0 ? ep.P0 : ep.P;  // a dummy (finite) read of P without P0
  const int32_t* possrc = pos ? pos : ep.pt;

  // a walker over this wave's tiles (items gw, gw + nw, ...; empty items have none); past the last
  // tile it stays on it (its stages then re-read that tile)
  struct Walk {
    int it;
    gasfm_work_item w;
    int64_t row0;
  };
  auto walk_init = [&](Walk& k) {
    k.it = gw;
    k.row0 = 0;
    k.w = gasfm_work_item{0, 0, 0, -1};
    while (k.it < n_items) {
      k.w = item_s(items, k.it);
      if (k.w.begin < k.w.end) {
        k.row0 = k.w.begin;
        return;
      }
      k.it += nw;
    }
  };
  auto walk_next = [&](Walk& k) {
    if (k.it >= n_items) return;
    if (k.row0 + TR < k.w.end) {
      k.row0 += TR;
      return;
    }
    int it2 = k.it + nw;
    while (it2 < n_items) {
      const gasfm_work_item w2 = item_s(items, it2);
      if (w2.begin < w2.end) {
        k.it = it2;
        k.w = w2;
        k.row0 = w2.begin;
        return;
      }
      it2 += nw;
    }
  };
  auto walk_rows = [](const Walk& k) { return int(k.w.end - k.row0 < TR ? k.w.end - k.row0 : TR); };
  // I stage of the walker's tile into index slot s (2 requests)
  // (a wave without any tile issues nothing: its walkers never had a tile to stay on)
  auto stage_i = [&](const Walk& k, int s) {
    if (k.w.begin >= k.w.end) return;
    float* ix = ixr + s * SL_IXF;
    const int nr = walk_rows(k);
    const int rr = (lane & 15) < nr ? (lane & 15) : 0;
    const int64_t e = k.row0 + rr;
    const void* src;
    if (lane < 16)
      src = ep.pt + e;
    else if (lane < 32)
      src = possrc + e;
    else
      src = p0src + (k.row0 + ((lane - 32) >> 1 < nr ? (lane - 32) >> 1 : 0)) * 2 + (lane & 1);
    __builtin_amdgcn_global_load_lds((glb_vp)src, (lds_vp)ix, 4, 0, 0);
    const int64_t seg = k.w.seg;
    const float* src2 = lane < 32 ? XR + seg * ldXR + lane : ep.Sv + seg * ep.ldSv + (lane - 32);
    __builtin_amdgcn_global_load_lds((glb_vp)src2, (lds_vp)(ix + 64), 4, 0, 0);
  };
  // A / B stages of the walker's tile into P / Sp slot s (2 + 2 requests); pt from index slot si
  auto stage_ab = [&](const Walk& k, int s, int si) {
    if (k.w.begin >= k.w.end) return;
    float* ps = ring + s * SL_PSF;
    const int32_t* ix = reinterpret_cast<const int32_t*>(ixr + si * SL_IXF);
    const int nr = walk_rows(k);
    int pts[2];  // the rows' points (clamped at their I stage)
    lds_read2i(ix + (lane >> 3), ix + 8 + (lane >> 3), pts[0], pts[1]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = 8 * u + (lane >> 3);
      const int ck = (lane & 7) ^ (row & 7);
      __builtin_amdgcn_global_load_lds((glb_vp)(ep.Sp + int64_t(pts[u]) * F + 4 * ck),
                                       (lds_vp)(ps + TR * F + u * 256), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = 8 * u + (lane >> 3);
      const int ck = (lane & 7) ^ (row & 7);
      const int64_t e = k.row0 + (row < nr ? row : 0);
      __builtin_amdgcn_global_load_lds((glb_vp)(ep.P + e * F + 4 * ck), (lds_vp)(ps + u * 256), 16, 0, 0);
    }
  };
  auto wait_vm = [](auto n) {
    if constexpr (decltype(n)::value == 4)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (decltype(n)::value == 8)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  Walk kI, kA;  // the I stage's walker (3 tiles ahead), the A / B stages' (2 ahead)
  walk_init(kI);
  kA = kI;
  // prologue: I(0), I(1), I(2); wait; B(0) A(0), B(1) A(1)
  stage_i(kI, 0);
  walk_next(kI);
  stage_i(kI, 1);
  walk_next(kI);
  stage_i(kI, 2);
  walk_next(kI);
  wait_vm(std::integral_constant<int, 0>{});
  __builtin_amdgcn_wave_barrier();
  stage_ab(kA, 0, 0);
  walk_next(kA);
  stage_ab(kA, 1, 1);
  walk_next(kA);
  int t = 0;  // this wave's tile counter
  for (int it = gw; it < n_items; it += nw) {
    const gasfm_work_item w = item_s(items, it);
    const int64_t seg = w.seg;
    float m[2] = {-INFINITY, -INFINITY}, s[2] = {0.f, 0.f};
    f32x4 a[2] = {zero4(), zero4()};
    f32x4 xr[2], sv[2];
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR, ++t) {
      const int nrows = int(w.end - row0 < TR ? w.end - row0 : TR);
      if (t == 0)
        wait_vm(std::integral_constant<int, 4>{});
      else
        wait_vm(std::integral_constant<int, 8>{});
      __builtin_amdgcn_wave_barrier();
      const float* ps = ring + (t % SL_PS) * SL_PSF;
      const float* ix = ixr + (t % SL_IX) * SL_IXF;
      f32x4 pb[2], sp[2];
      f32x2v q0v;
      int npos;
      {
        const int k0 = g ^ (c & 7), k1 = (4 + g) ^ (c & 7);
        lds_tile_reads(ps + c * F + 4 * k0, ps + c * F + 4 * k1, ps + TR * F + c * F + 4 * k0,
                       ps + TR * F + c * F + 4 * k1, ix + 32 + 2 * c, ix + 16 + c, pb[0], pb[1], sp[0], sp[1], q0v,
                       npos);
      }
      const float2 q0 = make_float2(q0v[0], q0v[1]);
      if (row0 == w.begin)
        lds_read4x4(ix + 64 + 4 * g, ix + 64 + 16 + 4 * g, ix + 96 + 4 * g, ix + 96 + 16 + 4 * g, xr[0], xr[1], sv[0],
                    sv[1]);
      const int64_t dst = pos ? int64_t(npos) : row0 + (c < nrows ? c : 0);
      // the stages of the tiles ahead (their slots were consumed an iteration ago)
      stage_i(kI, (t + 3) % SL_IX);
      walk_next(kI);
      stage_ab(kA, (t + 2) % SL_PS, (t + 2) % SL_IX);
      walk_next(kA);
      const bool valid = c < nrows;
      // ---- epilogue of block b (T layout): edge_seam_fwd_kernel's
      f32x4 pn[2];
      {
        f32x4 ph[2] = {pb[0], pb[1]};
        float gs[2][4], bs[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 ga = vec(0, q), be = vec(1, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gs[q][r] = ga[r];
            bs[q][r] = be[r];
          }
        }
        phat_slabs<true>(ph, gs, bs, ep.eps);
        f32x4 y[2] = {zero4(), zero4()};
        xl_slabs<2>(reinterpret_cast<const float4*>(WpQ), ph, y, lane);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 cs = vec(2, q), w32 = vec(3, q), w33 = vec(4, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float d = y[q][r] + cs[r];
            d = fmaf(w32[r], q0.x, fmaf(w33[r], q0.y, d));
            d = (d + sv[q][r]) + sp[q][r];
            pn[q][r] = fmaf(d, ep.scale, pb[q][r]);
          }
        }
      }
      {
        const int64_t prow = row0 + (valid ? c : 0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
          *reinterpret_cast<float4*>(ep.Pout + prow * F + 16 * q + 4 * g) =
              make_float4(pn[q][0], pn[q][1], pn[q][2], pn[q][3]);
      }
      // ---- prologue + camera attention of block b+1 on P'
      {
        float gs[2][4], bs[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 ga = vec(5, q), be = vec(6, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gs[q][r] = ga[r];
            bs[q][r] = be[r];
          }
        }
        phat_slabs<LN>(pn, gs, bs, eps);
      }
      f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
      xl_slabs<4>(reinterpret_cast<const float4*>(Wl), pn, acc, lane);
      {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
          const f32x4 b = vec(7, ot);
          __builtin_nontemporal_store(v4f{acc[ot][0] + b[0], acc[ot][1] + b[1], acc[ot][2] + b[2], acc[ot][3] + b[3]},
                                      reinterpret_cast<v4f*>(XLp + dst * ldXLp + 16 * ot + 4 * g));
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 bcq = vec(8, q), atq = vec(9, q);
        float xl[4], p = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = acc[2 + q][r] + bcq[r];
          p = fmaf(leaky(xl[r] + xr[q][r], slope), atq[r], p);
        }
        p += __shfl_xor(p, 16);
        if (valid) {
          const float mn = fmaxf(m[q], p);
          const float sc = __expf(m[q] - mn), wt = __expf(p - mn);
          s[q] = fmaf(s[q], sc, wt);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[q][r] = fmaf(a[q][r], sc, wt * xl[r]);
          m[q] = mn;
        }
      }
      __builtin_amdgcn_wave_barrier();  // this tile's slot reads before a later stage rewrites it
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float M = row_max16(m[q]);
      const float f = (m[q] > -INFINITY) ? __expf(m[q] - M) : 0.f;
      const float S = group_sum<16>(s[q] * f);
      float A[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) A[r] = group_sum<16>(a[q][r] * f);
      if (c == 0) {
        const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
        if (w.slot < 0) {
          const float inv = 1.f / (S + 1e-16f);
          float4 o;
          if (finalize) {
            const f32x4 bq = vec(10, q);
            o = make_float4(fmaf(A[0], inv, bq[0]), fmaf(A[1], inv, bq[1]), fmaf(A[2], inv, bq[2]),
                            fmaf(A[3], inv, bq[3]));
          } else {
            o = make_float4(A[0], A[1], A[2], A[3]);
          }
          *reinterpret_cast<float4*>(out + seg * ldOut + f0) = o;
          if ((g & 1) == 0) {
            seg_max[seg * ldStat + h] = M;
            seg_sum[seg * ldStat + h] = S;
          }
        } else {
          float* pr = part + int64_t(w.slot) * PART;
          *reinterpret_cast<float4*>(pr + f0) = make_float4(A[0], A[1], A[2], A[3]);
          if ((g & 1) == 0) {
            pr[F + h] = M;
            pr[F + H + h] = S;
          }
        }
      }
    }
  }
  wait_vm(std::integral_constant<int, 0>{});  // no LDS-DMA outstanding at the end of the wave
}

// =============================================================================================
// backward of the camera attention, XLc recomputed from P
// =============================================================================================
// per workgroup partial row: [32 datt | 32 dbias]
constexpr int BP_PART = 2 * F;

template <bool LN>
__global__ __launch_bounds__(kThreads, GASFM_CAM_MINW) void edge_cam_bwd_kernel(
    const float* __restrict__ P, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wc, const float* __restrict__ bc, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum, int64_t ldStat,
    const float* __restrict__ gout, int64_t ldG, const gasfm_work_item* __restrict__ items, int n_items,
    float* __restrict__ dXLc, int64_t ldD, float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float Wl[kCamR ? F * F : F * LDA];  // slabs, or Wl[n][k] = Wc[n][k]
  __shared__ float tiles[kWaves][TR * LD34];  // (also the final reduction's scratch)
  if (kCamR) {
    stage_slabs32<F, kThreads>([&](int q) { return Wc[q]; }, Wl);
  } else {
    Stage<F * F, kThreads> sw;
    sw.load([&](int q) { return Wc[q]; });
    sw.store([&](int q, float v) { Wl[(q / F) * LDA + q % F] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T = tiles[wave];
  float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float g8[2][4], b8[2][4];  // gamma / beta at the slab features 16 u + 4 g + j
  if (LN) {
    g4 = *reinterpret_cast<const float4*>(gam + (lane & 7) * 4);
    b4 = *reinterpret_cast<const float4*>(bet + (lane & 7) * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g8[u][j] = gam[16 * u + 4 * g + j];
        b8[u][j] = bet[16 * u + 4 * g + j];
      }
  }
  float bcv[2][4], attv[2][4], biasv[2][4], datt[2][4], dbias[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * q + 4 * g + r;
      bcv[q][r] = bc[f];
      attv[q][r] = att[f];
      biasv[q][r] = bias[f];
      datt[q][r] = dbias[q][r] = 0.f;
    }
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;

  float4 np[2];
  f32x4 ns[2];
  auto issue = [&](int64_t row0, int nrows) {
    if (kCamR)
      load_slabs32(P, row0, nrows, ns, lane);
    else
      load_rows(P, F, row0, nrows, np, lane);
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };
  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) issue(w.begin, rows_at(w, w.begin));
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    // per-camera constants: XR, gout, out - bias at this lane's features; per head the forward's
    // max, 1 / (sum + 1e-16) and delta = sum_j alpha_j (g . XL_j) = g . (out - bias)
    float xr[2][4], gv[2][4], M[2], inv[2], delta[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
      const float4 x4 = *reinterpret_cast<const float4*>(XR + seg * ldXR + f0);
      const float4 g4v = *reinterpret_cast<const float4*>(gout + seg * ldG + f0);
      const float4 o4 = *reinterpret_cast<const float4*>(out + seg * ldOut + f0);
      xr[q][0] = x4.x, xr[q][1] = x4.y, xr[q][2] = x4.z, xr[q][3] = x4.w;
      gv[q][0] = g4v.x, gv[q][1] = g4v.y, gv[q][2] = g4v.z, gv[q][3] = g4v.w;
      const float o[4] = {o4.x, o4.y, o4.z, o4.w};
      float d = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) d = fmaf(gv[q][r], o[r] - biasv[q][r], d);
      delta[q] = d + __shfl_xor(d, 16);
      M[q] = seg_max[seg * ldStat + h];
      inv[q] = 1.f / (seg_sum[seg * ldStat + h] + 1e-16f);
    }
    const bool first = it == 0 || items[it - 1].seg != w.seg;
    if (first && c == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) dbias[q][r] += gv[q][r];
    }
    float dxr[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) issue(wn.begin, rows_at(wn, wn.begin));
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 ph[2] = {ns[0], ns[1]};
      if (!kCamR) phat_to_lds<LN>(np, nrows, g4, b4, eps, T, lane);
      {  // the next tile (see edge_cam_fwd_kernel)
        int64_t r1 = row0;
        int n1 = nrows;
        if (row0 + TR < w.end) {
          r1 = row0 + TR;
          n1 = rows_at(w, r1);
        } else if (more && wn.begin < wn.end) {
          r1 = wn.begin;
          n1 = rows_at(wn, r1);
        }
        issue(r1, n1);
      }
      f32x4 xc[2] = {zero4(), zero4()};
      if (kCamR) {
        phat_slabs<LN>(ph, g8, b8, eps);
        xl_slabs<2>(reinterpret_cast<const float4*>(Wl), ph, xc, lane);
      } else {
        wave_sync();
        xl_t<2>(Wl, T, xc, c, g);
      }
      const bool valid = c < nrows;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float xl[4], z[4], lz[4], p = 0.f, da = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = xc[q][r] + bcv[q][r];
          z[r] = xl[r] + xr[q][r];
          lz[r] = leaky(z[r], slope);
          p = fmaf(lz[r], attv[q][r], p);
          da = fmaf(gv[q][r], xl[r], da);
        }
        p += __shfl_xor(p, 16);
        da += __shfl_xor(da, 16);
        const float alpha = valid ? __expf(p - M[q]) * inv[q] : 0.f;
        const float de = alpha * (da - delta[q]);
        float dx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dz = de * attv[q][r] * (z[r] > 0.f ? 1.f : slope);
          dx[r] = fmaf(alpha, gv[q][r], dz);
          dxr[q][r] += dz;
          datt[q][r] = fmaf(de, lz[r], datt[q][r]);
        }
        if (valid)
          *reinterpret_cast<float4*>(dXLc + (row0 + c) * ldD + 16 * q + 4 * g) = make_float4(dx[0], dx[1], dx[2], dx[3]);
      }
      if (!kCamR) wave_sync();  // T is rewritten by the next tile
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = group_sum<16>(dxr[q][r]);
      if (c == 0) {
        float* d = (w.slot < 0) ? dXR + seg * ldDXR : part_dxr + int64_t(w.slot) * F;
        *reinterpret_cast<float4*>(d + 16 * q + 4 * g) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    w = wn;
  }
  // d att / d bias: sum over the 16 edge columns, then over the workgroup's waves (ordered)
  float v[16];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[q * 4 + r] = group_sum<16>(datt[q][r]);
      v[8 + q * 4 + r] = group_sum<16>(dbias[q][r]);
    }
  wg_reduce_ordered<16, kWaves, kWaves * TR * LD34>(v, &tiles[0][0], wave, lane);
  if (wave == 0 && c == 0) {
    float* o = part + int64_t(blockIdx.x) * BP_PART;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *reinterpret_cast<float4*>(o + 16 * q + 4 * g) = make_float4(v[q * 4], v[q * 4 + 1], v[q * 4 + 2], v[q * 4 + 3]);
      *reinterpret_cast<float4*>(o + F + 16 * q + 4 * g) =
          make_float4(v[8 + q * 4], v[8 + q * 4 + 1], v[8 + q * 4 + 2], v[8 + q * 4 + 3]);
    }
  }
}

// =============================================================================================
// backward, fused: camera attention + edge prologue of the block in ONE pass over the camera
// plan's items (gasfm_edge_cam_pbwd).  Per 16-edge tile:
//   XLc = Wc relu(LN(P)) + bc recomputed (T layout, as edge_cam_bwd), the camera attention's
//   backward -> dXLc in registers (T layout: the A operand of the next products as it stands);
//   dP_hat = dXLp Wpt + dXLc Wc + dRes (scale Wp[:, :32])  (C layout, A = T-layout rows);
//   dP = LN_bwd(mask * dP_hat) + dRes  (C layout, stored), dgamma, dbeta;
//   dW += [dXLp | dXLc]^T relu(LN(P)), db  (C-layout operands; dXLc through a per-wave LDS
//   transpose, dXLp / P / dRes re-read in C layout from L1).
// Replaces edge_cam_bwd + edge_prologue_bwd: dXLc (128 B per edge) is neither written nor read
// back, and P is read once.  Semantics: exactly those two kernels' (same partial-row layouts,
// concatenated: [dW 64x32 | db 64 | dgamma 32 | dbeta 32 | datt 32 | dbias 32] per workgroup).
// =============================================================================================
// 1: the C-layout LayerNorm statistics are the T-layout ones (computed for XLc) moved across by lane
// shuffles, and dP is stored through a bounds-checked buffer descriptor per work item (rows past
// the item's end are dropped by the range check): no per-row branch splits the tile's code, so
// the LayerNorm backward and the dW MFMAs schedule together (~900 -> ~700 instructions per tile;
// 683-692 -> 645-649 us in tools/edge_bench.py, same box).  0: C-layout statistics recomputed,
// per-row guarded stores.
#ifndef GASFM_PBWD_V2
#define GASFM_PBWD_V2 1
#endif
constexpr int PB2_PRO = NX * F + NX + 2 * F;  // the prologue_bwd part row
constexpr int PB2_PART = PB2_PRO + BP_PART;
constexpr int LDT = F + 4;                    // transpose tile row stride
constexpr int PB_NDW = 20;                    // (DWP) per-lane dWp sums: 16 MFMA values + 4 P0 terms
constexpr int PB_E0 = 164;                    // (EPI == 2) block 0's epilogue part: dWp 64 | dWsk 64 | dbsk 32 | 4

// The edge epilogues' backward folded into edge_cam_pbwd (round 3).  With SeamFn, the kernel that
// produces block b+1's dP is the one place where block b's epilogue gradient dP' (= that dP) is in
// registers in camera order, and block b's own edge_cam_pbwd later holds both dRes (= dP') and
// relu(LN_b(P_b)):
//   EPI (block b+1's launch): dSv_b[cam] = scale_e sum_e dP[e] (per camera item; split cameras as
//     partial rows), dP0_b[e] = scale_e We[:, 32:34]^T dP[e]
//   DWP (block b's launch): dWp_b = scale sum_e dRes[e]^T [relu(LN(P[e])) | P0[e]] as part rows
// which is everything edge_epilogue_bwd computed except dSp (segment_rowsum, point order).
struct PbwdEpi {
  const float* We;    // EPI: the previous block's lin_proj weight [32 x ldWe]
  int ldWe;
  float scale;        // EPI: the previous block's epilogue scale
  float* dSv;         // EPI: [m, 32]
  float* part_dsv;    // EPI: split-camera partial rows
  float* dP0;         // EPI: [E, 2] or null (no P0 skip input)
  const float* P0;    // DWP: [E, 2] or null
  int ldWpo;          // DWP: dWp row width in the part row (34 with P0, 32 without)
  // EPI == 2 (block 0's epilogue, round 4): its 2-wide weights Wp0 / Wsk0 [32 x 2] (We = Wp0), the
  // two 2-feature LayerNorms' affines [ga | ba | gb | bb] (2 each), their eps, the per-edge output
  // aux [E, 4] = (dP_hat_a (2), dP through the skip branch (2)) that edge0_prologue_bwd consumes
  const float* Wsk0;
  const float* ln0;
  float eps0;
  float* aux;
  const float* XLc;   // (XS, round 4 experiment) XLc [E, 32] kept by the forward seam, or null
};

// C-layout rows of a [*, 32] tensor: v[ft][r] = X[row0 + 4 g + r][16 ft + c] (rows clamped, not masked)
__device__ __forceinline__ void cl_load32(const float* __restrict__ X, int64_t ld, int64_t row0, int nrows,
                                          f32x4 (&v)[2], int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = 4 * g + r;
    const float* p = X + (row0 + (rr < nrows ? rr : 0)) * ld + c;
    v[0][r] = p[0];
    v[1][r] = p[16];
  }
}

// acc[nt] += X M^T, X (T-layout slabs, K = 32) as the A operand: acc[nt][r] = Y[row 4 g + r][16 nt + c]
__device__ __forceinline__ void prod_c2(const float4* __restrict__ Q, const f32x4 (&x)[2], f32x4 (&acc)[2],
                                        int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float4 w[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) w[nt] = Q[(nt * 2 + u) * 64 + lane];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(x[u][0], w[nt].x, acc[nt]);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(x[u][1], w[nt].y, acc[nt]);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(x[u][2], w[nt].z, acc[nt]);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(x[u][3], w[nt].w, acc[nt]);
  }
}

#ifndef GASFM_PBWD_MINW
#define GASFM_PBWD_MINW 2
#endif
// EPI's dP0: 1 = dP back to the T layout through tile 0 (a dot per lane, 2 cross-group sums per
// row tile); 0 = eight 16-lane DPP sums per tile.  DWP's LDS sums: 1 = float4 read-modify-writes
// (lane-major), 0 = scalar.  tools/gpu_pbwd_ab.sh, same box (us per launch, EPI+DWP): 785-790 with
// (1, 1), 792-798 with (0, 1), 775 with (1, 0, the default), 788-791 with (0, 0); the unfolded
// kernel 655-672 there, i.e. the fold adds ~110 us where edge_epilogue_bwd took ~220.
#ifndef GASFM_PBWD_EPI_T
#define GASFM_PBWD_EPI_T 1
#endif
// 1: the camera item's XR and gout rows (8 VGPRs each, live across the item's tiles) parked in the
// wave's LDS and re-read per tile; 0 (default): held in registers.  tools/gpu_pbwd_ab.sh, same box:
// config 4 30.36-30.40 ms with 1 vs 30.23-30.26 with 0 (the unfolded kernel's 4 spills go, the
// folded one keeps its 18, and the per-tile LDS reads cost more).
#ifndef GASFM_PBWD_ITEM_LDS
#define GASFM_PBWD_ITEM_LDS 0
#endif
#ifndef GASFM_PBWD_LW4
#define GASFM_PBWD_LW4 0
#endif
// 3: no exec-mask branches inside the tile loop (round 4).  Bit 2: the work item is made
// wave-uniform (scalar registers), so the next-tile choice is a scalar select; bit 1: the dead-row
// masks of the
// attention weights, the LayerNorm backward input, the dW / dWp operands and the dSv sums are
// multiplications by a 0 / 1 factor (every masked value is finite: dead rows are clamped copies of
// a live row) instead of selects the compiler turned into branches around LDS reads and v_exp,
// each of which ended a basic block and with it the scheduler's freedom to interleave the MFMA
// chains with the VALU work.
#ifndef GASFM_PBWD_BF
#define GASFM_PBWD_BF 0
#endif
// 1: the camera bias gradient's sums (added once per camera, by lanes c = 0) live in LDS, 8 floats
// per lane group, instead of 8 VGPRs held across every tile of the kernel (round 4); 2: also the
// LayerNorm affine of the lane's two C-layout columns re-read from LDS in each tile (4 VGPRs); 3: also
// the camera's softmax constants (max, 1 / sum, delta: 6 VGPRs) parked per lane group in LDS
#ifndef GASFM_PBWD_DB_LDS
#define GASFM_PBWD_DB_LDS 0
#endif
#ifndef GASFM_PBWD_PRIO
#define GASFM_PBWD_PRIO 0
#endif

// EPI == 2 (round 4): the previous block is block 0, whose epilogue is 2-wide
// (P' = Wsk relu(LN_b(P0)) + bsk + scale (Wp relu(LN_a(P0)) + bp + Sp + Sv + Sg), edge_block0.hip),
// folded like the 32-wide one: dSv from the same column sums, per edge the four dots
// (scale Wp, Wsk)^T dP and the LN_b backward on P0 (this launch's DWP P0 rows, i.e. block 0's
// input) to aux, and the weight sums [dWp dWsk | dbsk] = dP^T [relu(LN_a P0) relu(LN_b P0) | 1]
// as 8 MFMA per tile (B operand: the five edge values in tile 1's padding columns).  Replaces
// edge0_epilogue_bwd's pass over dP' (128 B per edge read back).
template <bool LN, bool RES, int EPI, bool DWP, bool XP = false, bool XS = false>
__global__ __launch_bounds__(kThreads, GASFM_PBWD_MINW) void edge_cam_pbwd_kernel(
    const float* __restrict__ P, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ Wc, const float* __restrict__ bc,
    const float* __restrict__ Wp, int ldWp, float scale, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum, int64_t ldStat,
    const float* __restrict__ gout, int64_t ldG, const gasfm_work_item* __restrict__ items, int n_items,
    const float* __restrict__ dXLp, int64_t ldXp, const float* __restrict__ dRes, float* __restrict__ dP,
    float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr, float* __restrict__ part, int64_t ldPart,
    PbwdEpi ep, const int32_t* __restrict__ dxl_pos) {
  static_assert(!DWP || (LN && RES), "edge_cam_pbwd: the epilogue weight gradient needs relu(LN(P)) and dRes");
  static_assert(EPI != 2 || DWP, "edge_cam_pbwd: block 0's epilogue fold reads block 0's input as the DWP P0 rows");
  // LDS: weight slabs (Wc for XLc; Wpt^T, Wc^T, (scale Wp)^T for dP_hat), the per-feature vectors,
  // per wave four 16 x 32 transpose tiles (T -> C layout of P, dXLp, dRes, dXLc), and (DWP) per
  // wave the lanes' running dWp sums
  constexpr int QW = F * F;  // floats per 32 x 32 slab set
  constexpr int OV = 4 * QW, OT = OV + (EPI == 2 ? 8 * F + 8 : EPI ? 6 * F : 4 * F), WT = 4 * TR * LDT;
  constexpr int OD = OT + kWaves * WT;
  constexpr int NLS = (DWP ? PB_NDW : 0) + (EPI ? 2 : 0);  // per-lane LDS sums
  constexpr int OX = OD + kWaves * NLS * kW;                 // per wave: the item's [XR | gout] rows
  // (EPI == 2) per wave 17 x 4 floats: the LN_b affine sums [dgb | dbb] of lanes c (group 0), then
  // one slot the other groups' (duplicate) values land in; per wave 21 x 8 floats: the weight sums
  // of the 20 lanes c < 5 (C layout), then a dummy slot (registers held across tiles spill here)
  constexpr int OG = OX + (GASFM_PBWD_ITEM_LDS ? kWaves * 2 * F : 0);
  constexpr int OA = OG + (EPI == 2 ? kWaves * 17 * 4 : 0);
  constexpr int OB = OA + (EPI == 2 ? kWaves * 21 * 8 : 0);
  constexpr int OC = OB + (GASFM_PBWD_DB_LDS ? kWaves * 4 * 8 : 0);
  constexpr int NL = OC + (GASFM_PBWD_DB_LDS >= 3 ? kWaves * 4 * 8 : 0);
  __shared__ __attribute__((aligned(16))) float lds[NL];
  float* WcQ = lds;
  float* WptTQ = lds + QW;
  float* WcTQ = lds + 2 * QW;
  float* WqTQ = lds + 3 * QW;
  float* V = lds + OV;  // [gamma | beta | bc | att] (32 each), (EPI) [scale_e We[:, 32] | scale_e We[:, 33]]
  stage_slabs32<F, kThreads>([&](int q) { return Wc[q]; }, WcQ);
  stage_slabs32<F, kThreads>([&](int q) { return Wpt[(q % F) * F + q / F]; }, WptTQ);
  stage_slabs32<F, kThreads>([&](int q) { return Wc[(q % F) * F + q / F]; }, WcTQ);
  if (RES) stage_slabs32<F, kThreads>([&](int q) { return scale * Wp[(q % F) * ldWp + q / F]; }, WqTQ);
  if (threadIdx.x < F) {
    V[threadIdx.x] = LN ? gam[threadIdx.x] : 1.f;
    V[F + threadIdx.x] = LN ? bet[threadIdx.x] : 0.f;
    V[2 * F + threadIdx.x] = bc[threadIdx.x];
    V[3 * F + threadIdx.x] = att[threadIdx.x];
    if (EPI == 1) {
      V[4 * F + threadIdx.x] = ep.dP0 ? ep.scale * ep.We[threadIdx.x * ep.ldWe + 32] : 0.f;
      V[5 * F + threadIdx.x] = ep.dP0 ? ep.scale * ep.We[threadIdx.x * ep.ldWe + 33] : 0.f;
    }
    if (EPI == 2) {  // [scale Wp0[:, 0] | scale Wp0[:, 1] | Wsk0[:, 0] | Wsk0[:, 1] | ga ba gb bb]
      V[4 * F + threadIdx.x] = ep.scale * ep.We[threadIdx.x * 2];
      V[5 * F + threadIdx.x] = ep.scale * ep.We[threadIdx.x * 2 + 1];
      V[6 * F + threadIdx.x] = ep.Wsk0[threadIdx.x * 2];
      V[7 * F + threadIdx.x] = ep.Wsk0[threadIdx.x * 2 + 1];
      if (threadIdx.x < 8) V[8 * F + threadIdx.x] = ep.ln0[threadIdx.x];
    }
  }
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Tt = lds + OT + wave * WT;  // tiles 0: P, 1: dXLp, 2: dRes, 3: dXLc
  // (DWP) value k of this lane's dWp sums at Lw[k]; (EPI) the item's dSv column sums at Ls[0, 1]
  float* Lw = lds + OD + (wave * kW + lane) * NLS;
  float* Ls = Lw + (DWP ? PB_NDW : 0);
  float* Xi = lds + OX + wave * 2 * F;  // (GASFM_PBWD_ITEM_LDS) [XR | gout] of the wave's camera item
  float* Lg = lds + OG + wave * 17 * 4 + (g == 0 ? c : 16) * 4;  // (EPI == 2) this lane's affine sums
  float* La = lds + OA + wave * 21 * 8 + (c < 5 ? 5 * g + c : 20) * 8;  // (EPI == 2) its weight sums
  float* Ldb = lds + OB + (wave * 4 + g) * 8;  // (GASFM_PBWD_DB_LDS) the lane group's dbias sums (lane c = 0)
  float* Lsm = lds + OC + (wave * 4 + g) * 8;  // (GASFM_PBWD_DB_LDS >= 3) [M | inv | delta] of the item
  if (GASFM_PBWD_DB_LDS && c == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) Ldb[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < NLS; ++k) Lw[k] = 0.f;
  if (EPI == 2) {
#pragma unroll
    for (int k = 0; k < 4; ++k) Lg[k] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) La[k] = 0.f;
  }
  const float gC0[2] = {LN ? gam[c] : 1.f, LN ? gam[16 + c] : 1.f}, bC0[2] = {LN ? bet[c] : 0.f, LN ? bet[16 + c] : 0.f};
  __syncthreads();
  // T-layout vector at this lane's features 16 q + 4 g .. + 3
  auto vecT = [&](int which, int q) {
    const float4 t = *reinterpret_cast<const float4*>(V + which * F + 16 * q + 4 * g);
    return f32x4{t.x, t.y, t.z, t.w};
  };
  // T -> C layout through tile k of this wave: writes the two slabs, returns the C-layout rows
  auto to_c = [&](int k, const f32x4 (&t)[2], f32x4 (&o)[2]) {
    float* T = Tt + k * TR * LDT;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<float4*>(T + c * LDT + 16 * u + 4 * g) = make_float4(t[u][0], t[u][1], t[u][2], t[u][3]);
    // one wave's LDS instructions execute in order: a compiler barrier suffices
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[ft][r] = T[(4 * g + r) * LDT + 16 * ft + c];
  };
  f32x4 accW[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) accW[mt][0] = accW[mt][1] = zero4();
  float db[4] = {0.f, 0.f, 0.f, 0.f}, dg[2] = {0.f, 0.f}, dbt[2] = {0.f, 0.f};
  f32x4 datt[2] = {zero4(), zero4()}, dbias[2] = {zero4(), zero4()};
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;
  // (GASFM_PBWD_PRIO) the second-dispatched half of the resident grid -- a CU's second workgroup,
  // whose waves share each SIMD with the first's -- issues at priority 1 (MI355X_MICROARCH.md
  // "Static priority for the younger half")
  if (GASFM_PBWD_PRIO && blockIdx.x >= gridDim.x / 2) __builtin_amdgcn_s_setprio(1);

  // next tile's rows of P, dXLp, dRes in T layout, one tile ahead (clamped, masked where consumed)
  f32x4 nPT[2], nXT[2], nRT[2], nXc[2];
  float2 nP0 = make_float2(0.f, 0.f);  // (DWP) P0 of edge c (a dummy read of P without P0)
  const float* p0p = (DWP && ep.P0) ? ep.P0 : P;
  // XP (round 4, dxl_pos): dXLp in point-segment order, edge e's row at dxl_pos[e] (the point
  // attention's backward then writes it streaming instead of scattering it).  The next tile's
  // position is the first load of issue(); its dXLp row is requested by issue_x() half a tile later,
  // once the position has arrived (waiting for it there does not wait for the loads issued after
  // it).  Without XP the dXLp row (edge row0 + c) is requested in issue() with the others.
  int npos = 0;
  auto load_x = [&](int64_t r) {
    const float* p = dXLp + r * ldXp + 4 * g;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float4 t = *reinterpret_cast<const float4*>(p + 16 * u);
      nXT[u] = f32x4{t.x, t.y, t.z, t.w};
    }
  };
  auto issue = [&](int64_t row0, int nrows) {
    const int64_t xrow = row0 + (c < nrows ? c : 0);
    if (XP) npos = dxl_pos[xrow];
    load_slabs32(P, row0, nrows, nPT, lane);
    if (!XP) load_x(xrow);
    if (XS) {  // XLc of edge c (T layout), kept by the forward seam
      const float* p = ep.XLc + xrow * F + 4 * g;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 t = *reinterpret_cast<const float4*>(p + 16 * u);
        nXc[u] = f32x4{t.x, t.y, t.z, t.w};
      }
    }
    if (RES) load_slabs32(dRes, row0, nrows, nRT, lane);
    if (DWP) nP0 = *reinterpret_cast<const float2*>(p0p + xrow * 2);
  };
  auto issue_x = [&]() {
    if (XP) load_x(npos);
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };
  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (GASFM_PBWD_BF & 2) w = uniform_item(w);
    if (w.begin < w.end) {
      issue(w.begin, rows_at(w, w.begin));
      issue_x();
    }
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    // dP's descriptor for this item's rows (wave-uniform inputs made provably uniform)
    const int64_t ibeg = __builtin_amdgcn_readfirstlane(int(w.begin));
    const int ilen = __builtin_amdgcn_readfirstlane(int(w.end - w.begin));
    const auto dPrs = __builtin_amdgcn_make_buffer_rsrc(dP + ibeg * F, 0, ilen * F * 4, 0x00020000);
    // (EPI) dP0 rows of this item; without dP0 an empty range (every store dropped)
    // (EPI == 2) aux rows of this item instead
    const auto dP0rs = EPI == 2 ? __builtin_amdgcn_make_buffer_rsrc(ep.aux + ibeg * 4, 0, ilen * 16, 0x00020000)
                                : __builtin_amdgcn_make_buffer_rsrc(EPI && ep.dP0 ? ep.dP0 + ibeg * 2 : dP, 0,
                                                                    EPI && ep.dP0 ? ilen * 8 : 0, 0x00020000);
    // per-camera constants of the attention backward (edge_cam_bwd_kernel)
    f32x4 xr[2], gv[2];
    float M[2], inv[2], delta[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
      const float4 x4 = *reinterpret_cast<const float4*>(XR + seg * ldXR + f0);
      const float4 g4v = *reinterpret_cast<const float4*>(gout + seg * ldG + f0);
      const float4 o4 = *reinterpret_cast<const float4*>(out + seg * ldOut + f0);
      const float4 b4 = *reinterpret_cast<const float4*>(bias + f0);
      xr[q] = f32x4{x4.x, x4.y, x4.z, x4.w};
      gv[q] = f32x4{g4v.x, g4v.y, g4v.z, g4v.w};
      if (GASFM_PBWD_ITEM_LDS && c == 0) {
        *reinterpret_cast<float4*>(Xi + f0) = x4;
        *reinterpret_cast<float4*>(Xi + F + f0) = g4v;
      }
      float d = fmaf(g4v.x, o4.x - b4.x, fmaf(g4v.y, o4.y - b4.y, fmaf(g4v.z, o4.z - b4.z, g4v.w * (o4.w - b4.w))));
      delta[q] = d + __shfl_xor(d, 16);
      M[q] = seg_max[seg * ldStat + h];
      inv[q] = 1.f / (seg_sum[seg * ldStat + h] + 1e-16f);
      if (GASFM_PBWD_DB_LDS >= 3 && c == 0) {
        Lsm[q] = M[q];
        Lsm[2 + q] = inv[q];
        Lsm[4 + q] = delta[q];
      }
    }
    const bool first = it == 0 || items[it - 1].seg != w.seg;
    if (first && c == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (GASFM_PBWD_DB_LDS) {
          const float4 o = *reinterpret_cast<const float4*>(Ldb + 4 * q);
          *reinterpret_cast<float4*>(Ldb + 4 * q) = make_float4(o.x + gv[q][0], o.y + gv[q][1], o.z + gv[q][2],
                                                                 o.w + gv[q][3]);
        } else {
          dbias[q] += gv[q];
        }
      }
    }
    f32x4 dxr[2] = {zero4(), zero4()};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (GASFM_PBWD_BF & 2) wn = uniform_item(wn);
    if (w.begin >= w.end && more && wn.begin < wn.end) {
      issue(wn.begin, rows_at(wn, wn.begin));
      issue_x();
    }
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 PT[2] = {nPT[0], nPT[1]}, XT[2] = {nXT[0], nXT[1]}, RT[2], XcT[2];
      if (XS) {
        XcT[0] = nXc[0];
        XcT[1] = nXc[1];
      }
      if (RES) {
        RT[0] = nRT[0];
        RT[1] = nRT[1];
      }
      const float2 p0t = nP0;
      if (GASFM_PBWD_BF & 2) {  // the same choice as scalar selects (w, wn are wave-uniform)
        const bool in_item = row0 + TR < w.end, nx = more && wn.begin < wn.end;
        const int64_t r1 = in_item ? row0 + TR : (nx ? int64_t(wn.begin) : row0);
        const int64_t e1 = in_item ? int64_t(w.end) : (nx ? int64_t(wn.end) : int64_t(w.end));
        issue(r1, int(e1 - r1 < TR ? e1 - r1 : TR));
      } else {  // the next tile (this item's, else the next item's first; the last one re-reads itself)
        int64_t r1 = row0;
        int n1 = nrows;
        if (row0 + TR < w.end) {
          r1 = row0 + TR;
          n1 = rows_at(w, r1);
        } else if (more && wn.begin < wn.end) {
          r1 = wn.begin;
          n1 = rows_at(wn, r1);
        }
        issue(r1, n1);
      }
      const bool valid = c < nrows;
      // (GASFM_PBWD_BF) 0 / 1 factors: edge c live (T layout), rows 4 g + r live (C layout)
      const float vmask = valid ? 1.f : 0.f;
      float lm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) lm[r] = 4 * g + r < nrows ? 1.f : 0.f;
      // C layouts of P, dXLp, dRes (raw) through LDS, before P's slabs are normalised in place
      f32x4 PC[2], XC[2], RC[2];
      to_c(0, PT, PC);
      to_c(1, XT, XC);
      if (RES) to_c(2, RT, RC);
      if (DWP) {  // edge c's P0 in tile 2's padding columns 32, 33 (read back in C layout by the dWp sums)
        float* T2 = Tt + 2 * TR * LDT + c * LDT + 32;
        T2[0] = p0t.x;
        T2[1] = p0t.y;
      }
      // ---- camera attention backward (T layout: edge c, features 16 q + 4 g + r)
      float tmean = 0.f, trstd = 1.f;  // LayerNorm statistics of edge c (T layout)
      if (LN) {
        float gs[2][4], bs[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 a = vecT(0, q), b = vecT(1, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gs[q][r] = a[r];
            bs[q][r] = b[r];
          }
        }
        phat_slabs_st<LN>(PT, gs, bs, eps, tmean, trstd);
      }
      f32x4 xc[2] = {vecT(2, 0), vecT(2, 1)};  // b_c, then + Wc P_hat^T (XS: the forward's rows)
      if (XS) {
        xc[0] = XcT[0];
        xc[1] = XcT[1];
      } else {
        xl_slabs<2>(reinterpret_cast<const float4*>(WcQ), PT, xc, lane);
      }
      f32x4 dXc[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 at = vecT(3, q);
        f32x4 xrq = xr[q], gvq = gv[q];
        if (GASFM_PBWD_ITEM_LDS) {
          const float4 t0 = *reinterpret_cast<const float4*>(Xi + 16 * q + 4 * g);
          const float4 t1 = *reinterpret_cast<const float4*>(Xi + F + 16 * q + 4 * g);
          xrq = f32x4{t0.x, t0.y, t0.z, t0.w};
          gvq = f32x4{t1.x, t1.y, t1.z, t1.w};
        }
        float z[4], lz[4], p = 0.f, da = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          z[r] = xc[q][r] + xrq[r];
          lz[r] = leaky(z[r], slope);
          p = fmaf(lz[r], at[r], p);
          da = fmaf(gvq[r], xc[q][r], da);
        }
        p += __shfl_xor(p, 16);
        da += __shfl_xor(da, 16);
        const float Mq = GASFM_PBWD_DB_LDS >= 3 ? Lsm[q] : M[q], iq = GASFM_PBWD_DB_LDS >= 3 ? Lsm[2 + q] : inv[q];
        const float dq = GASFM_PBWD_DB_LDS >= 3 ? Lsm[4 + q] : delta[q];
        const float alpha = (GASFM_PBWD_BF & 1) ? __expf(p - Mq) * iq * vmask : (valid ? __expf(p - Mq) * iq : 0.f);
        const float de = alpha * (da - dq);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dz = de * at[r] * (z[r] > 0.f ? 1.f : slope);
          dXc[q][r] = fmaf(alpha, gvq[r], dz);  // 0 for invalid edges
          dxr[q][r] += dz;
          datt[q][r] = fmaf(de, lz[r], datt[q][r]);
        }
      }
      issue_x();  // the next tile's dXLp rows (its position was loaded at the top of this tile)
      // ---- dP_hat (C layout) = dXLp Wpt + dXLc Wc (+ dRes scale Wp)
      f32x4 dph[2] = {zero4(), zero4()};
      prod_c2(reinterpret_cast<const float4*>(WptTQ), XT, dph, lane);
      prod_c2(reinterpret_cast<const float4*>(WcTQ), dXc, dph, lane);
      if (RES) prod_c2(reinterpret_cast<const float4*>(WqTQ), RT, dph, lane);
      f32x4 XcC[2];
      to_c(3, dXc, XcC);
      // ---- LayerNorm statistics of the C-layout rows, LN backward, dP
      float gC[2], bC[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        gC[nt] = GASFM_PBWD_DB_LDS >= 2 ? (LN ? V[16 * nt + c] : 1.f) : gC0[nt];
        bC[nt] = GASFM_PBWD_DB_LDS >= 2 ? (LN ? V[F + 16 * nt + c] : 0.f) : bC0[nt];
      }
      f32x4 ph[2];  // relu(LN(P)) (C layout) for the weight gradient
      float dv[4][2];  // dP (C layout) for the branch-free stores (GASFM_PBWD_V2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool live = 4 * g + r < nrows;
        float mean = 0.f, rstd = 1.f;
        if (LN && GASFM_PBWD_V2) {
          mean = __shfl(tmean, 4 * g + r);  // edge 4 g + r's statistics live on lane c = 4 g + r
          rstd = __shfl(trstd, 4 * g + r);
        } else if (LN) {
          mean = sum16(PC[0][r] + PC[1][r]) * (1.f / F);
          const float d0 = PC[0][r] - mean, d1 = PC[1][r] - mean;
          rstd = rsqrtf(sum16(fmaf(d0, d0, d1 * d1)) * (1.f / F) + eps);
        }
        float xh[2], gvv[2], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          xh[nt] = LN ? (PC[nt][r] - mean) * rstd : PC[nt][r];
          ph[nt][r] = LN ? fmaxf(fmaf(xh[nt], gC[nt], bC[nt]), 0.f) : xh[nt];
          float dy = (GASFM_PBWD_BF & 1) ? dph[nt][r] * lm[r] : (live ? dph[nt][r] : 0.f);
          if (LN) {
            dy = (fmaf(xh[nt], gC[nt], bC[nt]) > 0.f) ? dy : 0.f;
            dg[nt] = fmaf(dy, xh[nt], dg[nt]);
            dbt[nt] += dy;
          }
          gvv[nt] = LN ? dy * gC[nt] : dy;
          s1 += gvv[nt];
          s2 = fmaf(gvv[nt], xh[nt], s2);
        }
        if (LN) {
          s1 = sum16(s1) * (1.f / F);
          s2 = sum16(s2) * (1.f / F);
        }
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          float v = LN ? rstd * (gvv[nt] - s1 - xh[nt] * s2) : gvv[nt];
          if (RES) v += RC[nt][r];
          dv[r][nt] = v;
        }
        if (!GASFM_PBWD_V2 && live) {
          float* d = dP + (row0 + 4 * g + r) * F + c;
          d[0] = dv[r][0];
          d[16] = dv[r][1];
        }
      }
      if (GASFM_PBWD_V2) {
        // rows past the item's end fall outside the descriptor's range: the hardware drops them
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            __builtin_amdgcn_raw_buffer_store_b32(  // (the builtin's data operand is a 32-bit integer)
                __float_as_uint(dv[r][nt]), dPrs, int(((row0 - ibeg + 4 * g + r) * F + 16 * nt + c) * 4), 0, 0);
      }
      if (EPI) {
        // the previous block's epilogue: column sums of dP (dSv), and dP0 = scale_e We[:, 32:34]^T dP
        // per row: dP through tile 0 (free since P's transpose) back to the T layout, lane (g, c)
        // dots row c's features 16 u + 4 g .. + 3, the 4 lane groups summed; group 0 stores the
        // row's pair (the other groups an out-of-range offset)
        float* T0 = Tt;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool live = 4 * g + r < nrows;
          // the item's column sums of dP (dSv) live in LDS: no registers held across tiles
          Ls[0] += (GASFM_PBWD_BF & 1) ? dv[r][0] * lm[r] : (live ? dv[r][0] : 0.f);
          Ls[1] += (GASFM_PBWD_BF & 1) ? dv[r][1] * lm[r] : (live ? dv[r][1] : 0.f);
          if (!GASFM_PBWD_EPI_T && EPI == 1) {  // A/B: 16-lane sums per row (DPP), lanes c = 0, 1 store
            const float s0 = sum16(fmaf(dv[r][0], V[4 * F + c], dv[r][1] * V[4 * F + 16 + c]));
            const float s1 = sum16(fmaf(dv[r][0], V[5 * F + c], dv[r][1] * V[5 * F + 16 + c]));
            const int off = c < 2 ? int(((row0 - ibeg + 4 * g + r) * 2 + c) * 4) : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(c ? s1 : s0), dP0rs, off, 0, 0);
          } else {
            T0[(4 * g + r) * LDT + c] = dv[r][0];
            T0[(4 * g + r) * LDT + 16 + c] = dv[r][1];
          }
        }
      }
      if (EPI == 1 && GASFM_PBWD_EPI_T) {
        float* T0 = Tt;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float4 d4 = *reinterpret_cast<const float4*>(T0 + c * LDT + 16 * u + 4 * g);
          const f32x4 a = vecT(4, u), b = vecT(5, u);
          s0 = fmaf(d4.x, a[0], fmaf(d4.y, a[1], fmaf(d4.z, a[2], fmaf(d4.w, a[3], s0))));
          s1 = fmaf(d4.x, b[0], fmaf(d4.y, b[1], fmaf(d4.z, b[2], fmaf(d4.w, b[3], s1))));
        }
        s0 = sum_groups(s0);
        s1 = sum_groups(s1);
        const int off = g == 0 ? int((row0 - ibeg + c) * 8) : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s0), dP0rs, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s1), dP0rs, off + 4, 0, 0);
      }
      if (EPI == 2) {
        // block 0's epilogue backward for edge c (T layout; the four lane groups hold the same values)
        float* T0 = Tt;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float4 d4 = *reinterpret_cast<const float4*>(T0 + c * LDT + 16 * u + 4 * g);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 a = vecT(4 + j, u);
            q[j] = fmaf(d4.x, a[0], fmaf(d4.y, a[1], fmaf(d4.z, a[2], fmaf(d4.w, a[3], q[j]))));
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = sum_groups(q[j]);
        const float4 la = *reinterpret_cast<const float4*>(V + 8 * F);      // ga0 ga1 ba0 ba1
        const float4 lb = *reinterpret_cast<const float4*>(V + 8 * F + 4);  // gb0 gb1 bb0 bb1
        const float mean = 0.5f * (p0t.x + p0t.y), e0 = p0t.x - mean, e1 = p0t.y - mean;
        const float rs = rsqrtf(0.5f * (e0 * e0 + e1 * e1) + ep.eps0);
        const float xh0 = e0 * rs, xh1 = e1 * rs;
        const float yb0 = fmaf(xh0, lb.x, lb.z), yb1 = fmaf(xh1, lb.y, lb.w);
        // LN_b / ReLU backward of the skip branch
        const float db0 = yb0 > 0.f ? q[2] : 0.f, db1 = yb1 > 0.f ? q[3] : 0.f;
        const float g0 = db0 * lb.x, g1 = db1 * lb.y;
        const float mg = 0.5f * (g0 + g1), mgx = 0.5f * (g0 * xh0 + g1 * xh1);
        const float dx0 = rs * (g0 - mg - xh0 * mgx), dx1 = rs * (g1 - mg - xh1 * mgx);
        // aux[edge c] = (qa0, qa1, dx0, dx1): lane group g stores component g (rows past the item's
        // end fall outside the descriptor's range)
        const float av = g == 0 ? q[0] : g == 1 ? q[1] : g == 2 ? dx0 : dx1;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(av), dP0rs, int(((row0 - ibeg + c) * 4 + g) * 4), 0, 0);
        const float f = vmask;  // group 0's slots count each live edge once (the others: the dummy slot)
        Lg[0] = fmaf(f * db0, xh0, Lg[0]);
        Lg[1] = fmaf(f * db1, xh1, Lg[1]);
        Lg[2] = fmaf(f, db0, Lg[2]);
        Lg[3] = fmaf(f, db1, Lg[3]);
        // [relu(LN_a P0) | relu(LN_b P0)] of edge c into tile 1's padding columns (tile 1's rows were
        // read back before the attention)
        if (g == 0)
          *reinterpret_cast<float4*>(Tt + TR * LDT + c * LDT + 32) =
              make_float4(fmaxf(fmaf(xh0, la.x, la.z), 0.f), fmaxf(fmaf(xh1, la.y, la.w), 0.f), fmaxf(yb0, 0.f),
                          fmaxf(yb1, 0.f));
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        // [dWp0 dWsk0 | dbsk0] += dP^T [h | 1] (dead rows zeroed in the B operand; dP re-read from tile 0
        // in the C layout rather than held in registers since the LayerNorm backward)
        const float* T1 = Tt + TR * LDT;
        f32x4 acc0[2] = {zero4(), zero4()};
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const float hv = T1[(4 * g + s2) * LDT + 32 + (c & 3)];
          const float b = (c < 4 ? hv : (c == 4 ? 1.f : 0.f)) * lm[s2];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc0[nt] = mfma16(T0[(4 * g + s2) * LDT + 16 * nt + c], b, acc0[nt]);
        }
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const float4 o = *reinterpret_cast<const float4*>(La + 4 * nt);
          *reinterpret_cast<float4*>(La + 4 * nt) =
              make_float4(o.x + acc0[nt][0], o.y + acc0[nt][1], o.z + acc0[nt][2], o.w + acc0[nt][3]);
        }
      }
      // ---- dW += [dXLp | dXLc]^T relu(LN(P)), db (C layout, row 4 g + s at step s)
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) XC[ft][r] = (GASFM_PBWD_BF & 1) ? XC[ft][r] * lm[r] : (4 * g + r < nrows ? XC[ft][r] : 0.f);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const float a = mt < 2 ? XC[mt][s2] : XcC[mt - 2][s2];
          db[mt] += a;
          accW[mt][0] = mfma16(a, ph[0][s2], accW[mt][0]);
          accW[mt][1] = mfma16(a, ph[1][s2], accW[mt][1]);
        }
      }
      if (DWP) {
        // this block's epilogue: dWp += dRes^T [relu(LN(P)) | P0] (dead rows zeroed), one 16-feature
        // half of dRes at a time, its rows and P0 re-read from tile 2 (no registers held across the
        // tile), the products added into the lanes' LDS sums
        const float* T2 = Tt + 2 * TR * LDT;
#pragma unroll
        for (int ft = 0; ft < 2; ++ft) {
          float rr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            rr[r] = (GASFM_PBWD_BF & 1) ? T2[(4 * g + r) * LDT + 16 * ft + c] * lm[r]
                                  : (4 * g + r < nrows ? T2[(4 * g + r) * LDT + 16 * ft + c] : 0.f);
          f32x4 ap[2] = {zero4(), zero4()};
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) ap[nt] = mfma16(rr[s2], ph[nt][s2], ap[nt]);
          float a0[2] = {0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a0[0] = fmaf(rr[r], T2[(4 * g + r) * LDT + 32], a0[0]);
            a0[1] = fmaf(rr[r], T2[(4 * g + r) * LDT + 33], a0[1]);
          }
          // this half's 10 sums: [ap[0] | ap[1] | a0] at Lw[lane * 20 + 10 ft ..] (lane stride 20
          // floats: a 16-lane b128 access touches 16 distinct bank quads)
          float* q = Lw + 10 * ft;
          if (!GASFM_PBWD_LW4) {  // A/B: scalar read-modify-writes
#pragma unroll
            for (int k = 0; k < 8; ++k) q[k] += ap[k / 4][k % 4];
            q[8] += a0[0];
            q[9] += a0[1];
          } else {
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const float4 o = *reinterpret_cast<const float4*>(q + 4 * nt);
            *reinterpret_cast<float4*>(q + 4 * nt) =
                make_float4(o.x + ap[nt][0], o.y + ap[nt][1], o.z + ap[nt][2], o.w + ap[nt][3]);
          }
          const float2 o2 = *reinterpret_cast<const float2*>(q + 8);
          *reinterpret_cast<float2*>(q + 8) = make_float2(o2.x + a0[0], o2.y + a0[1]);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // this tile's transpose reads before the next tile's writes
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = group_sum<16>(dxr[q][r]);
      if (c == 0) {
        float* d = (w.slot < 0) ? dXR + seg * ldDXR : part_dxr + int64_t(w.slot) * F;
        *reinterpret_cast<float4*>(d + 16 * q + 4 * g) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    if (EPI) {
      const float s0 = sum_groups(Ls[0]) * ep.scale, s1 = sum_groups(Ls[1]) * ep.scale;
      Ls[0] = Ls[1] = 0.f;
      if (g == 0) {
        float* d = (w.slot < 0) ? ep.dSv + seg * F : ep.part_dsv + int64_t(w.slot) * F;
        d[c] = s0;
        d[16 + c] = s1;
      }
    }
    w = wn;
  }
  // workgroup reduction: 32 accW + 4 db + 2 dg + 2 dbt (C layout) + 16 (datt, dbias summed over
  // the 16 edge columns first) (+ DWP: the lanes' 20 dWp sums, read before the scratch is reused)
  constexpr int NB2 = 56 + (DWP ? PB_NDW : 0);  // (EPI == 2) v[NB2 ..]: acc0 (8), then Lg (4)
  constexpr int NV = NB2 + (EPI == 2 ? 12 : 0);
  float v[NV];
  if (EPI == 2) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[NB2 + nt * 4 + r] = c < 5 ? La[nt * 4 + r] : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[NB2 + 8 + k] = g == 0 ? Lg[k] : 0.f;
  }
  if (DWP) {  // v[56 + (ft * 2 + nt) * 4 + r] = the MFMA sums, v[72 + ft * 2 + j] = the P0 terms
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[56 + ft * 8 + k] = Lw[10 * ft + k];
#pragma unroll
      for (int j = 0; j < 2; ++j) v[72 + ft * 2 + j] = Lw[10 * ft + 8 + j];
    }
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(mt * 2 + nt) * 4 + r] = accW[mt][nt][r];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) v[32 + mt] = db[mt];
  v[36] = dg[0];
  v[37] = dg[1];
  v[38] = dbt[0];
  v[39] = dbt[1];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[40 + q * 4 + r] = group_sum<16>(datt[q][r]);
      v[48 + q * 4 + r] = group_sum<16>(GASFM_PBWD_DB_LDS ? (c == 0 ? Ldb[4 * q + r] : 0.f) : dbias[q][r]);
    }
  wg_reduce_ordered<NV, kWaves, NL>(v, lds, wave, lane);
  if (wave == 0) {
    float* o = part + int64_t(blockIdx.x) * ldPart;
    if (EPI == 2) {  // [dWp0 64 | dWsk0 64 | dbsk0 32 | dgb 2 | dbb 2] after the dWp block (edge0_epilogue_bwd's row)
      float* o2 = o + PB2_PART + F * ep.ldWpo;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 16 * nt + 4 * g + r;
          const float x = v[NB2 + nt * 4 + r];
          if (c < 2)
            o2[2 * f + c] = x * ep.scale;
          else if (c < 4)
            o2[64 + 2 * f + c - 2] = x;
          else if (c == 4)
            o2[128 + f] = x;
        }
      float t2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) t2[k] = sum_groups(group_sum<16>(v[NB2 + 8 + k]));
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) o2[160 + k] = t2[k];
      }
    }
    if (DWP) {  // [32 x ldWpo] after the prologue/attention part, scaled as the epilogue's
      float* od = o + PB2_PART;
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            od[(16 * ft + 4 * g + r) * ep.ldWpo + 16 * nt + c] = v[56 + (ft * 2 + nt) * 4 + r] * scale;
      float t0[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) t0[k] = sum_groups(v[72 + k]);
      if (ep.P0 && g == 0) {
#pragma unroll
        for (int ft = 0; ft < 2; ++ft)
#pragma unroll
          for (int j = 0; j < 2; ++j) od[(16 * ft + c) * ep.ldWpo + 32 + j] = t0[ft * 2 + j] * scale;
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(mt * 16 + 4 * g + r) * F + nt * 16 + c] = v[(mt * 2 + nt) * 4 + r];
    float tt[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) tt[k] = sum_groups(v[32 + k]);
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) o[NX * F + mt * 16 + c] = tt[mt];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        o[NX * F + NX + nt * 16 + c] = tt[4 + nt];
        o[NX * F + NX + F + nt * 16 + c] = tt[6 + nt];
      }
    }
    if (c == 0) {
      float* oa = o + PB2_PRO;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<float4*>(oa + 16 * q + 4 * g) =
            make_float4(v[40 + q * 4], v[40 + q * 4 + 1], v[40 + q * 4 + 2], v[40 + q * 4 + 3]);
        *reinterpret_cast<float4*>(oa + F + 16 * q + 4 * g) =
            make_float4(v[48 + q * 4], v[48 + q * 4 + 1], v[48 + q * 4 + 2], v[48 + q * 4 + 3]);
      }
    }
  }
}

int grid_cam_pbwd(int n_items) {
  return resident_grid(reinterpret_cast<const void*>(&edge_cam_pbwd_kernel<true, true, false, false>), kThreads, 0,
                       n_items, kWaves);
}

int grid_cam_bwd(int n_items) {
  return resident_grid(reinterpret_cast<const void*>(&edge_cam_bwd_kernel<true>), kThreads, 0, n_items, kWaves);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int32_t gasfm_edge_cam_bwd_part_rows(int32_t n_items) { return grid_cam_bwd(n_items > 0 ? n_items : 1); }
extern "C" int32_t gasfm_edge_cam_bwd_part_cols(void) { return BP_PART; }

extern "C" int gasfm_edge_cam_fwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                  const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                  const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                  const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                  int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                  int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && Wpt && bpt && Wc && bc && XLp && XR && att && items,
                "gasfm_edge_cam_fwd: null pointer");
  GASFM_REQUIRE((out && seg_max && seg_sum && (bias || !finalize)) || part, "gasfm_edge_cam_fwd: no outputs");
  GASFM_REQUIRE(ldXLp >= F && ldXLp % 4 == 0 && ldXR >= F && ldXR % 4 == 0 && (!out || (ldOut >= F && ldOut % 4 == 0)) &&
                    aligned16(P) && aligned16(XLp) && aligned16(XR) && (!out || aligned16(out)) &&
                    (!part || aligned16(part)) && (!ln_w || (aligned16(ln_w) && aligned16(ln_b))),
                "gasfm_edge_cam_fwd: 16-byte rows required");
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto launch = [&](auto kern) {
    const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, 0, n_items, kWaves);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, P, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp,
                       pos, XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max, seg_sum,
                       ldStat, part);
  };
  if (ln_w)
    launch(&edge_cam_fwd_kernel<true>);
  else
    launch(&edge_cam_fwd_kernel<false>);
  return launch_status("gasfm_edge_cam_fwd");
}

extern "C" int gasfm_edge_cam_bwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wc,
                                  const float* bc, const float* XR, int64_t ldXR, const float* att, const float* bias,
                                  float slope, const float* out, int64_t ldOut, const float* seg_max,
                                  const float* seg_sum, int64_t ldStat, const float* gout, int64_t ldG,
                                  const gasfm_work_item* items, int32_t n_items, float* dXLc, int64_t ldD, float* dXR,
                                  int64_t ldDXR, float* part_dxr, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && Wc && bc && XR && att && bias && out && seg_max && seg_sum && gout && items &&
                    dXLc && dXR && part,
                "gasfm_edge_cam_bwd: null pointer");
  GASFM_REQUIRE(ldXR % 4 == 0 && ldOut % 4 == 0 && ldG % 4 == 0 && ldD % 4 == 0 && ldDXR % 4 == 0 && aligned16(P) &&
                    aligned16(XR) && aligned16(out) && aligned16(gout) && aligned16(dXLc) && aligned16(dXR) &&
                    (!part_dxr || aligned16(part_dxr)) && (!ln_w || (aligned16(ln_w) && aligned16(ln_b))),
                "gasfm_edge_cam_bwd: 16-byte rows required");
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_cam_bwd(n_items);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, P, ln_w, ln_b, eps, Wc, bc, XR, ldXR, att, bias, slope,
                       out, ldOut, seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLc, ldD, dXR, ldDXR,
                       part_dxr, part);
  };
  if (ln_w)
    launch(&edge_cam_bwd_kernel<true>);
  else
    launch(&edge_cam_bwd_kernel<false>);
  return launch_status("gasfm_edge_cam_bwd");
}

extern "C" int32_t gasfm_edge_cam_pbwd_part_rows(int32_t n_items) { return grid_cam_pbwd(n_items > 0 ? n_items : 1); }
extern "C" int32_t gasfm_edge_cam_pbwd_part_cols(void) { return PB2_PART; }

namespace {
// the launcher behind gasfm_edge_cam_pbwd_ex and gasfm_edge_cam_pbwd_e0 (ep.aux set: block 0's fold)
int pbwd_launch(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt, const float* Wc,
                const float* bc, const float* Wp, int32_t ldWp, float scale, const float* XR, int64_t ldXR,
                const float* att, const float* bias, float slope, const float* out, int64_t ldOut,
                const float* seg_max, const float* seg_sum, int64_t ldStat, const float* gout, int64_t ldG,
                const gasfm_work_item* items, int32_t n_items, const float* dXLp, int64_t ldXp, const float* dRes,
                float* dP, float* dXR, int64_t ldDXR, float* part_dxr, float* part, int64_t ldPart,
                const PbwdEpi& ep, const int32_t* dxl_pos, void* stream) {
  const float *We = ep.We, *P0 = ep.P0;
  const int32_t ldWe = ep.ldWe, ldWpo = ep.ldWpo;
  float *dSv_e = ep.dSv, *dP0_e = ep.dP0;
  const bool e0 = ep.aux != nullptr;
  GASFM_REQUIRE(n_items >= 0 && P && Wpt && Wc && bc && XR && att && bias && out && seg_max && seg_sum && gout &&
                    items && dXLp && dP && dXR && part && (!dRes || (Wp && ldWp >= F)),
                "gasfm_edge_cam_pbwd: null pointer");
  GASFM_REQUIRE(ldXR % 4 == 0 && ldOut % 4 == 0 && ldG % 4 == 0 && ldXp % 4 == 0 && ldXp >= F && ldDXR % 4 == 0 &&
                    aligned16(P) && aligned16(XR) && aligned16(out) && aligned16(gout) && aligned16(dXLp) &&
                    aligned16(dP) && aligned16(dXR) && (!dRes || aligned16(dRes)) &&
                    (!part_dxr || aligned16(part_dxr)) && (!ln_w || (aligned16(ln_w) && aligned16(ln_b))),
                "gasfm_edge_cam_pbwd: 16-byte rows required");
  const bool epi = dSv_e != nullptr, dwp = ldWpo > 0;
  GASFM_REQUIRE(!epi || (We && (e0 || ldWe >= F + (dP0_e ? 2 : 0)) && (ln_w != nullptr) == (dRes != nullptr)),
                "gasfm_edge_cam_pbwd: the previous epilogue's outputs need its lin_proj weight (and LN == RES)");
  GASFM_REQUIRE(!dwp || (ln_w && dRes && ldWpo == (P0 ? F + 2 : F)),
                "gasfm_edge_cam_pbwd: the epilogue weight gradient needs LN, dRes and ldWpo = 32 (+2 with P0)");
  GASFM_REQUIRE(!e0 || (epi && dwp && P0 && ep.Wsk0 && ep.ln0 && !dP0_e && aligned16(ep.aux)),
                "gasfm_edge_cam_pbwd_e0: block 0's fold needs dSv, the DWP P0 rows (block 0's input), Wsk0, "
                "the LayerNorm affines and a 16-byte aligned aux");
  GASFM_REQUIRE(ldPart >= PB2_PART + (dwp ? int64_t(F) * ldWpo : 0) + (e0 ? PB_E0 : 0),
                "gasfm_edge_cam_pbwd: part row too narrow");
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_cam_pbwd(n_items);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR,
                       ldXR, att, bias, slope, out, ldOut, seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp,
                       ldXp, dRes, dP, dXR, ldDXR, part_dxr, part, ldPart, ep, dxl_pos);
  };
  auto pick = [&](auto xp) {
    constexpr bool X = decltype(xp)::value;
    if (ln_w && dRes) {
      if (e0)
        launch(&edge_cam_pbwd_kernel<true, true, 2, true, X>);
      else if (epi && dwp && ep.XLc)
        launch(&edge_cam_pbwd_kernel<true, true, 1, true, X, true>);
      else if (epi && dwp)
        launch(&edge_cam_pbwd_kernel<true, true, true, true, X>);
      else if (epi)
        launch(&edge_cam_pbwd_kernel<true, true, true, false, X>);
      else if (dwp)
        launch(&edge_cam_pbwd_kernel<true, true, false, true, X>);
      else
        launch(&edge_cam_pbwd_kernel<true, true, false, false, X>);
    } else if (ln_w) {
      launch(&edge_cam_pbwd_kernel<true, false, false, false, X>);
    } else if (dRes) {
      launch(&edge_cam_pbwd_kernel<false, true, false, false, X>);
    } else if (epi) {
      launch(&edge_cam_pbwd_kernel<false, false, true, false, X>);
    } else {
      launch(&edge_cam_pbwd_kernel<false, false, false, false, X>);
    }
  };
  if (dxl_pos)
    pick(std::true_type{});
  else
    pick(std::false_type{});
  return launch_status("gasfm_edge_cam_pbwd");
}
}  // namespace

extern "C" int gasfm_edge_cam_pbwd_ex(const float* P, const float* ln_w, const float* ln_b, float eps,
                                      const float* Wpt, const float* Wc, const float* bc, const float* Wp, int32_t ldWp,
                                      float scale, const float* XR, int64_t ldXR, const float* att, const float* bias,
                                      float slope, const float* out, int64_t ldOut, const float* seg_max,
                                      const float* seg_sum, int64_t ldStat, const float* gout, int64_t ldG,
                                      const gasfm_work_item* items, int32_t n_items, const float* dXLp, int64_t ldXp,
                                      const float* dRes, float* dP, float* dXR, int64_t ldDXR, float* part_dxr,
                                      float* part, int64_t ldPart, const float* We, int32_t ldWe, float scale_e,
                                      float* dSv_e, float* part_dsv_e, float* dP0_e, const float* P0, int32_t ldWpo,
                                      const int32_t* dxl_pos, void* stream) {
  const PbwdEpi ep{We, ldWe, scale_e, dSv_e, part_dsv_e, dP0_e, P0, ldWpo, nullptr, nullptr, 0.f, nullptr};
  return pbwd_launch(P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR, ldXR, att, bias, slope, out, ldOut,
                     seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp, ldXp, dRes, dP, dXR, ldDXR, part_dxr,
                     part, ldPart, ep, dxl_pos, stream);
}

extern "C" int gasfm_edge_cam_pbwd_xlc(const float* P, const float* ln_w, const float* ln_b, float eps,
                                       const float* Wpt, const float* Wc, const float* bc, const float* Wp,
                                       int32_t ldWp, float scale, const float* XR, int64_t ldXR, const float* att,
                                       const float* bias, float slope, const float* out, int64_t ldOut,
                                       const float* seg_max, const float* seg_sum, int64_t ldStat, const float* gout,
                                       int64_t ldG, const gasfm_work_item* items, int32_t n_items, const float* dXLp,
                                       int64_t ldXp, const float* dRes, float* dP, float* dXR, int64_t ldDXR,
                                       float* part_dxr, float* part, int64_t ldPart, const float* We, int32_t ldWe,
                                       float scale_e, float* dSv_e, float* part_dsv_e, float* dP0_e, const float* P0,
                                       int32_t ldWpo, const int32_t* dxl_pos, const float* XLc, void* stream) {
  GASFM_REQUIRE(XLc && aligned16(XLc), "gasfm_edge_cam_pbwd_xlc: XLc must be a 16-byte aligned [E, 32] array");
  const PbwdEpi ep{We, ldWe, scale_e, dSv_e, part_dsv_e, dP0_e, P0, ldWpo, nullptr, nullptr, 0.f, nullptr, XLc};
  return pbwd_launch(P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR, ldXR, att, bias, slope, out, ldOut,
                     seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp, ldXp, dRes, dP, dXR, ldDXR, part_dxr,
                     part, ldPart, ep, dxl_pos, stream);
}

extern "C" int32_t gasfm_edge_cam_pbwd_e0_cols(void) { return PB_E0; }

extern "C" int gasfm_edge_cam_pbwd_e0(const float* P, const float* ln_w, const float* ln_b, float eps,
                                      const float* Wpt, const float* Wc, const float* bc, const float* Wp, int32_t ldWp,
                                      float scale, const float* XR, int64_t ldXR, const float* att, const float* bias,
                                      float slope, const float* out, int64_t ldOut, const float* seg_max,
                                      const float* seg_sum, int64_t ldStat, const float* gout, int64_t ldG,
                                      const gasfm_work_item* items, int32_t n_items, const float* dXLp, int64_t ldXp,
                                      const float* dRes, float* dP, float* dXR, int64_t ldDXR, float* part_dxr,
                                      float* part, int64_t ldPart, const float* P0, const float* Wp0,
                                      const float* Wsk0, const float* ln0, float eps0, float scale0, float* dSv0,
                                      float* part_dsv0, float* aux0, const int32_t* dxl_pos, void* stream) {
  GASFM_REQUIRE(Wp0 && Wsk0 && ln0 && dSv0 && aux0 && P0, "gasfm_edge_cam_pbwd_e0: null pointer");
  const PbwdEpi ep{Wp0, 2, scale0, dSv0, part_dsv0, nullptr, P0, F + 2, Wsk0, ln0, eps0, aux0};
  return pbwd_launch(P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR, ldXR, att, bias, slope, out, ldOut,
                     seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp, ldXp, dRes, dP, dXR, ldDXR, part_dxr,
                     part, ldPart, ep, dxl_pos, stream);
}

extern "C" int gasfm_edge_cam_pbwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                   const float* Wc, const float* bc, const float* Wp, int32_t ldWp, float scale,
                                   const float* XR, int64_t ldXR, const float* att, const float* bias, float slope,
                                   const float* out, int64_t ldOut, const float* seg_max, const float* seg_sum,
                                   int64_t ldStat, const float* gout, int64_t ldG, const gasfm_work_item* items,
                                   int32_t n_items, const float* dXLp, int64_t ldXp, const float* dRes, float* dP,
                                   float* dXR, int64_t ldDXR, float* part_dxr, float* part, void* stream) {
  return gasfm_edge_cam_pbwd_ex(P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR, ldXR, att, bias, slope, out,
                                ldOut, seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp, ldXp, dRes, dP, dXR,
                                ldDXR, part_dxr, part, PB2_PART, nullptr, 0, 0.f, nullptr, nullptr, nullptr, nullptr, 0,
                                nullptr, stream);
}

extern "C" int gasfm_edge_seam_fwd_x(const float* Pb, const float* P0, const int32_t* pt, const float* ln_wb,
                                     const float* ln_bb, float eps_b, const float* Wp, int32_t ldWp, const float* bp,
                                     const float* Sp, const float* Sv, int64_t ldSv, const float* Sg, float scale,
                                     float* Pout, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                     const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                     const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                     const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                     int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                     int64_t ldStat, float* part, float* XLc, void* stream) {
  GASFM_REQUIRE(!XLc || (aligned16(XLc) && ln_w && tune(GASFM_TUNE_SEAM_LDS) == 0),
                "gasfm_edge_seam_fwd_x: XLc needs 16-byte rows, the LayerNorm and the register seam");
  GASFM_REQUIRE(n_items >= 0 && Pb && pt && ln_wb && ln_bb && Wp && bp && Sp && Sv && Sg && Pout && Wpt && bpt &&
                    Wc && bc && XLp && XR && att && items,
                "gasfm_edge_seam_fwd: null pointer");
  GASFM_REQUIRE(ldWp >= (P0 ? F + 2 : F), "gasfm_edge_seam_fwd: ldWp");
  GASFM_REQUIRE((out && seg_max && seg_sum && (bias || !finalize)) || part, "gasfm_edge_seam_fwd: no outputs");
  GASFM_REQUIRE(ldXLp >= F && ldXLp % 4 == 0 && ldXR >= F && ldXR % 4 == 0 && ldSv >= F && ldSv % 4 == 0 &&
                    (!out || (ldOut >= F && ldOut % 4 == 0)) && aligned16(Pb) && aligned16(Pout) && aligned16(Sp) &&
                    aligned16(Sv) && aligned16(XLp) && aligned16(XR) && (!out || aligned16(out)) &&
                    (!part || aligned16(part)) && (!P0 || (reinterpret_cast<uintptr_t>(P0) % 8 == 0)),
                "gasfm_edge_seam_fwd: aligned rows required");
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const SeamEpi ep{Pb, P0, pt, ln_wb, ln_bb, eps_b, Wp, ldWp, bp, Sp, Sv, ldSv, Sg, scale, Pout,
                   nullptr, nullptr, nullptr, nullptr, XLc};
  auto launch = [&](auto kern) {
    const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, 0, n_items, kWaves);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, ep, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp,
                       pos, XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max, seg_sum,
                       ldStat, part);
  };
  if (tune(GASFM_TUNE_SEAM_LDS) != 0) {
    note_dispatch(GASFM_K_SEAM_LDS);
    auto launch_lds = [&](auto kern) {
      static bool attr = false;  // > 64 KB of LDS per workgroup (static + dynamic)
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(SL_DYN));
        attr = true;
      }
      const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, SL_DYN, n_items, kWaves);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), SL_DYN, st, ep, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp,
                         ldXLp, pos, XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max,
                         seg_sum, ldStat, part);
    };
    if (ln_w)
      launch_lds(&edge_seam_lds_kernel<true>);
    else
      launch_lds(&edge_seam_lds_kernel<false>);
    return launch_status("gasfm_edge_seam_fwd");
  }
  note_dispatch(GASFM_K_SEAM_REG);
  if (ln_w && XLc)
    launch(&edge_seam_fwd_kernel<true, false, true>);
  else if (ln_w)
    launch(&edge_seam_fwd_kernel<true, false>);
  else
    launch(&edge_seam_fwd_kernel<false, false>);
  return launch_status("gasfm_edge_seam_fwd");
}

extern "C" int gasfm_edge_seam_fwd(const float* Pb, const float* P0, const int32_t* pt, const float* ln_wb,
                                   const float* ln_bb, float eps_b, const float* Wp, int32_t ldWp, const float* bp,
                                   const float* Sp, const float* Sv, int64_t ldSv, const float* Sg, float scale,
                                   float* Pout, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                   const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                   const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                   const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                   int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                   int64_t ldStat, float* part, void* stream) {
  return gasfm_edge_seam_fwd_x(Pb, P0, pt, ln_wb, ln_bb, eps_b, Wp, ldWp, bp, Sp, Sv, ldSv, Sg, scale, Pout, ln_w,
                               ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp, pos, XR, ldXR, att, bias, slope, items,
                               n_items, finalize, out, ldOut, seg_max, seg_sum, ldStat, part, nullptr, stream);
}

extern "C" int gasfm_edge0_seam_fwd(const float* P, const int32_t* pt, const float* ln_a_w, const float* ln_a_b,
                                    const float* ln_b_w, const float* ln_b_b, float eps0, const float* Wp,
                                    const float* bp, const float* Wsk, const float* bsk, const float* Sp,
                                    const float* Sv, int64_t ldSv, const float* Sg, float scale, float* Pout,
                                    const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                    const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                    const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                    const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                    int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                    int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && pt && ln_a_w && ln_a_b && ln_b_w && ln_b_b && Wp && bp && Wsk && bsk && Sp &&
                    Sv && Sg && Pout && ln_w && ln_b && Wpt && bpt && Wc && bc && XLp && XR && att && items,
                "gasfm_edge0_seam_fwd: null pointer");
  GASFM_REQUIRE((out && seg_max && seg_sum && (bias || !finalize)) || part, "gasfm_edge0_seam_fwd: no outputs");
  GASFM_REQUIRE(ldXLp >= F && ldXLp % 4 == 0 && ldXR >= F && ldXR % 4 == 0 && ldSv >= F && ldSv % 4 == 0 &&
                    (!out || (ldOut >= F && ldOut % 4 == 0)) && reinterpret_cast<uintptr_t>(P) % 8 == 0 &&
                    aligned16(Pout) && aligned16(Sp) && aligned16(Sv) && aligned16(XLp) && aligned16(XR) &&
                    (!out || aligned16(out)) && (!part || aligned16(part)),
                "gasfm_edge0_seam_fwd: aligned rows required");
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const SeamEpi ep{P, nullptr, pt, ln_a_w, ln_a_b, eps0, Wp, 2, bp, Sp, Sv, ldSv, Sg, scale, Pout,
                   ln_b_w, ln_b_b, Wsk, bsk};
  const auto kern = &edge_seam_fwd_kernel<true, true>;
  const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, 0, n_items, kWaves);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, ep, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp, pos,
                     XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max, seg_sum, ldStat, part);
  return launch_status("gasfm_edge0_seam_fwd");
}
