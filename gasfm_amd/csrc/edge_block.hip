// Fused per-edge body of a GASFM block (blocks >= 1 and the final update), gfx950.
//
// Replaces, for the E x 32 projection features of GraphAttnSfMLayer
// (code/models/layers.py:222-263) and GraphAttnSfMProjectionFeatureUpdate
// (layers.py:911-956), the reference's chain of aten kernels
//   LayerNorm -> ReLU -> cat -> GATv2 lin_l (x2, on E+N rows) -> ... ->
//   lin_proj(cat(P_hat, P0)) + Sp[pt] + Sv[cam] + Sg -> /4 -> + P
// and their autograd backward (LayerNorm backward, index_add scatters of the
// gathers, K=E weight-gradient GEMMs) with four kernels:
//
//   edge_prologue_fwd   P -> XL = [Wl_pt; Wl_cam] relu(LN(P)) + b      (LN optional)
//   edge_epilogue_fwd   P' = P + (Wp [relu(LN(P)) | P0] + bp + Sp[pt] + Sv[cam] + Sg) / 4
//   edge_epilogue_bwd   dSv (per camera), dWp, dP0 from dP'          (camera work items)
//   edge_prologue_bwd   dP = LN_bwd(mask * (Wl^T dXL + Wp^T dP'/4)) + dP', dWl, dbl, dgamma, dbeta
// plus segment_rowsum (dSp = per-point sum of dP'/4 through the point permutation).
//
// Layout: each wavefront owns 16-edge tiles.  A tile is staged row-major in the
// wave's LDS slice (row strides 34 / 66 floats: the "row per lane" reads of the
// MFMA A operand hit 32 distinct banks), the workgroup's weights are staged once
// in LDS with row stride 48 (the two k-rows one B read touches fall 16 banks
// apart), and the GEMM-shaped parts run on the exact-fp32 MFMA
// v_mfma_f32_16x16x4_f32 (lane l: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15],
// C: col = l&15, row = 4(l>>4) + r):
//   tile x W     A[i][k] = T[i][4s+g]                      -> per-edge outputs
//   T1^T x T2    A[m][k] = T1[4s+g][m], B[k][n] = T2[4s+g][n] -> reduction over edges
// Per-row reductions (LayerNorm backward) stay in registers: a row's 32 columns
// live on 16 lanes x 2 column tiles and are summed with 4 xor-shuffles.
// Weight-gradient partials are reduced over the workgroup's waves in LDS and
// written once per workgroup; gasfm_colsum finishes them (deterministic).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

using namespace tile;

// minimum waves per SIMD of the launch bounds (A/B knobs; tools/ab_lib.sh)
#ifndef GASFM_PFWD_MINWAVES
#define GASFM_PFWD_MINWAVES 1
#endif
#ifndef GASFM_EFWD_MINWAVES
#define GASFM_EFWD_MINWAVES 1
#endif
#ifndef GASFM_EBWD_MINWAVES
#define GASFM_EBWD_MINWAVES 1
#endif
#ifndef GASFM_EFWD_XCD
#define GASFM_EFWD_XCD 1  // XCD-contiguous tile ranges in the edge epilogue forward (A/B knob)
#endif
constexpr bool kEfwdXcd = GASFM_EFWD_XCD != 0;
#ifndef GASFM_XL_NT
#define GASFM_XL_NT 1
#endif
// Non-temporal (streamed) XL stores in the prologue: the 1 GB of XL would otherwise sit as dirty
// L2 / MALL lines that the next kernel (the point attention) has to write back while it reads;
// measured in-step: point attention forward 142 -> 115 us, step time unchanged (A/B knob)
constexpr bool kXlNt = GASFM_XL_NT != 0;
constexpr int kXcds = 8;  // MI355X: 8 XCDs, workgroups dispatched round-robin across them

constexpr int F = 32;            // projection feature width (n_feat_proj)
constexpr int NX = 64;           // XL width: 32 (point conv) + 32 (camera conv)
constexpr int LD34 = 34;         // LDS row stride of 32-wide tiles
constexpr int LD66 = 66;         // LDS row stride of 64-wide tiles
constexpr int LDW = 48;          // LDS row stride of staged weights (<= 32 columns)
constexpr int LDW64 = 80;        // LDS row stride of staged 64-column weights

// Load a 16 x 32 tile of P (rows row0.., global stride 32): the 8 lanes 8k..8k+7 hold row
// k + 8u (u = 0, 1).  Row layout of a 16 x 32 tile: lane l holds row (l>>3) + 8u (u = 0, 1),
// columns 4(l&7)..+3.  Rows >= nrows re-read row 0 of the tile and are NOT zeroed here: the
// loads are a prefetch one tile ahead, and a select on the loaded registers right after them
// makes the wave wait for the loads at once (s_waitcnt vmcnt), i.e. no prefetch at all.  The
// consumers mask dead rows (norm_rows32 writes zeros for them; mask_rows32 for raw rows).
__device__ __forceinline__ void load_rows32(const float* __restrict__ P, int64_t row0, int nrows, float4 (&v)[2],
                                            int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (lane >> 3) + 8 * u;
    v[u] = *reinterpret_cast<const float4*>(P + (row0 + (r < nrows ? r : 0)) * F + (lane & 7) * 4);  // see load_tile
  }
}
__device__ __forceinline__ float4 mask_row(float4 v, bool live) {
  return live ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

// LayerNorm of the row-layout registers v (rows >= nrows written as zeros): x_hat (pre-affine;
// identity when !LN) to Xh, relu(x_hat*g+b) (x when !LN) to Ph, raw values to Raw (each
// optional, LDS stride 34) and rstd to Rs.  Row statistics by 3 xor-shuffles over 8 lanes.
// LayerNorm affine parameters of this lane's 4 columns (row layout), loaded once per kernel:
// a per-tile reload is a plain load consumed at once, which drains any prefetch in flight.
struct Affine4 {
  float4 g, b;
};
template <bool LN>
__device__ __forceinline__ Affine4 load_affine(const float* __restrict__ gam, const float* __restrict__ bet,
                                               int lane) {
  Affine4 a{make_float4(1.f, 1.f, 1.f, 1.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  if (LN && gam) {
    a.g = *reinterpret_cast<const float4*>(gam + (lane & 7) * 4);
    a.b = *reinterpret_cast<const float4*>(bet + (lane & 7) * 4);
  }
  return a;
}

template <bool LN>
__device__ __forceinline__ void norm_rows32(const float4 (&v)[2], int nrows, const Affine4& af, float eps,
                                            float* Xh, float* Ph, float* Raw, float* Rs, int lane) {
  const int c = (lane & 7) * 4;
  const float4 g4 = af.g, b4 = af.b;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (lane >> 3) + 8 * u;
    const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    if (Raw) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Raw[r * LD34 + c + k] = x[k];
    }
    float mean = 0.f, rstd = 1.f;
    if (LN) {
      float s = x[0] + x[1] + x[2] + x[3];
      s = group_sum<8>(s);
      mean = s * (1.f / F);
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) q = fmaf(x[k] - mean, x[k] - mean, q);
      q = group_sum<8>(q);
      rstd = rsq_normal(q * (1.f / F) + eps);
    }
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = LN ? (x[k] - mean) * rstd : x[k];
      if (Xh) Xh[r * LD34 + c + k] = (r < nrows) ? xh : 0.f;
      if (Ph) Ph[r * LD34 + c + k] = (r < nrows) ? (LN ? fmaxf(fmaf(xh, gg[k], bb[k]), 0.f) : xh) : 0.f;
    }
    if (Rs && (lane & 7) == 0) Rs[r] = rstd;
  }
}

// =====================================================================================
// edge_prologue_fwd: XL[e] = W relu(LN(P[e])) + b     (W: [64 x 32], XL row stride ldY)
// W / b may come as two halves (W2, b2 non-null: rows 32..63), i.e. the two convs' lin_l
// parameters themselves, so the host does not concatenate them every forward
// =====================================================================================
template <bool LN>
__global__ __launch_bounds__(kThreads, GASFM_PFWD_MINWAVES) void edge_prologue_fwd_kernel(const float* __restrict__ P, int64_t E,
                                                                    const float* __restrict__ gam,
                                                                    const float* __restrict__ bet, float eps,
                                                                    const float* __restrict__ W,
                                                                    const float* __restrict__ W2,
                                                                    const float* __restrict__ b,
                                                                    const float* __restrict__ b2,
                                                                    float* __restrict__ Y, int64_t ldY,
                                                                    const int32_t* __restrict__ pos) {
  constexpr int LD68 = 68;                   // 16-byte aligned rows for the float4 read-back
  __shared__ float Wt[F * LDW64];            // W^T: Wt[k][n] = W[n][k]
  __shared__ float tiles[kWaves][TR * LD34 + TR * LD68];
  {
    tile::Stage<NX * F, kThreads> sw;
    sw.load([&](int q) { return (W2 && q >= (NX / 2) * F) ? W2[q - (NX / 2) * F] : W[q]; });
    sw.store([&](int q, float v) { Wt[(q % F) * LDW64 + q / F] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  const int c4 = (lane & 15) * 4;            // row layout: row (lane>>4) + 4u, columns c4..c4+3
  float* T = tiles[wave];
  float* Yt = T + TR * LD34;
  const float4 bias = *reinterpret_cast<const float4*>((b2 && c4 >= NX / 2) ? b2 + (c4 - NX / 2) : b + c4);
  const Affine4 af = load_affine<LN>(gam, bet, lane);
  const int64_t ntiles = (E + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  auto rows_of = [&](int64_t t) { return int(E - t * TR < TR ? E - t * TR : TR); };
  // register copy of the next tile: P rows (row layout of load_rows32) and the point-order
  // destinations of this lane's output rows (row (lane>>4) + 4u)
  float4 np[2];
  int32_t npos[4] = {0, 0, 0, 0};
  auto issue = [&](int64_t t) {
    const int64_t row0 = t * TR;
    const int nrows = rows_of(t);
    load_rows32(P, row0, nrows, np, lane);
    if (pos) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = (lane >> 4) + 4 * u;
        npos[u] = pos[row0 + (r < nrows ? r : 0)];  // clamped, no per-element branch
      }
    }
  };
  if (gw < ntiles) issue(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = rows_of(t);
    int64_t dst[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = (lane >> 4) + 4 * u;
      // the point half (columns 0..31) goes to the edge's position in point order
      dst[u] = (pos && c4 < F) ? int64_t(npos[u]) : row0 + r;
    }
    norm_rows32<LN>(np, nrows, af, eps, nullptr, T, nullptr, nullptr, lane);
    // next tile in flight during this tile's MFMA and stores (unconditional: the last tile
    // re-reads itself; a load under a branch makes the join wait for every outstanding load)
    issue(t + nw < ntiles ? t + nw : t);
    wave_sync();
    f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < F / 4; ++s) {
      const float a = T[c * LD34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(a, Wt[(4 * s + g) * LDW64 + nt * 16 + c], acc[nt]);
    }
    // C layout -> LDS -> row layout: each store instruction writes whole 128-byte half rows
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) Yt[(4 * g + r) * LD68 + nt * 16 + c] = acc[nt][r];
    wave_sync();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = (lane >> 4) + 4 * u;
      if (r < nrows) {
        const float4 y = *reinterpret_cast<const float4*>(Yt + r * LD68 + c4);
        const float4 o = make_float4(y.x + bias.x, y.y + bias.y, y.z + bias.z, y.w + bias.w);
        float4* q = reinterpret_cast<float4*>(Y + dst[u] * ldY + c4);
        if constexpr (kXlNt) {  // streamed: no dirty L2 / MALL lines left behind
          typedef float v4f __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(v4f{o.x, o.y, o.z, o.w}, reinterpret_cast<v4f*>(q));
        } else {
          *q = o;
        }
      }
    }
    wave_sync();
  }
}

// =====================================================================================
// edge_epilogue_fwd: P'[e] = P[e] + scale (Wp [relu(LN(P[e])) | P0[e]] + bp + Sp[pt] + Sv[cam] + Sg)
// Wp: [32 x ldWp] (ldWp = 34 with the init-feature skip, 32 without: P0 == null)
// =====================================================================================
__global__ __launch_bounds__(kThreads, GASFM_EFWD_MINWAVES) void edge_epilogue_fwd_kernel(
    const float* __restrict__ P, const float* __restrict__ P0, const int32_t* __restrict__ cam,
    const int32_t* __restrict__ pt, int64_t E, const float* __restrict__ gam, const float* __restrict__ bet,
    float eps, const float* __restrict__ Wp, int ldWp, const float* __restrict__ bp, const float* __restrict__ Sp,
    const float* __restrict__ Sv, int64_t ldSv, const float* __restrict__ Sg, float scale,
    float* __restrict__ Pout) {
  constexpr int LD36 = 36;                   // 16-byte aligned rows for the float4 read-back
  __shared__ float Wt[F * LDW];              // Wt[k][n] = Wp[n][k], k < 32
  __shared__ float tiles[kWaves][TR * LD34 + TR * LD36];
  {
    tile::Stage<F * F, kThreads> sw;
    sw.load([&](int q) { return Wp[(q / F) * ldWp + q % F]; });
    sw.store([&](int q, float v) { Wt[(q % F) * LDW + q / F] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  const int cc = (lane & 7) * 4;             // row layout: row (lane>>3) + 8u, columns cc..cc+3
  float* Ph = tiles[wave];
  float* Yt = Ph + TR * LD34;
  const Affine4 af = load_affine<true>(gam, bet, lane);
  float w32[4], w33[4], cst[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = cc + k;
    w32[k] = P0 ? Wp[j * ldWp + 32] : 0.f;
    w33[k] = P0 ? Wp[j * ldWp + 33] : 0.f;
    cst[k] = bp[j] + Sg[j];
  }
  const int64_t ntiles = (E + TR - 1) / TR;
  // XCD-aware tile ranges: workgroup b runs on XCD b % 8 (round-robin dispatch), so the
  // workgroups of one XCD take one contiguous eighth of the (camera-major) tiles.  The point
  // rows Sp[pt] a camera window gathers are then re-read from that XCD's L2 by the neighbouring
  // cameras instead of being fetched by all eight XCDs (1.30x -> ~1.0x of the algorithmic bytes).
  // Any placement stays correct: the eight ranges partition the tiles.
  const int nx = (kEfwdXcd && gridDim.x >= kXcds) ? kXcds : 1;
  const int xg = int(blockIdx.x % nx);
  const int64_t t_lo = ntiles * xg / nx, t_hi = ntiles * (xg + 1) / nx;
  const int64_t blk_x = (int64_t(gridDim.x) - xg + nx - 1) / nx;  // workgroups in this group
  const int64_t gw = t_lo + int64_t(blockIdx.x / nx) * kWaves + wave, nw = blk_x * kWaves;
  auto rows_of = [&](int64_t t) { return int(E - t * TR < TR ? E - t * TR : TR); };
  // register copy of the next tile (row layout): P rows, P0 pairs, camera / point indices.
  // With the indices one tile ahead, a tile's Sp / Sv gathers wait one latency, not two.
  float4 np[2];
  float2 nq[2];
  int32_t ncam[2], npt[2];
  auto issue = [&](int64_t t) {
    const int64_t row0 = t * TR;
    const int nrows = rows_of(t);
    load_rows32(P, row0, nrows, np, lane);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = (lane >> 3) + 8 * u;
      const int64_t e = row0 + (r < nrows ? r : 0);  // clamped, no per-element branch
      ncam[u] = cam[e];
      npt[u] = pt[e];
      nq[u] = P0 ? *reinterpret_cast<const float2*>(P0 + e * 2) : make_float2(0.f, 0.f);
    }
  };
  if (gw < t_hi) issue(gw);
  for (int64_t t = gw; t < t_hi; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = rows_of(t);
    // this tile's node-term gathers: their latency overlaps the LayerNorm and the MFMA
    float4 sp[2], sv[2];
    float2 q0[2];
    float4 raw[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      sp[u] = *reinterpret_cast<const float4*>(Sp + int64_t(npt[u]) * F + cc);
      sv[u] = *reinterpret_cast<const float4*>(Sv + int64_t(ncam[u]) * ldSv + cc);
      q0[u] = nq[u];
      raw[u] = np[u];
    }
    norm_rows32<true>(raw, nrows, af, eps, nullptr, Ph, nullptr, nullptr, lane);
    issue(t + nw < t_hi ? t + nw : t);  // unconditional (see edge_prologue_fwd)
    wave_sync();
    f32x4 acc[2] = {zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < F / 4; ++s) {
      const float a = Ph[c * LD34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(a, Wt[(4 * s + g) * LDW + nt * 16 + c], acc[nt]);
    }
    // C layout -> LDS -> row layout: full 128-byte rows per store
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) Yt[(4 * g + r) * LD36 + nt * 16 + c] = acc[nt][r];
    wave_sync();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = (lane >> 3) + 8 * u;
      if (r < nrows) {
        const float4 y = *reinterpret_cast<const float4*>(Yt + r * LD36 + cc);
        const float yy[4] = {y.x, y.y, y.z, y.w};
        const float spv[4] = {sp[u].x, sp[u].y, sp[u].z, sp[u].w}, svv[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
        const float rw[4] = {raw[u].x, raw[u].y, raw[u].z, raw[u].w};
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float d = yy[k] + cst[k];
          if (P0) d = fmaf(w32[k], q0[u].x, fmaf(w33[k], q0[u].y, d));
          d += spv[k] + svv[k];
          o[k] = fmaf(d, scale, rw[k]);
        }
        *reinterpret_cast<float4*>(Pout + (row0 + r) * F + cc) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    wave_sync();
  }
}

// =====================================================================================
// edge_epilogue_bwd, one wave per camera work item (contiguous edges of one camera):
//   d = dP' * scale;  dSv[cam] = sum_e d_e;  dWp += d^T [relu(LN(P)) | P0];  dP0[e] = Wp[:,32:34]^T d_e
// part layout per workgroup: [32*ldWp] dWp
// =====================================================================================
__global__ __launch_bounds__(kThreads, GASFM_EBWD_MINWAVES) void edge_epilogue_bwd_kernel(
    const gasfm_work_item* __restrict__ items, int n_items, const float* __restrict__ dPo,
    const float* __restrict__ P, const float* __restrict__ P0, const float* __restrict__ gam,
    const float* __restrict__ bet, float eps, const float* __restrict__ Wp, int ldWp, float scale,
    float* __restrict__ dSv, float* __restrict__ part_dsv, float* __restrict__ dP0, float* __restrict__ part_w) {
  __shared__ float lds[kWaves * 20 * kW > kWaves * (2 * TR * LD34 + 2 * TR) ? kWaves * 20 * kW
                                                                              : kWaves * (2 * TR * LD34 + 2 * TR)];
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* D = lds + wave * (2 * TR * LD34 + 2 * TR);
  float* Ph = D + TR * LD34;
  float* Q0 = Ph + TR * LD34;
  // dP0[e][c'] = sum_j d[e][j] Wp[j][32+c']: lane (e = c, group g) sums j in [8g, 8g+8)
  float w2[8][2];
  if (P0) {  // wave-uniform: the 16 loads issue together
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = 8 * g + k;
      w2[k][0] = Wp[j * ldWp + 32] * scale;
      w2[k][1] = Wp[j * ldWp + 33] * scale;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) w2[k][0] = w2[k][1] = 0.f;
  }
  f32x4 accW[2][2] = {{zero4(), zero4()}, {zero4(), zero4()}};
  float accP0[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  const Affine4 af = load_affine<true>(gam, bet, lane);
  // register copy of the next tile: dP' and P rows (row layout), P0 (lanes < 2*nrows)
  float4 nd[2], np[2];
  float nq = 0.f;
  // dead rows masked where staged (see load_rows32); branch-free: without P0 the P0 load reads
  // P's first words and is not used (a load under a branch makes the join wait for every load)
  const float* p0p = P0 ? P0 : P;
  auto issue = [&](int64_t row0, int nrows) {
    load_rows32(dPo, row0, nrows, nd, lane);
    load_rows32(P, row0, nrows, np, lane);
    nq = p0p[row0 * 2 + (lane < 2 * nrows ? lane : 0)];
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;
  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) issue(w.begin, rows_at(w, w.begin));
  }
  for (int it = gw; it < n_items; it += nw) {
    float dsv[2] = {0.f, 0.f};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) issue(wn.begin, rows_at(wn, wn.begin));
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      // stage the prefetched tile, then request the next one before the MFMA work
      {
        const int cc = (lane & 7) * 4;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float* d = D + ((lane >> 3) + 8 * u) * LD34 + cc;
          const float4 v = mask_row(nd[u], (lane >> 3) + 8 * u < nrows);
          d[0] = v.x;
          d[1] = v.y;
          d[2] = v.z;
          d[3] = v.w;
        }
        norm_rows32<true>(np, nrows, af, eps, nullptr, Ph, nullptr, nullptr, lane);
        if (lane < 2 * TR) Q0[lane] = (P0 && lane < 2 * nrows) ? nq : 0.f;
      }
      {  // the next tile: this item's, else the next item's first; the last one re-reads itself
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
      wave_sync();
#pragma unroll
      for (int s = 0; s < TR / 4; ++s) {
        const int row = 4 * s + g;
        float a[2], bb[2];
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          a[t2] = D[row * LD34 + t2 * 16 + c] * scale;
          bb[t2] = Ph[row * LD34 + t2 * 16 + c];
          dsv[t2] += a[t2];
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) accW[mt][nt] = mfma16(a[mt], bb[nt], accW[mt][nt]);
          if (P0) {
            accP0[mt][0] = fmaf(a[mt], Q0[2 * row], accP0[mt][0]);
            accP0[mt][1] = fmaf(a[mt], Q0[2 * row + 1], accP0[mt][1]);
          }
        }
      }
      if (P0) {
        float q0 = 0.f, q1 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = D[c * LD34 + 8 * g + k];
          q0 = fmaf(d, w2[k][0], q0);
          q1 = fmaf(d, w2[k][1], q1);
        }
        q0 = sum_groups(q0);
        q1 = sum_groups(q1);
        if (g < 2 && c < nrows) dP0[(row0 + c) * 2 + g] = g ? q1 : q0;
      }
      wave_sync();
    }
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) dsv[t2] = sum_groups(dsv[t2]);
    if (g == 0) {
      float* dst = (w.slot < 0) ? dSv + int64_t(w.seg) * F : part_dsv + int64_t(w.slot) * F;
      dst[c] = dsv[0];
      dst[16 + c] = dsv[1];
    }
    w = wn;
  }
  float v[20];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(mt * 2 + nt) * 4 + r] = accW[mt][nt][r];
  v[16] = accP0[0][0];
  v[17] = accP0[0][1];
  v[18] = accP0[1][0];
  v[19] = accP0[1][1];
  wg_reduce<20>(v, lds, wave, lane);
  if (wave == 0) {
    float* out = part_w + int64_t(blockIdx.x) * 32 * ldWp;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(mt * 16 + 4 * g + r) * ldWp + nt * 16 + c] = v[(mt * 2 + nt) * 4 + r];
    if (P0) {
      float p[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] = sum_groups(v[16 + k]);
      if (g == 0) {
        out[c * ldWp + 32] = p[0];
        out[c * ldWp + 33] = p[1];
        out[(16 + c) * ldWp + 32] = p[2];
        out[(16 + c) * ldWp + 33] = p[3];
      }
    }
  }
}

// =====================================================================================
// edge_prologue_bwd: dP = LN_bwd(mask * (W^T dXL + scale Wp[:, :32]^T dRes)) + dRes
// part layout per workgroup: [64*32 dW][64 db][32 dgamma][32 dbeta]
// =====================================================================================
constexpr int PB_WAVE = TR * LD66 + 2 * TR * LD34 + TR;  // dXL, x_hat (then dP), dRes tiles + rstd
constexpr int PB_W = NX * LDW + F * LDW;                  // W [64 x 32], scale*Wp [32 x 32]

// Register copy of one prologue_bwd tile: dXL 16x64 (lane row (l>>4)+4u, cols 4(l&15)), P and
// dRes 16x32 (lane row (l>>3)+8u, cols 4(l&7)).  The next tile's copy is requested before the
// current tile's MFMA work, so every wave keeps its loads in flight through its compute.
struct PbTile {
  float4 x[4], p[2], d[2];
};

template <bool RES>
__device__ __forceinline__ void pb_issue(PbTile& T, const float* __restrict__ dXL, int64_t ldX, int64_t row0,
                                         const float* __restrict__ P, const float* __restrict__ dRes,
                                         int nrows, int lane) {
  // Rows past the end re-read row 0 of the tile (always valid) and are zeroed afterwards: a
  // conditional load would be lowered to a flat access through a pointer select.
  // dXL: this lane's column block of the gradient (the point or the camera half, see the kernel)
  // Dead rows are masked where the tile is staged, not here (see load_rows32).
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (lane >> 4) + 4 * u;
    const int rr = r < nrows ? r : 0;
    T.x[u] = *reinterpret_cast<const float4*>(dXL + (row0 + rr) * ldX);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = (lane >> 3) + 8 * u;
    const int rr = r < nrows ? r : 0;
    T.p[u] = *reinterpret_cast<const float4*>(P + (row0 + rr) * F + (lane & 7) * 4);
    if (RES) T.d[u] = *reinterpret_cast<const float4*>(dRes + (row0 + rr) * F + (lane & 7) * 4);
  }
}

__device__ __forceinline__ void st2(float* p, float a, float b) { *reinterpret_cast<float2*>(p) = make_float2(a, b); }

template <bool LN, bool RES>
#ifndef GASFM_PBWD_MINWAVES
#define GASFM_PBWD_MINWAVES 3  // 162 VGPRs, no spills: 3 waves/SIMD (2 at 180); edge_bench 611 -> 588 us
#endif
__global__ __launch_bounds__(kThreads, GASFM_PBWD_MINWAVES) void edge_prologue_bwd_kernel(
    const float* __restrict__ dXL, int64_t ldX, const float* __restrict__ P, const float* __restrict__ dRes,
    int64_t E, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ W, const float* __restrict__ W2, const float* __restrict__ Wp, int ldWp, float scale,
    float* __restrict__ dP, float* __restrict__ part, const float* __restrict__ dXLc, int64_t ldC) {
  __shared__ float lds[PB_W + kWaves * PB_WAVE];
  float* Wl = lds;                  // B[k][j] = W[k][j]     (k < 64)
  float* Wq = lds + NX * LDW;       // B[k][j] = scale Wp[k][j] (k < 32)
  {
    tile::Stage<NX * F, kThreads> sw;
    tile::Stage<F * F, kThreads> sq;
    sw.load([&](int q) { return (W2 && q >= (NX / 2) * F) ? W2[q - (NX / 2) * F] : W[q]; });
    if (RES) sq.load([&](int q) { return Wp[(q / F) * ldWp + q % F]; });
    sw.store([&](int q, float v) { Wl[(q / F) * LDW + q % F] = v; });
    if (RES) sq.store([&](int q, float v) { Wq[(q / F) * LDW + q % F] = scale * v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T1 = lds + PB_W + wave * PB_WAVE;  // dXL            16 x 66
  float* T2 = T1 + TR * LD66;               // x_hat -> dP    16 x 34
  float* T3 = T2 + TR * LD34;               // dRes           16 x 34
  float* Rs = T3 + TR * LD34;               // rstd           16
  float gi[2], bi[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    gi[nt] = LN ? gam[nt * 16 + c] : 1.f;
    bi[nt] = LN ? bet[nt * 16 + c] : 0.f;
  }
  f32x4 accW[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) accW[mt][0] = accW[mt][1] = zero4();
  float db[4] = {0.f, 0.f, 0.f, 0.f}, dg[2] = {0.f, 0.f}, dbt[2] = {0.f, 0.f};
  const int64_t ntiles = (E + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  auto rows_of = [&](int64_t t) { return int(E - t * TR < TR ? E - t * TR : TR); };
  // columns (lane & 15) * 4 .. + 3 of the 64-wide dXL: from dXL itself, or its camera half from dXLc
  // when the two halves live in separate [E, 32] buffers (edge_cam.hip writes dXLc)
  const int c4 = (lane & 15) * 4;
  const float* dxl = (dXLc && c4 >= F) ? dXLc + (c4 - F) : dXL + c4;
  const int64_t ldx = (dXLc && c4 >= F) ? ldC : ldX;
  PbTile nxt;
  if (gw < ntiles) pb_issue<RES>(nxt, dxl, ldx, gw * TR, P, dRes, rows_of(gw), lane);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = rows_of(t);
    // stage the current tile into LDS: dXL, x_hat (+ rstd), dRes
    {
      const PbTile& cur = nxt;  // consumed before the next pb_issue overwrites it
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float* d = T1 + ((lane >> 4) + 4 * u) * LD66 + (lane & 15) * 4;
        const float4 x = mask_row(cur.x[u], (lane >> 4) + 4 * u < nrows);
        st2(d, x.x, x.y);
        st2(d + 2, x.z, x.w);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = (lane >> 3) + 8 * u;
        const float x[4] = {cur.p[u].x, cur.p[u].y, cur.p[u].z, cur.p[u].w};
        float mean = 0.f, rstd = 1.f;
        if (LN) {
          float sm = x[0] + x[1] + x[2] + x[3];
          sm = group_sum<8>(sm);
          mean = sm * (1.f / F);
          float q = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) q = fmaf(x[k] - mean, x[k] - mean, q);
          q = group_sum<8>(q);
          rstd = rsq_normal(q * (1.f / F) + eps);
        }
        const bool live = r < nrows;
        float* d = T2 + r * LD34 + (lane & 7) * 4;
        st2(d, live ? (x[0] - mean) * rstd : 0.f, live ? (x[1] - mean) * rstd : 0.f);
        st2(d + 2, live ? (x[2] - mean) * rstd : 0.f, live ? (x[3] - mean) * rstd : 0.f);
        if ((lane & 7) == 0) Rs[r] = rstd;
        if (RES) {
          float* q3 = T3 + r * LD34 + (lane & 7) * 4;
          const float4 d3 = mask_row(cur.d[u], live);
          st2(q3, d3.x, d3.y);
          st2(q3 + 2, d3.z, d3.w);
        }
      }
    }
    // request the next tile before this one's MFMA work (unconditional: the last tile re-reads
    // itself; a load under a branch makes the join wait for every outstanding load)
    {
      const int64_t tn = t + nw < ntiles ? t + nw : t;
      pb_issue<RES>(nxt, dxl, ldx, tn * TR, P, dRes, rows_of(tn), lane);
    }
    wave_sync();
    // dP_hat (C layout: edge 4g+r, column nt*16+c) = dXL W (+ dRes scale Wp)
    f32x4 acc[2] = {zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < NX / 4; ++s) {
      const float a = T1[c * LD66 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(a, Wl[(4 * s + g) * LDW + nt * 16 + c], acc[nt]);
    }
    if (RES) {
#pragma unroll
      for (int s = 0; s < F / 4; ++s) {
        const float a = T3[c * LD34 + 4 * s + g];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma16(a, Wq[(4 * s + g) * LDW + nt * 16 + c], acc[nt]);
      }
    }
    // dW += dXL^T P_hat ; db += column sums of dXL
#pragma unroll
    for (int s = 0; s < TR / 4; ++s) {
      const int row = 4 * s + g;
      float ph[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const float xh = T2[row * LD34 + nt * 16 + c];
        ph[nt] = LN ? fmaxf(fmaf(xh, gi[nt], bi[nt]), 0.f) : xh;
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const float a = T1[row * LD66 + mt * 16 + c];
        db[mt] += a;
        accW[mt][0] = mfma16(a, ph[0], accW[mt][0]);
        accW[mt][1] = mfma16(a, ph[1], accW[mt][1]);
      }
    }
    // ReLU mask + LayerNorm backward in the C layout; dx overwrites x_hat in place (each lane
    // reads then writes only its own elements)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      float gv[2], xh[2];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        xh[nt] = T2[e * LD34 + nt * 16 + c];
        float dy = acc[nt][r];
        if (LN) {
          dy = (fmaf(xh[nt], gi[nt], bi[nt]) > 0.f) ? dy : 0.f;
          dg[nt] = fmaf(dy, xh[nt], dg[nt]);
          dbt[nt] += dy;
        }
        gv[nt] = LN ? dy * gi[nt] : dy;
        s1 += gv[nt];
        s2 = fmaf(gv[nt], xh[nt], s2);
      }
      if (LN) {
        s1 = sum16(s1) * (1.f / F);
        s2 = sum16(s2) * (1.f / F);
      }
      const float rs = Rs[e];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) T2[e * LD34 + nt * 16 + c] = LN ? rs * (gv[nt] - s1 - xh[nt] * s2) : gv[nt];
    }
    wave_sync();
    // row layout: dP = dx (+ dRes), whole 128-byte rows per store
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = (lane >> 3) + 8 * u;
      if (r < nrows) {
        const int cc = (lane & 7) * 4;
        const float2 a0 = *reinterpret_cast<const float2*>(T2 + r * LD34 + cc);
        const float2 a1 = *reinterpret_cast<const float2*>(T2 + r * LD34 + cc + 2);
        float4 o = make_float4(a0.x, a0.y, a1.x, a1.y);
        if (RES) {
          const float2 d0 = *reinterpret_cast<const float2*>(T3 + r * LD34 + cc);
          const float2 d1 = *reinterpret_cast<const float2*>(T3 + r * LD34 + cc + 2);
          o.x += d0.x;
          o.y += d0.y;
          o.z += d1.x;
          o.w += d1.y;
        }
        *reinterpret_cast<float4*>(dP + (row0 + r) * F + cc) = o;
      }
    }
    wave_sync();
  }
  // workgroup reduction (LDS reused): 32 accW + 4 db + 2 dg + 2 dbt per lane
  float v[40];
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
  wg_reduce<40>(v, lds, wave, lane);
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * (NX * F + NX + 2 * F);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(mt * 16 + 4 * g + r) * F + nt * 16 + c] = v[(mt * 2 + nt) * 4 + r];
    float tt[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) tt[k] = sum_groups(v[32 + k]);
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) out[NX * F + mt * 16 + c] = tt[mt];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        out[NX * F + NX + nt * 16 + c] = tt[4 + nt];
        out[NX * F + NX + F + nt * 16 + c] = tt[6 + nt];
      }
    }
  }
}

// =====================================================================================
// segment_rowsum: out[seg] = scale * sum_{e in item} X[src_e]   (32-wide rows, optional perm)
// 8 lanes x float4 per row, 8 rows per wave, 4 row groups in flight.  Items are pipelined two
// deep across a wave's grid-stride loop (round 5): while item i's rows are in flight, item i+1's
// first 32 source indices and item i+2's descriptor are requested, so an item costs one memory
// round trip (its rows) instead of three (descriptor -> indices -> rows).  The per-lane summation
// order is unchanged: the outputs are bitwise those of the unpipelined loop.
// =====================================================================================
__device__ __forceinline__ void rowsum_idx(const int32_t* __restrict__ perm, const gasfm_work_item& w, int row,
                                           int (&src)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = w.begin + 8 * u + row;
    src[u] = e < w.end ? (perm ? perm[e] : e) : -1;
  }
}

__global__ __launch_bounds__(kThreads) void segment_rowsum_kernel(const gasfm_work_item* __restrict__ items,
                                                                 int n_items, const int32_t* __restrict__ perm,
                                                                 const float* __restrict__ X, int64_t ldX,
                                                                 float scale, float* __restrict__ out,
                                                                 float* __restrict__ part) {
  const int lane = threadIdx.x & (kW - 1);
  const int row = lane >> 3, c = (lane & 7) * 4;
  const int nw = gridDim.x * kWaves;
  const gasfm_work_item none{0, 0, 0, 0};
  int it = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + threadIdx.x / kW);
  gasfm_work_item w = it < n_items ? items[it] : none;
  gasfm_work_item wn = it + nw < n_items ? items[it + nw] : none;
  int src[4];
  rowsum_idx(perm, w, row, src);
  for (; it < n_items; it += nw) {
    // item it's first 32 rows
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = src[u] >= 0 ? *reinterpret_cast<const float4*>(X + int64_t(src[u]) * ldX + c)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
    // the next item's first indices and the one after it's descriptor, behind them
    int srcn[4];
    rowsum_idx(perm, wn, row, srcn);
    const gasfm_work_item wnn = it + 2 * nw < n_items ? items[it + 2 * nw] : none;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e0 = w.begin;;) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x;
        acc.y += v[u].y;
        acc.z += v[u].z;
        acc.w += v[u].w;
      }
      e0 += 32;
      if (e0 >= w.end) break;
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // long items: the remaining rows, 32 at a time
        const int e = e0 + 8 * u + row;
        if (e < w.end) {
          const int64_t s2 = perm ? perm[e] : e;
          v[u] = *reinterpret_cast<const float4*>(X + s2 * ldX + c);
        } else {
          v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    acc.x = xor_sum_from<8>(acc.x);
    acc.y = xor_sum_from<8>(acc.y);
    acc.z = xor_sum_from<8>(acc.z);
    acc.w = xor_sum_from<8>(acc.w);
    if (row == 0) {
      const float4 r = make_float4(acc.x * scale, acc.y * scale, acc.z * scale, acc.w * scale);
      float* dst = (w.slot < 0) ? out + int64_t(w.seg) * F : part + int64_t(w.slot) * F;
      *reinterpret_cast<float4*>(dst + c) = r;
    }
    w = wn;
    wn = wnn;
#pragma unroll
    for (int u = 0; u < 4; ++u) src[u] = srcn[u];
  }
}

// Grids: at most the workgroups resident at once (a grid-stride loop covers the rest); the
// backward partial buffers have one row per workgroup, so their size follows the same grid.
int64_t tiles_of(int64_t E) { return (E + TR - 1) / TR; }
int grid_pbwd(int64_t E) {
  return resident_grid(reinterpret_cast<const void*>(&edge_prologue_bwd_kernel<true, true>), kThreads, 0,
                       tiles_of(E), kWaves);
}
int grid_ebwd(int n_items) {
  return resident_grid(reinterpret_cast<const void*>(&edge_epilogue_bwd_kernel), kThreads, 0, n_items, kWaves);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_edge_part_floats(int32_t which, int64_t E, int32_t n_items) {
  // which: 0 = prologue_bwd partial rows, 1 = epilogue_bwd partial rows (ldWp = 34)
  return which == 0 ? grid_pbwd(E) * (NX * F + NX + 2 * F) : grid_ebwd(n_items > 0 ? n_items : 1) * 32 * 34;
}

extern "C" int gasfm_edge_prologue_fwd(const float* P, int64_t E, const float* ln_w, const float* ln_b,
                                       float eps, const float* W, const float* W2, const float* b,
                                       const float* b2, float* Y, int64_t ldY, const int32_t* pos, void* stream) {
  GASFM_REQUIRE(E >= 0 && P && W && b && Y && (!W2) == (!b2), "gasfm_edge_prologue_fwd: bad args");
  GASFM_REQUIRE(!b2 || (aligned16(b2) && aligned16(W2)), "gasfm_edge_prologue_fwd: W2/b2 not 16-byte aligned");
  GASFM_REQUIRE(ldY >= NX && ldY % 4 == 0, "gasfm_edge_prologue_fwd: ldY < 64 or not a multiple of 4");
  GASFM_REQUIRE(aligned16(P) && aligned16(Y) && aligned16(b), "gasfm_edge_prologue_fwd: P/Y/b not 16-byte aligned");
  if (E == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (ln_w) {
    const int g = resident_grid(reinterpret_cast<const void*>(&edge_prologue_fwd_kernel<true>), kThreads, 0,
                                tiles_of(E), kWaves);
    hipLaunchKernelGGL(edge_prologue_fwd_kernel<true>, dim3(g), dim3(kThreads), 0, st, P, E, ln_w, ln_b, eps, W, W2, b,
                       b2, Y, ldY, pos);
  } else {
    const int g = resident_grid(reinterpret_cast<const void*>(&edge_prologue_fwd_kernel<false>), kThreads, 0,
                                tiles_of(E), kWaves);
    hipLaunchKernelGGL(edge_prologue_fwd_kernel<false>, dim3(g), dim3(kThreads), 0, st, P, E, ln_w, ln_b, eps, W, W2, b,
                       b2, Y, ldY, pos);
  }
  return launch_status("gasfm_edge_prologue_fwd");
}

extern "C" int gasfm_edge_epilogue_fwd(const float* P, const float* P0, const int32_t* cam, const int32_t* pt,
                                       int64_t E, const float* ln_w, const float* ln_b, float eps, const float* Wp,
                                       int32_t ldWp, const float* bp, const float* Sp, const float* Sv,
                                       int64_t ldSv, const float* Sg, float scale, float* Pout, void* stream) {
  GASFM_REQUIRE(E >= 0 && P && cam && pt && ln_w && ln_b && Wp && bp && Sp && Sv && Sg && Pout,
                "gasfm_edge_epilogue_fwd: null pointer");
  GASFM_REQUIRE((P0 && ldWp == 34) || (!P0 && ldWp == 32), "gasfm_edge_epilogue_fwd: ldWp=%d vs P0", ldWp);
  GASFM_REQUIRE(ldSv >= 32 && ldSv % 4 == 0, "gasfm_edge_epilogue_fwd: ldSv=%lld", (long long)ldSv);
  GASFM_REQUIRE(aligned16(P) && aligned16(Sp) && aligned16(Sv) && aligned16(Pout) &&
                    (!P0 || reinterpret_cast<uintptr_t>(P0) % 8 == 0),
                "gasfm_edge_epilogue_fwd: P/Sp/Sv/Pout not 16-byte aligned (P0 8-byte)");
  if (E == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = resident_grid(reinterpret_cast<const void*>(&edge_epilogue_fwd_kernel), kThreads, 0, tiles_of(E),
                              kWaves);
  hipLaunchKernelGGL(edge_epilogue_fwd_kernel, dim3(g), dim3(kThreads), 0, st, P, P0, cam, pt, E, ln_w,
                     ln_b, eps, Wp, ldWp, bp, Sp, Sv, ldSv, Sg, scale, Pout);
  return launch_status("gasfm_edge_epilogue_fwd");
}

extern "C" int gasfm_edge_epilogue_bwd(const gasfm_work_item* items, int32_t n_items, const float* dPo,
                                       const float* P, const float* P0, const float* ln_w, const float* ln_b,
                                       float eps, const float* Wp, int32_t ldWp, float scale, float* dSv,
                                       float* part_dsv, float* dP0, float* part_w, void* stream) {
  GASFM_REQUIRE(items && dPo && P && ln_w && ln_b && Wp && dSv && part_w, "gasfm_edge_epilogue_bwd: null pointer");
  GASFM_REQUIRE((P0 && dP0 && ldWp == 34) || (!P0 && ldWp == 32), "gasfm_edge_epilogue_bwd: ldWp=%d vs P0",
                ldWp);
  GASFM_REQUIRE(aligned16(dPo) && aligned16(P), "gasfm_edge_epilogue_bwd: dPo/P not 16-byte aligned");
  if (n_items <= 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = grid_ebwd(n_items);
  hipLaunchKernelGGL(edge_epilogue_bwd_kernel, dim3(g), dim3(kThreads), 0, st, items, n_items, dPo, P, P0, ln_w,
                     ln_b, eps, Wp, ldWp, scale, dSv, part_dsv, dP0, part_w);
  return launch_status("gasfm_edge_epilogue_bwd");
}

extern "C" int gasfm_edge_prologue_bwd(const float* dXL, int64_t ldX, const float* P, const float* dRes, int64_t E,
                                       const float* ln_w, const float* ln_b, float eps, const float* W,
                                       const float* W2, const float* Wp, int32_t ldWp, float scale, float* dP,
                                       float* part, const float* dXLc, int64_t ldC, void* stream) {
  GASFM_REQUIRE(dXL && P && W && dP && part && ldX >= (dXLc ? F : NX), "gasfm_edge_prologue_bwd: bad args");
  GASFM_REQUIRE(!dXLc || (ldC >= F && ldC % 4 == 0 && aligned16(dXLc)), "gasfm_edge_prologue_bwd: dXLc rows");
  GASFM_REQUIRE(!dRes || Wp, "gasfm_edge_prologue_bwd: dRes needs Wp");
  GASFM_REQUIRE(aligned16(dXL) && ldX % 4 == 0 && aligned16(P) && (!dRes || aligned16(dRes)) && aligned16(dP),
                "gasfm_edge_prologue_bwd: dXL/P/dRes/dP not 16-byte aligned");
  if (E == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = grid_pbwd(E);
  const bool ln = ln_w != nullptr, res = dRes != nullptr;
#define GASFM_LAUNCH(LNV, RESV)                                                                                 \
  hipLaunchKernelGGL((edge_prologue_bwd_kernel<LNV, RESV>), dim3(g), dim3(kThreads), 0, st, dXL, ldX, P, dRes, \
                     E, ln_w, ln_b, eps, W, W2, Wp, ldWp, scale, dP, part, dXLc, ldC)
  if (ln && res)
    GASFM_LAUNCH(true, true);
  else if (ln)
    GASFM_LAUNCH(true, false);
  else if (res)
    GASFM_LAUNCH(false, true);
  else
    GASFM_LAUNCH(false, false);
#undef GASFM_LAUNCH
  return launch_status("gasfm_edge_prologue_bwd");
}

extern "C" int gasfm_segment_rowsum(const gasfm_work_item* items, int32_t n_items, const int32_t* perm,
                                    const float* X, int64_t ldX, float scale, float* out, float* part,
                                    void* stream) {
  GASFM_REQUIRE(items && X && out, "gasfm_segment_rowsum: null pointer");
  GASFM_REQUIRE(aligned16(X) && ldX % 4 == 0 && aligned16(out), "gasfm_segment_rowsum: alignment");
  if (n_items <= 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = resident_grid(reinterpret_cast<const void*>(&segment_rowsum_kernel), kThreads, 0, n_items, kWaves);
  hipLaunchKernelGGL(segment_rowsum_kernel, dim3(g), dim3(kThreads), 0, st, items,
                     n_items, perm, X, ldX, scale, out, part);
  return launch_status("gasfm_segment_rowsum");
}
