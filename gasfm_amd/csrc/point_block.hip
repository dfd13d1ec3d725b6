// Fused scene-point (64-wide row) chains of a GASFM block, gfx950.
//
// Every consumer of a block's point features p [n x 64] runs in ONE kernel per direction:
//
//   tail (produces p, reference Proj2ScenePoint.forward, code/models/layers.py:418-458):
//     x = prev + W_p agg + b_p                     proj_proj2scenepoint + state skip  :438-444
//     p = x + W_m relu(LN(x)) + b_m                norm_pre_mlp, ReLU, mlp, skip      :447-454
//   hub (consumes p):
//     s  = W_A relu(LN_A(p))                       ProjectionFeatureUpdate lin_scenepoint  :924-935
//     xl = W_B p + b_B                             ViewAndScenePoint2Global scenepoint lin_l (:560-575)
//     xr = W_D (W_C relu(LN_C(p)) + b_C) + b_D     NEXT block's norm_and_proj_scenepoint2proj
//                                                  (:429) and its GATv2 lin_r (target rows)
//   plus the identity output p -> next block's state skip (:442).
//
// The point tensor is 51 MB at config 4.  aten runs these chains as ~8 kernels forward
// (LayerNorm, clamp, GEMMs, adds) and ~20 backward, re-reading p for every consumer, and
// autograd sums the four gradients of p with three more full-size adds.  Here the backward
// of the hub reads the four upstream gradients once and writes dp once (the skip gradient
// arrives as the hub's identity output), and the tail's backward writes d prev (== dx) and
// d agg in the same pass.
//
// Layout: wave = 16-row tile (tile.hpp); GEMMs on v_mfma_f32_16x16x4_f32 against weights
// staged once per workgroup in LDS (row stride 80 for 64 columns, 48 for 32: == 16 mod 32,
// conflict-free B reads).  LayerNorm statistics are recomputed from p in the backward pass.
// Weight / bias / gamma / beta gradients leave as per-workgroup partial rows reduced by
// gasfm_colsum in a fixed order (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

using namespace tile;

constexpr int FP = 64;  // n_feat_scenepoint
constexpr int FA = 32;  // n_feat_proj (aggregation / projection width)
constexpr int L66 = 66, L34 = 34, L80 = 80, L48 = 48;
// A/B knobs (tools/point_bench.py): next-tile register prefetch in the forward / backward
// kernels, and waves per backward workgroup (8: 2 waves per SIMD at <= 256 VGPRs each; 4: one
// wave per SIMD, room for the prefetch registers without spilling)
#ifndef GASFM_PT_FWD_PREFETCH
#define GASFM_PT_FWD_PREFETCH 1
#endif
#ifndef GASFM_PT_BWD_PREFETCH
#define GASFM_PT_BWD_PREFETCH 0
#endif
#ifndef GASFM_PT_BWD_WAVES
#define GASFM_PT_BWD_WAVES 8
#endif
constexpr bool kFwdPf = GASFM_PT_FWD_PREFETCH != 0, kBwdPf = GASFM_PT_BWD_PREFETCH != 0;
constexpr int kWaves8 = GASFM_PT_BWD_WAVES, kThreads8 = kWaves8 * kW;

// partial-row layouts (floats)
constexpr int TAIL_PART = FP * FP + FP * FA + 4 * FP;                 // dWm dWp dbm dbp dgam dbet

// per-row mean / rstd of a 64-wide tile in row layout (rows_load<64>: the 16 lanes of a lane
// group hold one row) -> MS, RS
__device__ __forceinline__ void row_stats64(const float4 (&v)[4], float eps, float* MS, float* RS, int lane) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (lane >> 4) + 4 * u;
    const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    const float mean = sum16(x[0] + x[1] + x[2] + x[3]) * (1.f / FP);
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) q = fmaf(x[k] - mean, x[k] - mean, q);
    const float rstd = rsq_normal(sum16(q) * (1.f / FP) + eps);
    if ((lane & 15) == 0) {
      MS[r] = mean;
      RS[r] = rstd;
    }
  }
}

// LayerNorm + ReLU backward of one row held as 16 lanes x 4 column tiles (C layout):
// returns dx, accumulates dgamma / dbeta.  dh: upstream gradient of relu(xh*g + b).
__device__ __forceinline__ void ln_relu_bwd_row(const float (&xh)[4], const float (&dh)[4], const float (&g)[4],
                                                const float (&b)[4], float rstd, float (&dg)[4], float (&db)[4],
                                                float (&dx)[4]) {
  float gv[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const float dy = fmaf(xh[nt], g[nt], b[nt]) > 0.f ? dh[nt] : 0.f;
    dg[nt] = fmaf(dy, xh[nt], dg[nt]);
    db[nt] += dy;
    gv[nt] = dy * g[nt];
    s1 += gv[nt];
    s2 = fmaf(gv[nt], xh[nt], s2);
  }
  s1 = sum16(s1) * (1.f / FP);
  s2 = sum16(s2) * (1.f / FP);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) dx[nt] = rstd * (gv[nt] - s1 - xh[nt] * s2);
}

// Every kernel below: per 16-row tile, all global loads are issued first as coalesced float4
// rows (tile.hpp rows_load), staged into the wave's LDS slice, consumed from LDS in the MFMA
// A / B / C layouts, and the outputs leave through an LDS staging tile as float4 rows.

// ----------------------------------------------------------------------------- tail
template <bool PREV>
__global__ __launch_bounds__(kThreads) void point_tail_fwd_kernel(
    const float* __restrict__ prev, const float* __restrict__ agg, int64_t N, const float* __restrict__ Wp,
    const float* __restrict__ bp, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wm, const float* __restrict__ bm, float* __restrict__ out) {
  constexpr int PW = TR * L34 + 2 * TR * L66;  // Ag, Pv (prev, then the output), Ph
  __shared__ float WpT[FA * L80];              // WpT[j][o] = Wp[o][j]
  __shared__ float WmT[FP * L80];              // WmT[k][o] = Wm[o][k]
  __shared__ float tiles[kWaves * PW];
  {
    Stage<FP * FA, kThreads> sp;
    Stage<FP * FP, kThreads> sm;
    sp.load([&](int q) { return Wp[q]; });
    sm.load([&](int q) { return Wm[q]; });
    sp.store([&](int q, float v) { WpT[(q % FA) * L80 + q / FA] = v; });
    sm.store([&](int q, float v) { WmT[(q % FP) * L80 + q / FP] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Ag = tiles + wave * PW;
  float* Pv = Ag + TR * L34;
  float* Ph = Pv + TR * L66;
  float bpv[4], bmv[4], gv[4], bv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bpv[nt] = bp[nt * 16 + c];
    bmv[nt] = bm[nt * 16 + c];
    gv[nt] = gam[nt * 16 + c];
    bv[nt] = bet[nt * 16 + c];
  }
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  // next-tile register prefetch: tile t + nw's rows are requested right after tile t's are
  // staged, so their latency overlaps this tile's MFMA work
  float4 va[2], vp[4];
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    rows_load<FA>(agg, FA, r0, nr, va, lane);
    if (PREV) rows_load<FP>(prev, FP, r0, nr, vp, lane);
  };
  if (kFwdPf && gw < ntiles) fetch(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if constexpr (!kFwdPf) fetch(t);
    rows_to_lds<FA, L34>(Ag, va, lane);
    if (PREV) rows_to_lds<FP, L66>(Pv, vp, lane);
    if (kFwdPf && t + nw < ntiles) fetch(t + nw);
    wave_sync();
    f32x4 xa[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FA / 4; ++s) {
      const float a = Ag[c * L34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) xa[nt] = mfma16(a, WpT[(4 * s + g) * L80 + nt * 16 + c], xa[nt]);
    }
    float xv[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      float s1 = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        xv[nt][r] = xa[nt][r] + bpv[nt] + (PREV ? Pv[e * L66 + nt * 16 + c] : 0.f);
        s1 += xv[nt][r];
      }
      const float mean = sum16(s1) * (1.f / FP);
      float q = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) q = fmaf(xv[nt][r] - mean, xv[nt][r] - mean, q);
      const float rstd = rsq_normal(sum16(q) * (1.f / FP) + eps);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        Ph[e * L66 + nt * 16 + c] = fmaxf(fmaf((xv[nt][r] - mean) * rstd, gv[nt], bv[nt]), 0.f);
    }
    wave_sync();
    f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) {
      const float a = Ph[c * L66 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(a, WmT[(4 * s + g) * L80 + nt * 16 + c], acc[nt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) Pv[(4 * g + r) * L66 + nt * 16 + c] = xv[nt][r] + acc[nt][r] + bmv[nt];
    wave_sync();
    float4 vo[4];
    rows_from_lds<FP, L66>(Pv, vo, lane);
    rows_store<FP>(out, FP, row0, nrows, vo, lane);
    wave_sync();
  }
}

// dx = dout + LN_bwd(mask * (dout W_m)) (== d prev), dagg = dx W_p; partial row per workgroup
// [dWm 64x64 | dWp 64x32 | dbm 64 | dbp 64 | dgam 64 | dbet 64]
template <bool PREV>
__global__ __launch_bounds__(kThreads8) void point_tail_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ prev, const float* __restrict__ agg, int64_t N,
    const float* __restrict__ Wp, const float* __restrict__ bp, const float* __restrict__ gam,
    const float* __restrict__ bet, float eps, const float* __restrict__ Wm, float* __restrict__ dx,
    float* __restrict__ dagg, float* __restrict__ part) {
  // per wave: D (dout; dagg staging at the end), XH (prev, then LN-normalised x), DX, Ag, rstd
  constexpr int PW = 3 * TR * L66 + TR * L34 + TR;
  constexpr int NRED = 64 + 32 + 16;
  static_assert(NRED * kW <= kWaves8 * PW, "reduction scratch");
  __shared__ float WmL[FP * L80];      // WmL[o][i] = Wm[o][i]   (dout W_m)
  __shared__ float WpL[FP * L48];      // WpL[o][j] = Wp[o][j]   (dx W_p; read transposed for x)
  __shared__ float tiles[kWaves8 * PW];
  {
    Stage<FP * FA, kThreads8> sp;
    Stage<FP * FP, kThreads8> sm;
    sp.load([&](int q) { return Wp[q]; });
    sm.load([&](int q) { return Wm[q]; });
    sp.store([&](int q, float v) { WpL[(q / FA) * L48 + q % FA] = v; });
    sm.store([&](int q, float v) { WmL[(q / FP) * L80 + q % FP] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* D = tiles + wave * PW;
  float* XH = D + TR * L66;
  float* DX = XH + TR * L66;
  float* Ag = DX + TR * L66;
  float* RSt = Ag + TR * L34;
  float bpv[4], gv[4], bv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bpv[nt] = bp[nt * 16 + c];
    gv[nt] = gam[nt * 16 + c];
    bv[nt] = bet[nt * 16 + c];
  }
  f32x4 dWm[4][4], dWp[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dWm[mt][nt] = zero4();
    dWp[mt][0] = dWp[mt][1] = zero4();
  }
  float dbm[4] = {0.f, 0.f, 0.f, 0.f}, dbp[4] = {0.f, 0.f, 0.f, 0.f};
  float dg[4] = {0.f, 0.f, 0.f, 0.f}, dbt[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves8 + wave, nw = int64_t(gridDim.x) * kWaves8;
  float4 va[2], vd[4], vp[4];  // next-tile register prefetch (see point_tail_fwd_kernel)
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    rows_load<FA>(agg, FA, r0, nr, va, lane);
    rows_load<FP>(dout, FP, r0, nr, vd, lane);
    if (PREV) rows_load<FP>(prev, FP, r0, nr, vp, lane);
  };
  if (kBwdPf && gw < ntiles) fetch(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if constexpr (!kBwdPf) fetch(t);
    rows_to_lds<FA, L34>(Ag, va, lane);
    rows_to_lds<FP, L66>(D, vd, lane);
    if (PREV) rows_to_lds<FP, L66>(XH, vp, lane);
    if (kBwdPf && t + nw < ntiles) fetch(t + nw);
    wave_sync();
    // recompute x (C layout): agg W_p^T (W_p read transposed from WpL) + b_p + prev
    f32x4 xa[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FA / 4; ++s) {
      const float a = Ag[c * L34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) xa[nt] = mfma16(a, WpL[(nt * 16 + c) * L48 + 4 * s + g], xa[nt]);
    }
    if (PREV) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) xa[nt][r] += XH[(4 * g + r) * L66 + nt * 16 + c];
      wave_sync();  // prev read before XH is overwritten
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      float xr[4], s1 = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        xr[nt] = xa[nt][r] + bpv[nt];
        s1 += xr[nt];
      }
      const float mean = sum16(s1) * (1.f / FP);
      float q = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) q = fmaf(xr[nt] - mean, xr[nt] - mean, q);
      const float rstd = rsq_normal(sum16(q) * (1.f / FP) + eps);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) XH[e * L66 + nt * 16 + c] = (xr[nt] - mean) * rstd;
      if (c == 0) RSt[e] = rstd;
    }
    wave_sync();
    // d relu-out = dout W_m; LayerNorm backward; dx = dout + ... (rows past nrows: dout is 0)
    f32x4 dph[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) {
      const float a = D[c * L66 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dph[nt] = mfma16(a, WmL[(4 * s + g) * L80 + nt * 16 + c], dph[nt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      float xr[4], o[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) xr[nt] = XH[e * L66 + nt * 16 + c];
      const float dh[4] = {dph[0][r], dph[1][r], dph[2][r], dph[3][r]};
      ln_relu_bwd_row(xr, dh, gv, bv, RSt[e], dg, dbt, o);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) DX[e * L66 + nt * 16 + c] = e < nrows ? o[nt] + D[e * L66 + nt * 16 + c] : 0.f;
    }
    wave_sync();
    // dW_m += dout^T relu(LN x), dW_p += dx^T agg, biases (rows past nrows: dout, dx, agg are 0)
#ifndef GASFM_PT_NODW
#pragma unroll 1
    for (int s = 0; s < TR / 4; ++s) {
      const int row = 4 * s + g;
      float ph[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) ph[nt] = fmaxf(fmaf(XH[row * L66 + nt * 16 + c], gv[nt], bv[nt]), 0.f);
      const float ag[2] = {Ag[row * L34 + c], Ag[row * L34 + 16 + c]};
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const float a = D[row * L66 + mt * 16 + c];
        dbm[mt] += a;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dWm[mt][nt] = mfma16(a, ph[nt], dWm[mt][nt]);
        const float a2 = DX[row * L66 + mt * 16 + c];
        dbp[mt] += a2;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) dWp[mt][nt] = mfma16(a2, ag[nt], dWp[mt][nt]);
      }
    }
#endif
    // dagg = dx W_p, staged into D (dead) as 16 x 32
    f32x4 da[2] = {zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) {
      const float a = DX[c * L66 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) da[nt] = mfma16(a, WpL[(4 * s + g) * L48 + nt * 16 + c], da[nt]);
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) D[(4 * g + r) * L34 + nt * 16 + c] = da[nt][r];
    wave_sync();
    {
      float4 vx[4], vg[2];
      rows_from_lds<FP, L66>(DX, vx, lane);
      rows_from_lds<FA, L34>(D, vg, lane);
      rows_store<FP>(dx, FP, row0, nrows, vx, lane);
      rows_store<FA>(dagg, FA, row0, nrows, vg, lane);
    }
    wave_sync();
  }
  float v[NRED];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) v[(mt * 4 + nt) * 4 + r] = dWm[mt][nt][r];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) v[64 + (mt * 2 + nt) * 4 + r] = dWp[mt][nt][r];
    }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[96 + k] = dbm[k];
    v[100 + k] = dbp[k];
    v[104 + k] = dg[k];
    v[108 + k] = dbt[k];
  }
#ifndef GASFM_PT_NORED
  wg_reduce_ordered<NRED, kWaves8, kWaves8 * PW>(v, tiles, wave, lane);
#endif
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * TAIL_PART;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = mt * 16 + 4 * g + r;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) out[o * FP + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) out[FP * FP + o * FA + nt * 16 + c] = v[64 + (mt * 2 + nt) * 4 + r];
      }
    float tt[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) tt[k] = sum_groups(v[96 + k]);
    if (g == 0) {
      float* o = out + FP * FP + FP * FA;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) o[q * FP + k * 16 + c] = tt[q * 4 + k];
    }
  }
}

// ----------------------------------------------------------------------------- hub
// With the C part (the usual case) 8 waves share the 50 KB of staged weights: 121 KB of LDS, one
// workgroup = 2 waves per SIMD (4 waves were 1 per SIMD at 87 KB).
template <bool HC>
__global__ __launch_bounds__(HC ? kThreads8 : kThreads) void point_hub_fwd_kernel(
    const float* __restrict__ X, int64_t N, float eps, const float* __restrict__ gA, const float* __restrict__ bA,
    const float* __restrict__ WA, float* __restrict__ SA, const float* __restrict__ WB,
    const float* __restrict__ bB, float* __restrict__ XL, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ WC, const float* __restrict__ bWC,
    const float* __restrict__ WD, const float* __restrict__ bD, float* __restrict__ XR) {
  constexpr int NW = HC ? kWaves8 : kWaves, NT = NW * kW;
  constexpr int PW = TR * L66 + 2 * TR * L34 + 2 * TR;  // Raw (then XL staging), Tt (t, then XR), So (SA), MS, RS
  __shared__ float WAt[FP * L48];               // WAt[k][j] = W_A[j][k]
  __shared__ float WBt[FP * L80];               // WBt[k][o] = W_B[o][k]
  __shared__ float WCt[HC ? FP * L48 : 1];      // WCt[k][j] = W_C[j][k]
  __shared__ float WDt[HC ? FA * L48 : 1];      // WDt[k][j] = W_D[j][k]
  __shared__ float GB[4 * FP];                  // gamma_A beta_A gamma_C beta_C
  __shared__ float tiles[NW * PW];
  {
    Stage<FA * FP, NT> sa, sc;
    Stage<FP * FP, NT> sb;
    Stage<FA * FA, NT> sd;
    sa.load([&](int q) { return WA[q]; });
    sb.load([&](int q) { return WB[q]; });
    if (HC) {
      sc.load([&](int q) { return WC[q]; });
      sd.load([&](int q) { return WD[q]; });
    }
    sa.store([&](int q, float v) { WAt[(q % FP) * L48 + q / FP] = v; });
    sb.store([&](int q, float v) { WBt[(q % FP) * L80 + q / FP] = v; });
    if (HC) {
      sc.store([&](int q, float v) { WCt[(q % FP) * L48 + q / FP] = v; });
      sd.store([&](int q, float v) { WDt[(q % FA) * L48 + q / FA] = v; });
    }
  }
  if (threadIdx.x < FP) {
    GB[threadIdx.x] = gA[threadIdx.x];
    GB[FP + threadIdx.x] = bA[threadIdx.x];
    GB[2 * FP + threadIdx.x] = HC ? gC[threadIdx.x] : 0.f;
    GB[3 * FP + threadIdx.x] = HC ? bC[threadIdx.x] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Raw = tiles + wave * PW;
  float* Tt = Raw + TR * L66;
  float* So = Tt + TR * L34;
  float* MS = So + TR * L34;
  float* RS = MS + TR;
  float bBv[4], bCv[2], bDv[2];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bBv[nt] = bB[nt * 16 + c];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    bCv[nt] = HC ? bWC[nt * 16 + c] : 0.f;
    bDv[nt] = HC ? bD[nt * 16 + c] : 0.f;
  }
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * NW + wave, nw = int64_t(gridDim.x) * NW;
  float4 vx[4];  // next-tile register prefetch (see point_tail_fwd_kernel)
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    rows_load<FP>(X, FP, r0, int(N - r0 < TR ? N - r0 : TR), vx, lane);
  };
  if (kFwdPf && gw < ntiles) fetch(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if constexpr (!kFwdPf) fetch(t);
    row_stats64(vx, eps, MS, RS, lane);
    rows_to_lds<FP, L66>(Raw, vx, lane);
    if (kFwdPf && t + nw < ntiles) fetch(t + nw);
    wave_sync();
    const float mi = MS[c], ri = RS[c];
    f32x4 accB[4] = {zero4(), zero4(), zero4(), zero4()}, accA[2] = {zero4(), zero4()}, accC[2] = {zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) {
      const int k = 4 * s + g;
      const float a = Raw[c * L66 + k];
      const float xh = (a - mi) * ri;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) accB[nt] = mfma16(a, WBt[k * L80 + nt * 16 + c], accB[nt]);
      const float pa = fmaxf(fmaf(xh, GB[k], GB[FP + k]), 0.f);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) accA[nt] = mfma16(pa, WAt[k * L48 + nt * 16 + c], accA[nt]);
      if (HC) {
        const float pc = fmaxf(fmaf(xh, GB[2 * FP + k], GB[3 * FP + k]), 0.f);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) accC[nt] = mfma16(pc, WCt[k * L48 + nt * 16 + c], accC[nt]);
      }
    }
    wave_sync();  // Raw reads done: it becomes the XL staging tile
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) Raw[e * L66 + nt * 16 + c] = accB[nt][r] + bBv[nt];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        So[e * L34 + nt * 16 + c] = accA[nt][r];
        if (HC) Tt[e * L34 + nt * 16 + c] = accC[nt][r] + bCv[nt];
      }
    }
    wave_sync();
    f32x4 accD[2] = {zero4(), zero4()};
    if (HC) {
#pragma unroll
      for (int s = 0; s < FA / 4; ++s) {
        const float a = Tt[c * L34 + 4 * s + g];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) accD[nt] = mfma16(a, WDt[(4 * s + g) * L48 + nt * 16 + c], accD[nt]);
      }
    }
    {
      float4 vl[4], vs[2];
      rows_from_lds<FP, L66>(Raw, vl, lane);
      rows_from_lds<FA, L34>(So, vs, lane);
      rows_store<FP>(XL, FP, row0, nrows, vl, lane);
      rows_store<FA>(SA, FA, row0, nrows, vs, lane);
    }
    if (HC) {
      wave_sync();  // t reads done: Tt becomes the XR staging tile
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) Tt[(4 * g + r) * L34 + nt * 16 + c] = accD[nt][r] + bDv[nt];
      wave_sync();
      float4 vr[2];
      rows_from_lds<FA, L34>(Tt, vr, lane);
      rows_store<FA>(XR, FA, row0, nrows, vr, lane);
    }
    wave_sync();
  }
}

// The hub backward runs as two passes, each adding its terms to the incoming gradient of p:
//   C pass:  dq = dRes + LN_C_bwd(mask (dt W_C)),  dt = dXR W_D       partials HC_* layout
//   AB pass: dp = dq + dXL W_B + LN_A_bwd(mask (dSA W_A))               partials HA_* layout
// (one pass would hold 144 weight-gradient accumulators and spill at 2 waves per SIMD; the
// split costs one extra write + read of dq).  dX may alias dRes: a tile's dRes rows are in LDS
// before any of its dX rows is stored.
constexpr int HA_WA = 0, HA_WB = HA_WA + FA * FP, HA_BB = HA_WB + FP * FP, HA_GA = HA_BB + FP, HA_BA = HA_GA + FP,
              HA_PART = HA_BA + FP;
constexpr int HC_WC = 0, HC_WD = HC_WC + FA * FP, HC_BC = HC_WD + FA * FA, HC_BD = HC_BC + FA, HC_GC = HC_BD + FA,
              HC_BCL = HC_GC + FP, HC_PART = HC_BCL + FP;

template <bool HR>
__global__ __launch_bounds__(kThreads8) void point_hub_bwd_ab_kernel(
    const float* __restrict__ X, int64_t N, float eps, const float* __restrict__ gA, const float* __restrict__ bA,
    const float* __restrict__ WA, const float* __restrict__ WB, const float* __restrict__ dSA,
    const float* __restrict__ dXL, const float* dRes, float* dX, float* __restrict__ part) {
  constexpr int PW = 3 * TR * L66 + TR * L34 + 2 * TR;  // Raw, XLt (dXL), DXo (dRes, then dX), SAt (dSA), MS, RS
  constexpr int NRED = 96 + 12;
  static_assert(NRED * kW <= kWaves8 * PW, "reduction scratch");
  __shared__ float WAl[FA * L80];        // W_A [32 x 64] row-major
  __shared__ float WBl[FP * L80];        // W_B [64 x 64]
  __shared__ float GB[2 * FP];           // gamma_A beta_A
  __shared__ float tiles[kWaves8 * PW];
  {
    Stage<FA * FP, kThreads8> sa;
    Stage<FP * FP, kThreads8> sb;
    sa.load([&](int q) { return WA[q]; });
    sb.load([&](int q) { return WB[q]; });
    sa.store([&](int q, float v) { WAl[(q / FP) * L80 + q % FP] = v; });
    sb.store([&](int q, float v) { WBl[(q / FP) * L80 + q % FP] = v; });
  }
  if (threadIdx.x < FP) {
    GB[threadIdx.x] = gA[threadIdx.x];
    GB[FP + threadIdx.x] = bA[threadIdx.x];
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Raw = tiles + wave * PW;
  float* XLt = Raw + TR * L66;
  float* DXo = XLt + TR * L66;
  float* SAt = DXo + TR * L66;
  float* MS = SAt + TR * L34;
  float* RS = MS + TR;
  f32x4 dWA[2][4], dWB[4][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    dWA[0][nt] = dWA[1][nt] = zero4();
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) dWB[mt][nt] = zero4();
  }
  float dbB[4] = {0.f, 0.f, 0.f, 0.f}, dgA[4] = {0.f, 0.f, 0.f, 0.f}, dbA[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves8 + wave, nw = int64_t(gridDim.x) * kWaves8;
  float4 vx[4], vl[4], vs[2], vr[4];  // next-tile register prefetch (see point_tail_fwd_kernel)
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    rows_load<FP>(X, FP, r0, nr, vx, lane);
    rows_load<FP>(dXL, FP, r0, nr, vl, lane);
    rows_load<FA>(dSA, FA, r0, nr, vs, lane);
    if (HR) rows_load<FP>(dRes, FP, r0, nr, vr, lane);
  };
  if (kBwdPf && gw < ntiles) fetch(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if constexpr (!kBwdPf) fetch(t);
    row_stats64(vx, eps, MS, RS, lane);
    rows_to_lds<FP, L66>(Raw, vx, lane);
    rows_to_lds<FP, L66>(XLt, vl, lane);
    rows_to_lds<FA, L34>(SAt, vs, lane);
    if (HR) rows_to_lds<FP, L66>(DXo, vr, lane);
    if (kBwdPf && t + nw < ntiles) fetch(t + nw);
    wave_sync();
    // weight gradients over the tile's rows (row = 4s + g; rows past nrows: dSA, dXL are 0)
#pragma unroll 1
    for (int s = 0; s < TR / 4; ++s) {
      const int row = 4 * s + g;
      const float mr = MS[row], rr = RS[row];
      float xr[4], pa[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        xr[nt] = Raw[row * L66 + nt * 16 + c];
        pa[nt] = fmaxf(fmaf((xr[nt] - mr) * rr, GB[nt * 16 + c], GB[FP + nt * 16 + c]), 0.f);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const float a = SAt[row * L34 + mt * 16 + c];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dWA[mt][nt] = mfma16(a, pa[nt], dWA[mt][nt]);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const float a = XLt[row * L66 + mt * 16 + c];
        dbB[mt] += a;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dWB[mt][nt] = mfma16(a, xr[nt], dWB[mt][nt]);
      }
    }
    // data gradient (C layout: row 4g+r, column nt*16+c)
    f32x4 dxb[4] = {zero4(), zero4(), zero4(), zero4()}, dp[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) {
      const float a = XLt[c * L66 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dxb[nt] = mfma16(a, WBl[(4 * s + g) * L80 + nt * 16 + c], dxb[nt]);
    }
#pragma unroll
    for (int s = 0; s < FA / 4; ++s) {
      const float a = SAt[c * L34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dp[nt] = mfma16(a, WAl[(4 * s + g) * L80 + nt * 16 + c], dp[nt]);
    }
    float gc[4], bc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      gc[nt] = GB[nt * 16 + c];
      bc[nt] = GB[FP + nt * 16 + c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      const float me = MS[e], re = RS[e];
      float xh[4], t1[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) xh[nt] = (Raw[e * L66 + nt * 16 + c] - me) * re;
      const float dh[4] = {dp[0][r], dp[1][r], dp[2][r], dp[3][r]};
      ln_relu_bwd_row(xh, dh, gc, bc, re, dgA, dbA, t1);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        float* d = DXo + e * L66 + nt * 16 + c;
        *d = dxb[nt][r] + t1[nt] + (HR ? *d : 0.f);
      }
    }
    wave_sync();
    {
      float4 vo[4];
      rows_from_lds<FP, L66>(DXo, vo, lane);
      rows_store<FP>(dX, FP, row0, nrows, vo, lane);
    }
    wave_sync();
  }
  float v[NRED];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) v[(mt * 4 + nt) * 4 + r] = dWA[mt][nt][r];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) v[32 + (mt * 4 + nt) * 4 + r] = dWB[mt][nt][r];
    }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[96 + k] = dbB[k];
    v[100 + k] = dgA[k];
    v[104 + k] = dbA[k];
  }
#ifndef GASFM_PT_NORED
  wg_reduce_ordered<NRED, kWaves8, kWaves8 * PW>(v, tiles, wave, lane);
#endif
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * HA_PART;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) out[HA_WA + (mt * 16 + 4 * g + r) * FP + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          out[HA_WB + (mt * 16 + 4 * g + r) * FP + nt * 16 + c] = v[32 + (mt * 4 + nt) * 4 + r];
      }
    float tt[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) tt[k] = sum_groups(v[96 + k]);
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        out[HA_BB + k * 16 + c] = tt[k];
        out[HA_GA + k * 16 + c] = tt[4 + k];
        out[HA_BA + k * 16 + c] = tt[8 + k];
      }
    }
  }
}

template <bool HR>
__global__ __launch_bounds__(kThreads8) void point_hub_bwd_c_kernel(
    const float* __restrict__ X, int64_t N, float eps, const float* __restrict__ gC, const float* __restrict__ bC,
    const float* __restrict__ WC, const float* __restrict__ bWC, const float* __restrict__ WD,
    const float* __restrict__ dXR, const float* dRes, float* dX, float* __restrict__ part) {
  // per wave: Raw, DXo (dRes, then dX), XRt (dXR), Dt (dt), Tt (t), MS, RS
  constexpr int PW = 2 * TR * L66 + 3 * TR * L34 + 2 * TR;
  constexpr int NRED = 48 + 12;
  static_assert(NRED * kW <= kWaves8 * PW, "reduction scratch");
  __shared__ float WCl[FA * L80];        // W_C [32 x 64]
  __shared__ float WCt[FP * L48];        // W_C^T
  __shared__ float WDl[FA * L48];        // W_D [32 x 32]
  __shared__ float GB[2 * FP];           // gamma_C beta_C
  __shared__ float tiles[kWaves8 * PW];
  {
    Stage<FA * FP, kThreads8> sc;
    Stage<FA * FA, kThreads8> sd;
    sc.load([&](int q) { return WC[q]; });
    sd.load([&](int q) { return WD[q]; });
    sc.store([&](int q, float v) {
      WCl[(q / FP) * L80 + q % FP] = v;
      WCt[(q % FP) * L48 + q / FP] = v;
    });
    sd.store([&](int q, float v) { WDl[(q / FA) * L48 + q % FA] = v; });
  }
  if (threadIdx.x < FP) {
    GB[threadIdx.x] = gC[threadIdx.x];
    GB[FP + threadIdx.x] = bC[threadIdx.x];
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Raw = tiles + wave * PW;
  float* DXo = Raw + TR * L66;
  float* XRt = DXo + TR * L66;
  float* Dt = XRt + TR * L34;
  float* Tt = Dt + TR * L34;
  float* MS = Tt + TR * L34;
  float* RS = MS + TR;
  const float bWCv[2] = {bWC[c], bWC[16 + c]};
  f32x4 dWC[2][4], dWD[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dWC[mt][nt] = zero4();
    dWD[mt][0] = dWD[mt][1] = zero4();
  }
  float dbC[2] = {0.f, 0.f}, dbD[2] = {0.f, 0.f}, dgC[4] = {0.f, 0.f, 0.f, 0.f}, dbCl[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves8 + wave, nw = int64_t(gridDim.x) * kWaves8;
  float4 vx[4], vq[2], vr[4];  // next-tile register prefetch (see point_tail_fwd_kernel)
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    rows_load<FP>(X, FP, r0, nr, vx, lane);
    rows_load<FA>(dXR, FA, r0, nr, vq, lane);
    if (HR) rows_load<FP>(dRes, FP, r0, nr, vr, lane);
  };
  if (kBwdPf && gw < ntiles) fetch(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if constexpr (!kBwdPf) fetch(t);
    row_stats64(vx, eps, MS, RS, lane);
    rows_to_lds<FP, L66>(Raw, vx, lane);
    rows_to_lds<FA, L34>(XRt, vq, lane);
    if (HR) rows_to_lds<FP, L66>(DXo, vr, lane);
    if (kBwdPf && t + nw < ntiles) fetch(t + nw);
    wave_sync();
    const float mi = MS[c], ri = RS[c];
    // t = W_C relu(LN_C p) + b_C (recomputed), dt = dXR W_D
    f32x4 ta[2] = {zero4(), zero4()}, da[2] = {zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) {
      const int k = 4 * s + g;
      const float pc = fmaxf(fmaf((Raw[c * L66 + k] - mi) * ri, GB[k], GB[FP + k]), 0.f);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) ta[nt] = mfma16(pc, WCt[k * L48 + nt * 16 + c], ta[nt]);
    }
#pragma unroll
    for (int s = 0; s < FA / 4; ++s) {
      const float a = XRt[c * L34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) da[nt] = mfma16(a, WDl[(4 * s + g) * L48 + nt * 16 + c], da[nt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        Tt[(4 * g + r) * L34 + nt * 16 + c] = ta[nt][r] + bWCv[nt];
        Dt[(4 * g + r) * L34 + nt * 16 + c] = da[nt][r];
      }
    wave_sync();
    // dW_C += dt^T relu(LN_C p), dW_D += dXR^T t (row = 4s + g; rows past nrows: dXR, dt are 0)
#pragma unroll
    for (int s = 0; s < TR / 4; ++s) {
      const int row = 4 * s + g;
      const float mr = MS[row], rr = RS[row];
      float pc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        pc[nt] = fmaxf(fmaf((Raw[row * L66 + nt * 16 + c] - mr) * rr, GB[nt * 16 + c], GB[FP + nt * 16 + c]), 0.f);
      const float tt[2] = {Tt[row * L34 + c], Tt[row * L34 + 16 + c]};
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const float a = Dt[row * L34 + mt * 16 + c];
        dbC[mt] += a;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dWC[mt][nt] = mfma16(a, pc[nt], dWC[mt][nt]);
        const float a2 = XRt[row * L34 + mt * 16 + c];
        dbD[mt] += a2;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) dWD[mt][nt] = mfma16(a2, tt[nt], dWD[mt][nt]);
      }
    }
    // data gradient: dq = dRes + LN_C_bwd(mask (dt W_C))
    f32x4 dp[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FA / 4; ++s) {
      const float a = Dt[c * L34 + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dp[nt] = mfma16(a, WCl[(4 * s + g) * L80 + nt * 16 + c], dp[nt]);
    }
    float gc[4], bc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      gc[nt] = GB[nt * 16 + c];
      bc[nt] = GB[FP + nt * 16 + c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      const float me = MS[e], re = RS[e];
      float xh[4], t1[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) xh[nt] = (Raw[e * L66 + nt * 16 + c] - me) * re;
      const float dh[4] = {dp[0][r], dp[1][r], dp[2][r], dp[3][r]};
      ln_relu_bwd_row(xh, dh, gc, bc, re, dgC, dbCl, t1);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        float* d = DXo + e * L66 + nt * 16 + c;
        *d = t1[nt] + (HR ? *d : 0.f);
      }
    }
    wave_sync();
    {
      float4 vo[4];
      rows_from_lds<FP, L66>(DXo, vo, lane);
      rows_store<FP>(dX, FP, row0, nrows, vo, lane);
    }
    wave_sync();
  }
  float v[NRED];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) v[(mt * 4 + nt) * 4 + r] = dWC[mt][nt][r];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) v[32 + (mt * 2 + nt) * 4 + r] = dWD[mt][nt][r];
    }
  v[48] = dbC[0];
  v[49] = dbC[1];
  v[50] = dbD[0];
  v[51] = dbD[1];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[52 + k] = dgC[k];
    v[56 + k] = dbCl[k];
  }
#ifndef GASFM_PT_NORED
  wg_reduce_ordered<NRED, kWaves8, kWaves8 * PW>(v, tiles, wave, lane);
#endif
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * HC_PART;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int o = mt * 16 + 4 * g + r;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) out[HC_WC + o * FP + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) out[HC_WD + o * FA + nt * 16 + c] = v[32 + (mt * 2 + nt) * 4 + r];
      }
    float tt[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) tt[k] = sum_groups(v[48 + k]);
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        out[HC_BC + k * 16 + c] = tt[k];
        out[HC_BD + k * 16 + c] = tt[2 + k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        out[HC_GC + k * 16 + c] = tt[4 + k];
        out[HC_BCL + k * 16 + c] = tt[8 + k];
      }
    }
  }
}

// ----------------------------------------------------------------------------- forward, register-resident
// The forward kernels above stage every 16-row tile through LDS twice per layer (rows in, C layout
// out, A layout back in).  Computing the TRANSPOSED products Y^T = W X^T instead keeps a tile in
// registers from load to store: with A = W and B = X^T, v_mfma_f32_16x16x4_f32 leaves lane
// (g = lane>>4, c = lane&15) holding Y[row c][16 ot + 4 g + r] (r < 4) -- 16 features of row c --
// and those registers are exactly the B operand of the next layer when its k index is permuted
// to k = 16 u + 4 g + j at step (u, j) (any consistent k order gives the same sum).  The weights
// are staged once per workgroup pre-permuted to match, as float4 slabs read with one conflict-free
// ds_read_b128 per 4 MFMAs.  Rows load and store as float4 (64 B per row per slab).  Row
// statistics: 16 values per lane, then a sum over the 4 lane groups.  Only weights live in LDS
// (24-37 KB per workgroup), so occupancy is set by VGPRs.
#ifndef GASFM_PT_FWD_T
#define GASFM_PT_FWD_T 1
#endif
#ifndef GASFM_PT_FWD_T_MINW
#define GASFM_PT_FWD_T_MINW 1
#endif
// 1: re-read the weight slabs from LDS every tile (a compiler memory barrier at the top of the
// tile loop keeps them from being hoisted into registers: ~100 fewer VGPRs, more waves per SIMD);
// 0: the compiler keeps them in VGPRs across tiles
#ifndef GASFM_PT_FWD_T_LDSW
#define GASFM_PT_FWD_T_LDSW 1
#endif
// waves per workgroup (4, 8 and 16 measured: 16 slowest, 4 and 8 within 1 us)
#ifndef GASFM_PT_FWD_T_WAVES
#define GASFM_PT_FWD_T_WAVES 4
#endif
constexpr int kWavesT = GASFM_PT_FWD_T_WAVES, kThreadsT = kWavesT * kW;

// W [O x K] (torch Linear [out, in]) -> float4 slabs Q[(ot * (K/16) + u) * 64 + 16 g + c] =
// (W[16 ot + c][16 u + 4 g + j], j < 4)
template <int O, int K, int NT>
__device__ __forceinline__ void stage_slabs(const float* __restrict__ W, float* Q) {
  Stage<O * K, NT> s;
  s.load([&](int q) { return W[q]; });
  s.store([&](int q, float v) {
    const int o = q / K, k = q % K;
    Q[(((o / 16) * (K / 16) + k / 16) * 64 + ((k % 16) / 4) * 16 + o % 16) * 4 + k % 4] = v;
  });
}

// acc[ot] += W . X^T over K = 16 KU (X as k-slabs xk[u] = X[row c][16 u + 4 g + j])
template <int OT, int KU>
__device__ __forceinline__ void layer_t(const float4* __restrict__ Q, const f32x4 (&xk)[KU], f32x4 (&acc)[OT],
                                        int lane) {
  // the OT accumulators interleaved (consecutive MFMAs independent: a dependent chain waits the
  // full pipeline latency per step), and the next k-slab's weights read from LDS while this one's
  // MFMAs run
  float4 w[OT];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) w[ot] = Q[ot * KU * 64 + lane];
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    float4 wn[OT];
    if (u + 1 < KU) {
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) wn[ot] = Q[(ot * KU + u + 1) * 64 + lane];
    }
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].x, xk[u][0], acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].y, xk[u][1], acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].z, xk[u][2], acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(w[ot].w, xk[u][3], acc[ot]);
    if (u + 1 < KU) {
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) w[ot] = wn[ot];
    }
  }
}

// per-feature vector V[64] (LDS) at this lane's features 16 ot + 4 g + r
__device__ __forceinline__ f32x4 vec_at(const float* V, int ot, int g) {
  const float4 v = *reinterpret_cast<const float4*>(V + 16 * ot + 4 * g);
  return f32x4{v.x, v.y, v.z, v.w};
}

// slab u of row c (clamped to a valid row; rows past nrows are computed and not stored)
template <int W>
__device__ __forceinline__ void slabs_load(const float* __restrict__ X, int64_t row0, int nrows, f32x4 (&v)[W / 16],
                                           int lane) {
  const int c = lane & 15, g = lane >> 4;
  const float* p = X + (row0 + (c < nrows ? c : nrows - 1)) * W + 4 * g;
#pragma unroll
  for (int u = 0; u < W / 16; ++u) {
    const float4 t = *reinterpret_cast<const float4*>(p + 16 * u);
    v[u] = f32x4{t.x, t.y, t.z, t.w};
  }
}
template <int W>
__device__ __forceinline__ void slabs_store(float* __restrict__ X, int64_t row0, int nrows, const f32x4 (&v)[W / 16],
                                            int lane) {
  const int c = lane & 15, g = lane >> 4;
  if (c >= nrows) return;
  float* p = X + (row0 + c) * W + 4 * g;
#pragma unroll
  for (int u = 0; u < W / 16; ++u) *reinterpret_cast<float4*>(p + 16 * u) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
}

// mean and rstd of the 64-wide rows held as 4 slabs per lane (row c over the 4 lane groups)
__device__ __forceinline__ void slab_stats(const f32x4 (&x)[4], float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) s += (x[u][0] + x[u][1]) + (x[u][2] + x[u][3]);
  mean = sum_groups(s) * (1.f / FP);
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) q = fmaf(x[u][j] - mean, x[u][j] - mean, q);
  rstd = rsq_normal(sum_groups(q) * (1.f / FP) + eps);
}

// One 16-row tile of the tail in registers (T layout in, T layout out): y = x + W_m relu(LN(x)) + b_m,
// x = prev + W_p agg + b_p; V = [b_p | gamma | beta | b_m] in LDS.  Shared by the tail kernel and the
// fused tail + hub kernel (the same instruction sequence: bitwise the same p).
__device__ __forceinline__ void tail_tile_t(const float4* __restrict__ WpQ, const float4* __restrict__ WmQ,
                                            const float* V, const f32x4 (&ag)[2], const f32x4 (&pv)[4], float eps,
                                            int lane, f32x4 (&y)[4]) {
  const int g = lane >> 4;
  f32x4 x[4];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) x[ot] = vec_at(V, ot, g) + pv[ot];  // b_p + prev, then + W_p agg
  layer_t<4, 2>(WpQ, ag, x, lane);
  f32x4 gm[4], bt[4];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) {
    gm[ot] = vec_at(V + FP, ot, g);
    bt[ot] = vec_at(V + 2 * FP, ot, g);
  }
  float mean, rstd;
  slab_stats(x, eps, mean, rstd);
  f32x4 h[4];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
#pragma unroll
    for (int j = 0; j < 4; ++j) h[ot][j] = fmaxf(fmaf((x[ot][j] - mean) * rstd, gm[ot][j], bt[ot][j]), 0.f);
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) y[ot] = vec_at(V + 3 * FP, ot, g);  // b_m, then + W_m h
  layer_t<4, 4>(WmQ, h, y, lane);
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) y[ot] = x[ot] + y[ot];
}

// One 16-row tile of the hub on p in registers (T layout): XL = W_B p + b_B, SA = W_A relu(LN_A p),
// (HC) XR = W_D (W_C relu(LN_C p) + b_C) + b_D, stored as rows row0 .. row0 + nrows - 1.
// V = [gamma_A | beta_A | gamma_C | beta_C | b_B | b_C (32) | b_D (32)] in LDS.
template <bool HC>
__device__ __forceinline__ void hub_tile_t(const f32x4 (&p)[4], float eps, const float4* __restrict__ WAQ,
                                           const float4* __restrict__ WBQ, const float4* __restrict__ WCQ,
                                           const float4* __restrict__ WDQ, const float* V, int lane, int64_t row0,
                                           int nrows, float* __restrict__ SA, float* __restrict__ XL,
                                           float* __restrict__ XR) {
  const int g = lane >> 4;
  float mean, rstd;
  slab_stats(p, eps, mean, rstd);
  {
    f32x4 xl[4];
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) xl[ot] = vec_at(V + 4 * FP, ot, g);  // b_B, then + W_B p
    layer_t<4, 4>(WBQ, p, xl, lane);
    slabs_store<FP>(XL, row0, nrows, xl, lane);
  }
  f32x4 h[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 gm = vec_at(V, u, g), bt = vec_at(V + FP, u, g);
#pragma unroll
    for (int j = 0; j < 4; ++j) h[u][j] = fmaxf(fmaf((p[u][j] - mean) * rstd, gm[j], bt[j]), 0.f);
  }
  {
    f32x4 sa[2] = {zero4(), zero4()};
    layer_t<2, 4>(WAQ, h, sa, lane);
    slabs_store<FA>(SA, row0, nrows, sa, lane);
  }
  if (HC) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 gm = vec_at(V + 2 * FP, u, g), bt = vec_at(V + 3 * FP, u, g);
#pragma unroll
      for (int j = 0; j < 4; ++j) h[u][j] = fmaxf(fmaf((p[u][j] - mean) * rstd, gm[j], bt[j]), 0.f);
    }
    f32x4 tq[2] = {vec_at(V + 5 * FP, 0, g), vec_at(V + 5 * FP, 1, g)};  // b_C, then + W_C h
    layer_t<2, 4>(WCQ, h, tq, lane);
    f32x4 xr[2] = {vec_at(V + 5 * FP + FA, 0, g), vec_at(V + 5 * FP + FA, 1, g)};  // b_D, then + W_D t
    layer_t<2, 2>(WDQ, tq, xr, lane);
    slabs_store<FA>(XR, row0, nrows, xr, lane);
  }
}

// weights and vectors of the hub in LDS (every thread of the workgroup takes part)
template <bool HC, int NT>
__device__ __forceinline__ void hub_stage_t(const float* __restrict__ gA, const float* __restrict__ bA,
                                            const float* __restrict__ WA, const float* __restrict__ WB,
                                            const float* __restrict__ bB, const float* __restrict__ gC,
                                            const float* __restrict__ bC, const float* __restrict__ WC,
                                            const float* __restrict__ bWC, const float* __restrict__ WD,
                                            const float* __restrict__ bD, float4* WAQ, float4* WBQ, float4* WCQ,
                                            float4* WDQ, float* V) {
  stage_slabs<FA, FP, NT>(WA, reinterpret_cast<float*>(WAQ));
  stage_slabs<FP, FP, NT>(WB, reinterpret_cast<float*>(WBQ));
  if (HC) {
    stage_slabs<FA, FP, NT>(WC, reinterpret_cast<float*>(WCQ));
    stage_slabs<FA, FA, NT>(WD, reinterpret_cast<float*>(WDQ));
  }
  if (threadIdx.x < FP) {
    V[threadIdx.x] = gA[threadIdx.x];
    V[FP + threadIdx.x] = bA[threadIdx.x];
    V[2 * FP + threadIdx.x] = HC ? gC[threadIdx.x] : 0.f;
    V[3 * FP + threadIdx.x] = HC ? bC[threadIdx.x] : 0.f;
    V[4 * FP + threadIdx.x] = bB[threadIdx.x];
    if (threadIdx.x < FA) {
      V[5 * FP + threadIdx.x] = HC ? bWC[threadIdx.x] : 0.f;
      V[5 * FP + FA + threadIdx.x] = HC ? bD[threadIdx.x] : 0.f;
    }
  }
}

template <bool PREV>
__global__ __launch_bounds__(kThreadsT, GASFM_PT_FWD_T_MINW) void point_tail_fwd_t_kernel(
    const float* __restrict__ prev, const float* __restrict__ agg, int64_t N, const float* __restrict__ Wp,
    const float* __restrict__ bp, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wm, const float* __restrict__ bm, float* __restrict__ out) {
  __shared__ float4 WpQ[FP * FA / 4], WmQ[FP * FP / 4];
  __shared__ float V[4 * FP];  // b_p gamma beta b_m
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWavesT + wave, nw = int64_t(gridDim.x) * kWavesT;
  f32x4 na[2], np[4];  // next tile's rows, requested before this tile's MFMA work
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    slabs_load<FA>(agg, r0, nr, na, lane);
    if (PREV) slabs_load<FP>(prev, r0, nr, np, lane);
  };
  if (gw < ntiles) fetch(gw);  // the first tile's rows fly while the weights are staged
  stage_slabs<FP, FA, kThreadsT>(Wp, reinterpret_cast<float*>(WpQ));
  stage_slabs<FP, FP, kThreadsT>(Wm, reinterpret_cast<float*>(WmQ));
  if (threadIdx.x < FP) {
    V[threadIdx.x] = bp[threadIdx.x];
    V[FP + threadIdx.x] = gam[threadIdx.x];
    V[2 * FP + threadIdx.x] = bet[threadIdx.x];
    V[3 * FP + threadIdx.x] = bm[threadIdx.x];
  }
  __syncthreads();
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if (GASFM_PT_FWD_T_LDSW) asm volatile("" ::: "memory");
    f32x4 ag[2] = {na[0], na[1]}, pv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pv[u] = PREV ? np[u] : zero4();
    if (t + nw < ntiles) fetch(t + nw);
    f32x4 y[4];
    tail_tile_t(WpQ, WmQ, V, ag, pv, eps, lane, y);
    slabs_store<FP>(out, row0, nrows, y, lane);
  }
}

template <bool HC>
__global__ __launch_bounds__(kThreadsT, GASFM_PT_FWD_T_MINW) void point_hub_fwd_t_kernel(
    const float* __restrict__ X, int64_t N, float eps, const float* __restrict__ gA, const float* __restrict__ bA,
    const float* __restrict__ WA, float* __restrict__ SA, const float* __restrict__ WB,
    const float* __restrict__ bB, float* __restrict__ XL, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ WC, const float* __restrict__ bWC,
    const float* __restrict__ WD, const float* __restrict__ bD, float* __restrict__ XR) {
  __shared__ float4 WAQ[FA * FP / 4], WBQ[FP * FP / 4], WCQ[HC ? FA * FP / 4 : 1], WDQ[HC ? FA * FA / 4 : 1];
  __shared__ float V[5 * FP + 2 * FA];  // gamma_A beta_A gamma_C beta_C b_B | b_C b_D
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWavesT + wave, nw = int64_t(gridDim.x) * kWavesT;
  f32x4 nx[4];
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    slabs_load<FP>(X, r0, int(N - r0 < TR ? N - r0 : TR), nx, lane);
  };
  if (gw < ntiles) fetch(gw);  // the first tile's rows fly while the weights are staged
  hub_stage_t<HC, kThreadsT>(gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, WAQ, WBQ, WCQ, WDQ, V);
  __syncthreads();
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if (GASFM_PT_FWD_T_LDSW) asm volatile("" ::: "memory");
    f32x4 p[4] = {nx[0], nx[1], nx[2], nx[3]};
    if (t + nw < ntiles) fetch(t + nw);
    hub_tile_t<HC>(p, eps, WAQ, WBQ, WCQ, WDQ, V, lane, row0, nrows, SA, XL, XR);
  }
}

// The tail and the hub in ONE pass (round 6): p = tail(prev, agg) stays in registers between the two
// bodies (the tail's T-layout output is the hub's T-layout input), is stored once as the block's
// point features, and feeds the hub's consumers directly: no re-read of p, one launch and one weight
// staging fewer per block.  Same tile bodies as the two kernels: bitwise the same outputs.
template <bool PREV, bool HC, int NWV>
__global__ __launch_bounds__(NWV * kW) void point_tail_hub_fwd_t_kernel(
    const float* __restrict__ prev, const float* __restrict__ agg, int64_t N, const float* __restrict__ Wp,
    const float* __restrict__ bp, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wm, const float* __restrict__ bm, float* __restrict__ out, float eps_h,
    const float* __restrict__ gA, const float* __restrict__ bA, const float* __restrict__ WA, float* __restrict__ SA,
    const float* __restrict__ WB, const float* __restrict__ bB, float* __restrict__ XL,
    const float* __restrict__ gC, const float* __restrict__ bC, const float* __restrict__ WC,
    const float* __restrict__ bWC, const float* __restrict__ WD, const float* __restrict__ bD,
    float* __restrict__ XR) {
  __shared__ float4 WpQ[FP * FA / 4], WmQ[FP * FP / 4];
  __shared__ float4 WAQ[FA * FP / 4], WBQ[FP * FP / 4], WCQ[HC ? FA * FP / 4 : 1], WDQ[HC ? FA * FA / 4 : 1];
  __shared__ float VT[4 * FP];               // b_p gamma beta b_m
  __shared__ float VH[5 * FP + 2 * FA];      // the hub's vectors (hub_stage_t)
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * NWV + wave, nw = int64_t(gridDim.x) * NWV;
  f32x4 na[2], np[4];
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    slabs_load<FA>(agg, r0, nr, na, lane);
    if (PREV) slabs_load<FP>(prev, r0, nr, np, lane);
  };
  if (gw < ntiles) fetch(gw);
  stage_slabs<FP, FA, NWV * kW>(Wp, reinterpret_cast<float*>(WpQ));
  stage_slabs<FP, FP, NWV * kW>(Wm, reinterpret_cast<float*>(WmQ));
  if (threadIdx.x < FP) {
    VT[threadIdx.x] = bp[threadIdx.x];
    VT[FP + threadIdx.x] = gam[threadIdx.x];
    VT[2 * FP + threadIdx.x] = bet[threadIdx.x];
    VT[3 * FP + threadIdx.x] = bm[threadIdx.x];
  }
  hub_stage_t<HC, NWV * kW>(gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, WAQ, WBQ, WCQ, WDQ, VH);
  __syncthreads();
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    if (GASFM_PT_FWD_T_LDSW) asm volatile("" ::: "memory");
    f32x4 ag[2] = {na[0], na[1]}, pv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pv[u] = PREV ? np[u] : zero4();
    if (t + nw < ntiles) fetch(t + nw);
    f32x4 p[4];
    tail_tile_t(WpQ, WmQ, VT, ag, pv, eps, lane, p);
    slabs_store<FP>(out, row0, nrows, p, lane);
    hub_tile_t<HC>(p, eps_h, WAQ, WBQ, WCQ, WDQ, VH, lane, row0, nrows, SA, XL, XR);
  }
}

// ----------------------------------------------------------------------------- backward, register-resident
// The backward needs every row tensor in two register layouts:
//   T (slab) layout  lane (g, c), f32x4 v[u]:  V[row c][16 u + 4 g + j]      (k = features along g)
//   C layout         lane (g, c), f32x4 v[ft]: V[row 4 g + r][16 ft + c]     (k = rows along g)
// A product over FEATURES (Y = X W^T) takes X in T layout; with X as the A operand the result
// lands in C layout (layer_c), with X as the B operand in T layout (layer_t).  A weight gradient
// (dW = dY^T X, K = rows) takes BOTH operands in C layout with the row index in the order 4 g + s
// at step s: no LDS at all.  So the loaded tensors are read in the layouts their consumers want
// (T: 16-B loads of 64-B row chunks; C: 4-B loads, 64 contiguous bytes per row per instruction --
// the second layout of a tensor comes from L1 / L2), the computed ones come out of the products
// in the layout needed, and only dx, consumed by both kinds of product, goes through a per-wave
// LDS transpose (16 x 64).  LDS holds the weight slabs and that transpose tile (~49 KB per
// 4-wave workgroup, the old kernels staged every tile: ~150 KB per 8-wave workgroup), and no MFMA
// operand of a row tile is read from LDS.
#ifndef GASFM_PT_BWD_R
#define GASFM_PT_BWD_R 1
#endif
// 1: scheduling barriers between the phases of a tile (each phase's MFMAs and VALU work stay
// together); 0: none (the compiler may interleave a phase's VALU with the next phase's MFMAs)
#ifndef GASFM_PT_SCHED
#define GASFM_PT_SCHED 1
#endif
#if GASFM_PT_SCHED
#define PT_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define PT_SCHED_BARRIER() ((void)0)
#endif
// 1 wave per SIMD (~210 VGPRs + 116 AGPRs) with the next tile's rows requested one tile ahead;
// 2 waves per SIMD spills (256 VGPRs, 52 spilled): 110 vs 86 us at n = 200k without the prefetch
#ifndef GASFM_PT_BWD_R_MINW
#define GASFM_PT_BWD_R_MINW 1
#endif
constexpr int kWavesR = 4, kThreadsR = kWavesR * kW;
constexpr int LDX = FP + 4;  // transpose tile row stride: the C-layout writes of the 4 lane groups hit 4 bank quarters

// float4 slabs of W^T for W [O x K] (out index k, K index o): Q[((k/16) (O/16) + o/16) 64 + 16 ((o%16)/4)
// + k%16][o%4] = W[o][k], i.e. stage_slabs of the transpose (W is read in its own row-major order)
template <int O, int K, int NT>
__device__ __forceinline__ void stage_slabs_tr(const float* __restrict__ W, float* Q) {
  Stage<O * K, NT> s;
  s.load([&](int q) { return W[q]; });
  s.store([&](int q, float v) {
    const int o = q / K, k = q % K;
    Q[(((k / 16) * (O / 16) + o / 16) * 64 + ((o % 16) / 4) * 16 + k % 16) * 4 + o % 4] = v;
  });
}

// acc[ot] += X W^T with X (T-layout k-slabs) as the A operand: acc[ot][r] = Y[row 4 g + r][16 ot + c]
template <int OT, int KU>
__device__ __forceinline__ void layer_c(const float4* __restrict__ Q, const f32x4 (&xk)[KU], f32x4 (&acc)[OT],
                                        int lane) {
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    float4 w[OT];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) w[ot] = Q[(ot * KU + u) * 64 + lane];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(xk[u][0], w[ot].x, acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(xk[u][1], w[ot].y, acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(xk[u][2], w[ot].z, acc[ot]);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) acc[ot] = mfma16(xk[u][3], w[ot].w, acc[ot]);
  }
}

// C-layout rows: v[ft][r] = X[row0 + 4 g + r][16 ft + c]; rows >= nrows read a valid row (cl_mask zeroes
// them where the values are consumed: a select right after the load would wait for it, so a load
// issued a tile ahead must not be masked in place)
template <int W>
__device__ __forceinline__ void cl_load(const float* __restrict__ X, int64_t row0, int nrows, f32x4 (&v)[W / 16],
                                        int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = 4 * g + r;
    const float* p = X + (row0 + (rr < nrows ? rr : 0)) * W + c;
#pragma unroll
    for (int ft = 0; ft < W / 16; ++ft) v[ft][r] = p[16 * ft];
  }
}
template <int NF>
__device__ __forceinline__ void cl_mask(f32x4 (&v)[NF], int nrows, int g) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int ft = 0; ft < NF; ++ft) v[ft][r] = 4 * g + r < nrows ? v[ft][r] : 0.f;
}

// C layout -> T layout of a 16 x 64 tile through the wave's LDS tile X (stride LDX)
__device__ __forceinline__ void c_to_t64(const f32x4 (&v)[4], float* X, f32x4 (&o)[4], int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ft = 0; ft < 4; ++ft)
#pragma unroll
    for (int r = 0; r < 4; ++r) X[(4 * g + r) * LDX + 16 * ft + c] = v[ft][r];
  // one wave's LDS instructions execute in order: a compiler barrier suffices (a wavefront fence
  // would also wait for the global loads in flight)
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 t = *reinterpret_cast<const float4*>(X + c * LDX + 16 * u + 4 * g);
    o[u] = f32x4{t.x, t.y, t.z, t.w};
  }
}

// LayerNorm statistics of the C-layout rows 4 g + r (64 features: 4 regs x 16 lanes)
__device__ __forceinline__ void cl_stats(const f32x4 (&x)[4], float eps, float (&mean)[4], float (&rstd)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    mean[r] = sum16((x[0][r] + x[1][r]) + (x[2][r] + x[3][r])) * (1.f / FP);
    float q = 0.f;
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) q = fmaf(x[ot][r] - mean[r], x[ot][r] - mean[r], q);
    rstd[r] = rsq_normal(sum16(q) * (1.f / FP) + eps);
  }
}

// LayerNorm + ReLU backward of the C-layout rows (xh: normalised x, dh: gradient of relu(xh g + b));
// rows >= nrows give 0.  Accumulates dgamma / dbeta per lane feature 16 ot + c.  Packed fp32 math
// (round 5): features (16 ot + c, 16 (ot + 1) + c) of a row as one pair per v_pk_* instruction.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void cl_ln_relu_bwd(const f32x4 (&xh)[4], const f32x4 (&dh)[4], const float (&gm)[4],
                                               const float (&bt)[4], const float (&rstd)[4], int nrows, int g,
                                               float (&dg)[4], float (&db)[4], f32x4 (&dx)[4]) {
  f32x2 dg2[2] = {{dg[0], dg[1]}, {dg[2], dg[3]}}, db2[2] = {{db[0], db[1]}, {db[2], db[3]}};
  const f32x2 gm2[2] = {{gm[0], gm[1]}, {gm[2], gm[3]}}, bt2[2] = {{bt[0], bt[1]}, {bt[2], bt[3]}};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool live = 4 * g + r < nrows;
    f32x2 s1p = {0.f, 0.f}, s2p = {0.f, 0.f}, gv[2], x2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      x2[h] = f32x2{xh[2 * h][r], xh[2 * h + 1][r]};
      const f32x2 pre = __builtin_elementwise_fma(x2[h], gm2[h], bt2[h]);
      const f32x2 dy = {(live && pre.x > 0.f) ? dh[2 * h][r] : 0.f, (live && pre.y > 0.f) ? dh[2 * h + 1][r] : 0.f};
      dg2[h] = __builtin_elementwise_fma(dy, x2[h], dg2[h]);
      db2[h] += dy;
      gv[h] = dy * gm2[h];
      s1p += gv[h];
      s2p = __builtin_elementwise_fma(gv[h], x2[h], s2p);
    }
    const float s1 = sum16(s1p.x + s1p.y) * (1.f / FP);
    const float s2 = sum16(s2p.x + s2p.y) * (1.f / FP);
    const f32x2 s1v = {s1, s1}, ms2 = {-s2, -s2}, r2 = {rstd[r], rstd[r]};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2 t = __builtin_elementwise_fma(x2[h], ms2, gv[h] - s1v) * r2;  // rstd ((gv - s1) - xh s2)
      dx[2 * h][r] = t.x;
      dx[2 * h + 1][r] = t.y;
    }
  }
  dg[0] = dg2[0].x, dg[1] = dg2[0].y, dg[2] = dg2[1].x, dg[3] = dg2[1].y;
  db[0] = db2[0].x, db[1] = db2[0].y, db[2] = db2[1].x, db[3] = db2[1].y;
}

// dx = dout + LN_bwd(mask * (dout W_m)) (== d prev), dagg = dx W_p; partial row per workgroup in the
// TAIL_PART layout of point_tail_bwd_kernel.  Per tile: x = agg W_p^T (+ b_p + prev) in C layout
// (agg T-layout as A), h = relu(LN x); dh = dout W_m in C layout (dout T-layout as A); dx (C);
// dW_m += dout^T h and dW_p += dx^T agg from C-layout registers; dx -> T layout (LDS), stored;
// dagg = dx W_p in T layout (dx as B), stored.
template <bool PREV>
__global__ __launch_bounds__(kThreadsR, GASFM_PT_BWD_R_MINW) void point_tail_bwd_r_kernel(
    const float* __restrict__ dout, const float* __restrict__ prev, const float* __restrict__ agg, int64_t N,
    const float* __restrict__ Wp, const float* __restrict__ bp, const float* __restrict__ gam,
    const float* __restrict__ bet, float eps, const float* __restrict__ Wm, float* __restrict__ dx,
    float* __restrict__ dagg, float* __restrict__ part) {
  constexpr int NRED = 64 + 32 + 16;
  constexpr int OQ = 0, OQT = FP * FA, OMT = 2 * FP * FA, OX = OMT + FP * FP, NLDS = OX + kWavesR * TR * LDX;
  __shared__ __attribute__((aligned(16))) float lds[NLDS];
  float4* WpQ = reinterpret_cast<float4*>(lds + OQ);    // slabs of W_p   (out o, k j)
  float4* WpTQ = reinterpret_cast<float4*>(lds + OQT);  // slabs of W_p^T (out j, k o)
  float4* WmTQ = reinterpret_cast<float4*>(lds + OMT);  // slabs of W_m^T (out i, k o)
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  stage_slabs<FP, FA, kThreadsR>(Wp, lds + OQ);
  stage_slabs_tr<FP, FA, kThreadsR>(Wp, lds + OQT);
  stage_slabs_tr<FP, FP, kThreadsR>(Wm, lds + OMT);
  float bpC[4], gmC[4], btC[4];
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) {
    bpC[ot] = bp[16 * ot + c];
    gmC[ot] = gam[16 * ot + c];
    btC[ot] = bet[16 * ot + c];
  }
  __syncthreads();
  float* X = lds + OX + wave * TR * LDX;
  f32x4 dWm[4][4], dWp[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dWm[mt][nt] = zero4();
    dWp[mt][0] = dWp[mt][1] = zero4();
  }
  float dbm[4] = {0.f, 0.f, 0.f, 0.f}, dbp[4] = {0.f, 0.f, 0.f, 0.f};
  float dg[4] = {0.f, 0.f, 0.f, 0.f}, dbt[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWavesR + wave, nw = int64_t(gridDim.x) * kWavesR;
  // every row of tile t + nw is requested before tile t's work (one tile of loads in flight)
  f32x4 n_agT[2], n_dT[4], n_pC[4], n_dC[4], n_agC[2];
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    slabs_load<FA>(agg, r0, nr, n_agT, lane);
    if (PREV) cl_load<FP>(prev, r0, nr, n_pC, lane);
    slabs_load<FP>(dout, r0, nr, n_dT, lane);
    cl_load<FP>(dout, r0, nr, n_dC, lane);
    cl_load<FA>(agg, r0, nr, n_agC, lane);
  };
  if (gw < ntiles) fetch(gw);
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    asm volatile("" ::: "memory");  // weight slabs re-read from LDS per tile (not hoisted into VGPRs)
    f32x4 agT[2] = {n_agT[0], n_agT[1]}, dT[4], x[4], dC[4], agC[2] = {n_agC[0], n_agC[1]};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      dT[u] = n_dT[u];
      dC[u] = n_dC[u];
      x[u] = PREV ? n_pC[u] : zero4();
    }
    // unconditional (the last tile re-reads itself): a load under a branch makes the loop header
    // wait for every outstanding load
    fetch(t + nw < ntiles ? t + nw : t);
    cl_mask(dC, nrows, g);
    cl_mask(agC, nrows, g);
    if (PREV) cl_mask(x, nrows, g);
    // phase 1: x (C layout) and its LayerNorm
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) x[ot] += bpC[ot];
    layer_c<4, 2>(WpQ, agT, x, lane);
    float mean[4], rstd[4];
    cl_stats(x, eps, mean, rstd);
#pragma unroll
    for (int ot = 0; ot < 4; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) x[ot][r] = (x[ot][r] - mean[r]) * rstd[r];  // x_hat from here on
    PT_SCHED_BARRIER();
    // phase 2: dh = dout W_m (C layout)
    f32x4 dh[4] = {zero4(), zero4(), zero4(), zero4()};
    layer_c<4, 4>(WmTQ, dT, dh, lane);
    PT_SCHED_BARRIER();
    // phase 3: LayerNorm backward -> dx (C layout), bias sums
    f32x4 dxc[4];
    cl_ln_relu_bwd(x, dh, gmC, btC, rstd, nrows, g, dg, dbt, dxc);
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) {
      dxc[ot] += dC[ot];  // rows >= nrows: 0 + 0
      dbm[ot] += (dC[ot][0] + dC[ot][1]) + (dC[ot][2] + dC[ot][3]);
      dbp[ot] += (dxc[ot][0] + dxc[ot][1]) + (dxc[ot][2] + dxc[ot][3]);
    }
    PT_SCHED_BARRIER();
    // phase 4: weight gradients over the tile's rows (step s: row 4 g + s; rows past nrows: dout,
    // dx are 0); h = relu(x_hat g + b) recomputed here (not live through phases 2-3)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float hs[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) hs[nt] = fmaxf(fmaf(x[nt][s], gmC[nt], btC[nt]), 0.f);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dWm[mt][nt] = mfma16(dC[mt][s], hs[nt], dWm[mt][nt]);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) dWp[mt][nt] = mfma16(dxc[mt][s], agC[nt][s], dWp[mt][nt]);
      }
    }
    PT_SCHED_BARRIER();
    f32x4 dxT[4];
    c_to_t64(dxc, X, dxT, lane);
    slabs_store<FP>(dx, row0, nrows, dxT, lane);
    f32x4 da[2] = {zero4(), zero4()};
    layer_t<2, 4>(WpTQ, dxT, da, lane);
    slabs_store<FA>(dagg, row0, nrows, da, lane);
    __builtin_amdgcn_wave_barrier();  // this tile's transpose reads before the next tile's writes
    asm volatile("" ::: "memory");
  }
  float v[NRED];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) v[(mt * 4 + nt) * 4 + r] = dWm[mt][nt][r];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) v[64 + (mt * 2 + nt) * 4 + r] = dWp[mt][nt][r];
    }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[96 + k] = dbm[k];
    v[100 + k] = dbp[k];
    v[104 + k] = dg[k];
    v[108 + k] = dbt[k];
  }
  wg_reduce_ordered<NRED, kWavesR, NLDS>(v, lds, wave, lane);
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * TAIL_PART;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = mt * 16 + 4 * g + r;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) out[o * FP + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) out[FP * FP + o * FA + nt * 16 + c] = v[64 + (mt * 2 + nt) * 4 + r];
      }
    float tt[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) tt[k] = sum_groups(v[96 + k]);
    if (g == 0) {
      float* o = out + FP * FP + FP * FA;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) o[q * FP + k * 16 + c] = tt[q * 4 + k];
    }
  }
}

// The whole hub backward (the C and AB passes above) in ONE register-resident pass.  Per tile:
//   t   = W_C relu(LN_C p) + b_C                     C layout (relu(LN_C p) T-layout as A)
//   dt  = dXR W_D                                    C layout (weight / bias gradients) and T layout
//                                                    (the A operand of dt W_C), both from dXR (T)
//   dp  = dXL W_B + (LN_A_bwd(mask (dSA W_A)) + (LN_C_bwd(mask (dt W_C)) + dRes))   C layout
//   dW_C += dt^T relu(LN_C p), dW_D += dXR^T t, dW_A += dSA^T relu(LN_A p), dW_B += dXL^T p
// The rows are requested one tile ahead in the T layout (the products over features); the
// C layout the weight gradients and the LayerNorm backward need is read back from a per-wave
// LDS copy of the tile (one write per row chunk, read just before use: the 256 architected VGPRs
// of a wave could not also hold a second, C-layout load of every tile).  The LayerNorm statistics
// come from the T rows and reach the C layout by lane shuffles.  dRes is read in the C layout at
// the top of its tile (before the next tile's requests), dp stored from the C layout.  Both
// passes' partial rows are written (HA_* into part_a, HC_* into part_c), so the colsums and the
// Python side are those of the two-pass form.  Algorithmic bytes per row:
// p 256 + dSA 128 + dXL 256 + dXR 128 + dRes 256 + dp 256 = 1,280 (the two passes: 2,048).
#ifndef GASFM_PT_HUB_BWD_R
#define GASFM_PT_HUB_BWD_R 1
#endif
#ifndef GASFM_PT_HUB_BWD_R_MINW
#define GASFM_PT_HUB_BWD_R_MINW 1
#endif
constexpr int LDA = FA + 4;  // 32-wide LDS tile row stride (4 lane groups -> 4 bank quarters)

// C-layout rows out (rows >= nrows not written)
template <int W>
__device__ __forceinline__ void cl_store(float* X, int64_t row0, int nrows, const f32x4 (&v)[W / 16], int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (4 * g + r >= nrows) continue;
    float* p = X + (row0 + 4 * g + r) * W + c;
#pragma unroll
    for (int ft = 0; ft < W / 16; ++ft) p[16 * ft] = v[ft][r];
  }
}

// T-layout rows (row c, features 16 u + 4 g + j) into the wave's LDS tile (row stride LD)
template <int W, int LD>
__device__ __forceinline__ void t_to_lds(const f32x4 (&v)[W / 16], float* X, int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int u = 0; u < W / 16; ++u)
    *reinterpret_cast<float4*>(X + c * LD + 16 * u + 4 * g) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
}

template <bool HR>
__global__ __launch_bounds__(kThreadsR, GASFM_PT_HUB_BWD_R_MINW) void point_hub_bwd_r_kernel(
    const float* __restrict__ X, int64_t N, float eps, const float* __restrict__ gA, const float* __restrict__ bA,
    const float* __restrict__ WA, const float* __restrict__ WB, const float* __restrict__ gC,
    const float* __restrict__ bC, const float* __restrict__ WC, const float* __restrict__ bWC,
    const float* __restrict__ WD, const float* __restrict__ dSA, const float* __restrict__ dXL,
    const float* __restrict__ dXR, const float* dRes, float* dX, float* __restrict__ part_a,
    float* __restrict__ part_c) {
  constexpr int OC = 0, ODT = OC + FA * FP, OCT = ODT + FA * FA, OAT = OCT + FA * FP, OBT = OAT + FA * FP,
                OV = OBT + FP * FP, OT = OV + 6 * FP;
  constexpr int TW = TR * (2 * LDX + 3 * LDA);  // per wave: p, dXL (64 wide), dSA, dXR, dt (32 wide)
  constexpr int NLDS = OT + kWavesR * TW;
  constexpr int NRED = 144 + 24;
  __shared__ __attribute__((aligned(16))) float lds[NLDS];
  const float4* WCQ = reinterpret_cast<const float4*>(lds + OC);     // slabs of W_C   (out t,  k p)
  const float4* WDTQ = reinterpret_cast<const float4*>(lds + ODT);   // slabs of W_D^T (out t,  k xr)
  const float4* WCTQ = reinterpret_cast<const float4*>(lds + OCT);   // slabs of W_C^T (out p,  k t)
  const float4* WATQ = reinterpret_cast<const float4*>(lds + OAT);   // slabs of W_A^T (out p,  k sa)
  const float4* WBTQ = reinterpret_cast<const float4*>(lds + OBT);   // slabs of W_B^T (out p,  k xl)
  const float* V = lds + OV;  // gamma_C beta_C gamma_A beta_A b_C(32) (pad)
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Tp = lds + OT + wave * TW;
  float* Tl = Tp + TR * LDX;
  float* Ts = Tl + TR * LDX;
  float* Tr = Ts + TR * LDA;
  float* Td = Tr + TR * LDA;  // dt's C -> T transpose
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWavesR + wave, nw = int64_t(gridDim.x) * kWavesR;
  f32x4 n_pT[4], n_rT[2], n_sT[2], n_lT[4];  // the next tile's T-layout rows
  auto fetch = [&](int64_t tt) {
    const int64_t r0 = tt * TR;
    const int nr = int(N - r0 < TR ? N - r0 : TR);
    slabs_load<FP>(X, r0, nr, n_pT, lane);
    slabs_load<FA>(dXR, r0, nr, n_rT, lane);
    slabs_load<FA>(dSA, r0, nr, n_sT, lane);
    slabs_load<FP>(dXL, r0, nr, n_lT, lane);
  };
  if (gw < ntiles) fetch(gw);  // the first tile's rows fly while the weights are staged
  stage_slabs<FA, FP, kThreadsR>(WC, lds + OC);
  stage_slabs_tr<FA, FA, kThreadsR>(WD, lds + ODT);
  stage_slabs_tr<FA, FP, kThreadsR>(WC, lds + OCT);
  stage_slabs_tr<FA, FP, kThreadsR>(WA, lds + OAT);
  stage_slabs_tr<FP, FP, kThreadsR>(WB, lds + OBT);
  if (threadIdx.x < FP) {
    lds[OV + threadIdx.x] = gC[threadIdx.x];
    lds[OV + FP + threadIdx.x] = bC[threadIdx.x];
    lds[OV + 2 * FP + threadIdx.x] = gA[threadIdx.x];
    lds[OV + 3 * FP + threadIdx.x] = bA[threadIdx.x];
    if (threadIdx.x < FA) lds[OV + 4 * FP + threadIdx.x] = bWC[threadIdx.x];
  }
  __syncthreads();
  f32x4 dWA[2][4], dWB[4][4], dWC[2][4], dWD[2][2];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    dWA[0][nt] = dWA[1][nt] = dWC[0][nt] = dWC[1][nt] = zero4();
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) dWB[mt][nt] = zero4();
  }
  dWD[0][0] = dWD[0][1] = dWD[1][0] = dWD[1][1] = zero4();
  float dbB[4] = {0.f, 0.f, 0.f, 0.f}, dgA[4] = {0.f, 0.f, 0.f, 0.f}, dbA[4] = {0.f, 0.f, 0.f, 0.f};
  float dgC[4] = {0.f, 0.f, 0.f, 0.f}, dbCl[4] = {0.f, 0.f, 0.f, 0.f}, dbC[2] = {0.f, 0.f}, dbD[2] = {0.f, 0.f};
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    asm volatile("" ::: "memory");  // weight slabs re-read from LDS per tile (not hoisted into VGPRs)
    f32x4 pT[4], rT[2] = {n_rT[0], n_rT[1]}, sT[2] = {n_sT[0], n_sT[1]}, lT[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      pT[u] = n_pT[u];
      lT[u] = n_lT[u];
    }
    // dRes of this tile, then the next tile's rows (unconditional: the last tile re-reads itself;
    // a load under a branch makes the loop header wait for every outstanding load)
    f32x4 acc[4];
    if (HR) cl_load<FP>(dRes, row0, nrows, acc, lane);
    fetch(t + nw < ntiles ? t + nw : t);
    t_to_lds<FP, LDX>(pT, Tp, lane);
    t_to_lds<FP, LDX>(lT, Tl, lane);
    t_to_lds<FA, LDA>(sT, Ts, lane);
    t_to_lds<FA, LDA>(rT, Tr, lane);
    // phase 1: statistics of the row c (T layout), t = W_C relu(LN_C p) + b_C (C layout)
    float mean, rstd;
    slab_stats(pT, eps, mean, rstd);
    f32x4 tC[2] = {zero4(), zero4()};
    {
      f32x4 pc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 gm = vec_at(V, u, g), bt = vec_at(V + FP, u, g);
#pragma unroll
        for (int j = 0; j < 4; ++j) pc[u][j] = fmaxf(fmaf((pT[u][j] - mean) * rstd, gm[j], bt[j]), 0.f);
      }
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) tC[ft] += V[4 * FP + 16 * ft + c];
      layer_c<2, 4>(WCQ, pc, tC, lane);
    }
    // row 4 g + r's statistics, computed on lane c = 4 g + r: through the padding columns 64, 65 of
    // the wave's p tile (row c; every lane group writes the same values), not 8 lane shuffles
    *reinterpret_cast<float2*>(Tp + c * LDX + FP) = make_float2(mean, rstd);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    float meanC[4], rstdC[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float2 st = *reinterpret_cast<const float2*>(Tp + (4 * g + r) * LDX + FP);
      meanC[r] = st.x;
      rstdC[r] = st.y;
    }
    PT_SCHED_BARRIER();
    // phase 2: dt (C and T layouts), dt W_C, LN_C backward onto dRes
    f32x4 dtC[2] = {zero4(), zero4()};
    f32x4 xh[4];
#pragma unroll
    for (int ot = 0; ot < 4; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) xh[ot][r] = (Tp[(4 * g + r) * LDX + 16 * ot + c] - meanC[r]) * rstdC[r];
    {
      f32x4 dtT[2] = {zero4(), zero4()}, dp[4] = {zero4(), zero4(), zero4(), zero4()}, dq[4];
      layer_c<2, 2>(WDTQ, rT, dtC, lane);
      // dt's T layout through the wave's LDS tile, not a second product (16 MFMA): the same
      // products summed in the same k order, so bitwise the layer_t result (round 5)
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) Td[(4 * g + r) * LDA + 16 * ft + c] = dtC[ft][r];
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 t4 = *reinterpret_cast<const float4*>(Td + c * LDA + 16 * u + 4 * g);
        dtT[u] = f32x4{t4.x, t4.y, t4.z, t4.w};
      }
      PT_SCHED_BARRIER();
      layer_c<4, 2>(WCTQ, dtT, dp, lane);
      float gm[4], bt[4];
#pragma unroll
      for (int ot = 0; ot < 4; ++ot) {
        gm[ot] = V[16 * ot + c];
        bt[ot] = V[FP + 16 * ot + c];
      }
      cl_ln_relu_bwd(xh, dp, gm, bt, rstdC, nrows, g, dgC, dbCl, dq);
#pragma unroll
      for (int ot = 0; ot < 4; ++ot) acc[ot] = HR ? dq[ot] + acc[ot] : dq[ot];
    }
    PT_SCHED_BARRIER();
    // phase 3: dSA W_A, LN_A backward; dXL W_B accumulated on top; dp stored
    {
      f32x4 dp[4] = {zero4(), zero4(), zero4(), zero4()}, da[4];
      layer_c<4, 2>(WATQ, sT, dp, lane);
      float gm[4], bt[4];
#pragma unroll
      for (int ot = 0; ot < 4; ++ot) {
        gm[ot] = V[2 * FP + 16 * ot + c];
        bt[ot] = V[3 * FP + 16 * ot + c];
      }
      cl_ln_relu_bwd(xh, dp, gm, bt, rstdC, nrows, g, dgA, dbA, da);
#pragma unroll
      for (int ot = 0; ot < 4; ++ot) acc[ot] = da[ot] + acc[ot];
    }
    PT_SCHED_BARRIER();
    layer_c<4, 4>(WBTQ, lT, acc, lane);
    cl_store<FP>(dX, row0, nrows, acc, lane);
    PT_SCHED_BARRIER();
    // phase 4: weight gradients over the tile's rows (step s: row 4 g + s, C-layout operands read
    // from the LDS copies; dead rows: the A operands are masked to 0), bias sums
    cl_mask(dtC, nrows, g);
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) dbC[ft] += (dtC[ft][0] + dtC[ft][1]) + (dtC[ft][2] + dtC[ft][3]);
    float gAv[4], bAv[4], gCv[4], bCv[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      gCv[nt] = V[16 * nt + c];
      bCv[nt] = V[FP + 16 * nt + c];
      gAv[nt] = V[2 * FP + 16 * nt + c];
      bAv[nt] = V[3 * FP + 16 * nt + c];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row = 4 * g + s;
      const bool live = row < nrows;
      float pa[4], pc[4], pr[4], la[4], sa[2], ra[2];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        pa[nt] = fmaxf(fmaf(xh[nt][s], gAv[nt], bAv[nt]), 0.f);
        pc[nt] = fmaxf(fmaf(xh[nt][s], gCv[nt], bCv[nt]), 0.f);
        pr[nt] = Tp[row * LDX + 16 * nt + c];
        la[nt] = live ? Tl[row * LDX + 16 * nt + c] : 0.f;
        dbB[nt] += la[nt];
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        sa[mt] = live ? Ts[row * LDA + 16 * mt + c] : 0.f;
        ra[mt] = live ? Tr[row * LDA + 16 * mt + c] : 0.f;
        dbD[mt] += ra[mt];
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          dWA[mt][nt] = mfma16(sa[mt], pa[nt], dWA[mt][nt]);
          dWC[mt][nt] = mfma16(dtC[mt][s], pc[nt], dWC[mt][nt]);
        }
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) dWD[mt][nt] = mfma16(ra[mt], tC[nt][s], dWD[mt][nt]);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) dWB[mt][nt] = mfma16(la[mt], pr[nt], dWB[mt][nt]);
    }
    __builtin_amdgcn_wave_barrier();  // this tile's LDS reads before the next tile's writes
    asm volatile("" ::: "memory");
  }
  float v[NRED];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        v[(mt * 4 + nt) * 4 + r] = dWA[mt][nt][r];
        v[96 + (mt * 4 + nt) * 4 + r] = dWC[mt][nt][r];
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) v[32 + (mt * 4 + nt) * 4 + r] = dWB[mt][nt][r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) v[128 + (mt * 2 + nt) * 4 + r] = dWD[mt][nt][r];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[144 + k] = dbB[k];
    v[148 + k] = dgA[k];
    v[152 + k] = dbA[k];
    v[156 + k] = dgC[k];
    v[160 + k] = dbCl[k];
  }
  v[164] = dbC[0];
  v[165] = dbC[1];
  v[166] = dbD[0];
  v[167] = dbD[1];
  wg_reduce_ordered<NRED, kWavesR, NLDS>(v, lds, wave, lane);
  if (wave == 0) {
    float* oa = part_a + int64_t(blockIdx.x) * HA_PART;
    float* oc = part_c + int64_t(blockIdx.x) * HC_PART;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int o = mt * 16 + 4 * g + r;
          oa[HA_WA + o * FP + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
          oc[HC_WC + o * FP + nt * 16 + c] = v[96 + (mt * 4 + nt) * 4 + r];
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) oa[HA_WB + (mt * 16 + 4 * g + r) * FP + nt * 16 + c] = v[32 + (mt * 4 + nt) * 4 + r];
      }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) oc[HC_WD + (mt * 16 + 4 * g + r) * FA + nt * 16 + c] = v[128 + (mt * 2 + nt) * 4 + r];
    float tt[24];
#pragma unroll
    for (int k = 0; k < 24; ++k) tt[k] = sum_groups(v[144 + k]);
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        oa[HA_BB + k * 16 + c] = tt[k];
        oa[HA_GA + k * 16 + c] = tt[4 + k];
        oa[HA_BA + k * 16 + c] = tt[8 + k];
        oc[HC_GC + k * 16 + c] = tt[12 + k];
        oc[HC_BCL + k * 16 + c] = tt[16 + k];
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        oc[HC_BC + k * 16 + c] = tt[20 + k];
        oc[HC_BD + k * 16 + c] = tt[22 + k];
      }
    }
  }
}

int64_t tiles_of(int64_t N) { return (N + TR - 1) / TR; }

template <class K>
int grid4(K kernel, int64_t N) {
  return resident_grid(reinterpret_cast<const void*>(kernel), kThreads, 0, tiles_of(N), kWaves);
}
template <class K>
int gridT(K kernel, int64_t N) {
  return resident_grid(reinterpret_cast<const void*>(kernel), kThreadsT, 0, tiles_of(N), kWavesT);
}
template <class K>
int grid8(K kernel, int64_t N) {
  return resident_grid(reinterpret_cast<const void*>(kernel), kThreads8, 0, tiles_of(N), kWaves8);
}

template <class K>
int gridR(K kernel, int64_t N) {
  return resident_grid(reinterpret_cast<const void*>(kernel), kThreadsR, 0, tiles_of(N), kWavesR);
}
int tail_bwd_grid(int64_t N, bool has_prev) {
  if (GASFM_PT_BWD_R)
    return has_prev ? gridR(&point_tail_bwd_r_kernel<true>, N) : gridR(&point_tail_bwd_r_kernel<false>, N);
  return has_prev ? grid8(&point_tail_bwd_kernel<true>, N) : grid8(&point_tail_bwd_kernel<false>, N);
}
int hub_ab_grid(int64_t N, bool hr) {
  return hr ? grid8(&point_hub_bwd_ab_kernel<true>, N) : grid8(&point_hub_bwd_ab_kernel<false>, N);
}
int hub_c_grid(int64_t N, bool hr) {
  return hr ? grid8(&point_hub_bwd_c_kernel<true>, N) : grid8(&point_hub_bwd_c_kernel<false>, N);
}
// the one-pass hub backward: both partial buffers have its grid's rows (whether dRes is given or not),
// and the two-pass entry points launch that many workgroups too while it is the default (their
// partial buffers come from gasfm_point_hub_part_shape)
int hub_r_grid(int64_t N) { return gridR(&point_hub_bwd_r_kernel<true>, N); }

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int32_t gasfm_point_tail_part_shape(int64_t N, int32_t has_prev, int32_t* cols) {
  if (cols) *cols = TAIL_PART;
  return N > 0 ? tail_bwd_grid(N, has_prev != 0) : 0;
}

extern "C" int32_t gasfm_point_hub_part_shape(int64_t N, int32_t which, int32_t has_res, int32_t* cols) {
  if (cols) *cols = which ? HC_PART : HA_PART;
  if (N <= 0) return 0;
  if (GASFM_PT_HUB_BWD_R) return hub_r_grid(N);
  return which ? hub_c_grid(N, has_res != 0) : hub_ab_grid(N, has_res != 0);
}
extern "C" int gasfm_point_tail_fwd(const float* prev, const float* agg, int64_t N, const float* Wp, const float* bp,
                                    const float* ln_w, const float* ln_b, float eps, const float* Wm,
                                    const float* bm, float* out, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_tail_fwd: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(agg && Wp && bp && ln_w && ln_b && Wm && bm && out, "gasfm_point_tail_fwd: null pointer");
  GASFM_REQUIRE(aligned16(agg) && (!prev || aligned16(prev)), "gasfm_point_tail_fwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (GASFM_PT_FWD_T) {
    if (prev)
      hipLaunchKernelGGL(point_tail_fwd_t_kernel<true>, dim3(gridT(&point_tail_fwd_t_kernel<true>, N)),
                         dim3(kThreadsT), 0, st, prev, agg, N, Wp, bp, ln_w, ln_b, eps, Wm, bm, out);
    else
      hipLaunchKernelGGL(point_tail_fwd_t_kernel<false>, dim3(gridT(&point_tail_fwd_t_kernel<false>, N)),
                         dim3(kThreadsT), 0, st, prev, agg, N, Wp, bp, ln_w, ln_b, eps, Wm, bm, out);
    return launch_status("gasfm_point_tail_fwd");
  }
  if (prev)
    hipLaunchKernelGGL(point_tail_fwd_kernel<true>, dim3(grid4(&point_tail_fwd_kernel<true>, N)), dim3(kThreads), 0,
                       st, prev, agg, N, Wp, bp, ln_w, ln_b, eps, Wm, bm, out);
  else
    hipLaunchKernelGGL(point_tail_fwd_kernel<false>, dim3(grid4(&point_tail_fwd_kernel<false>, N)), dim3(kThreads),
                       0, st, prev, agg, N, Wp, bp, ln_w, ln_b, eps, Wm, bm, out);
  return launch_status("gasfm_point_tail_fwd");
}

extern "C" int gasfm_point_tail_bwd(const float* dout, const float* prev, const float* agg, int64_t N,
                                    const float* Wp, const float* bp, const float* ln_w, const float* ln_b,
                                    float eps, const float* Wm, float* dx, float* dagg, float* part, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_tail_bwd: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(dout && agg && Wp && bp && ln_w && ln_b && Wm && dx && dagg && part,
                "gasfm_point_tail_bwd: null pointer");
  GASFM_REQUIRE(aligned16(dout) && aligned16(agg), "gasfm_point_tail_bwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int gsz = tail_bwd_grid(N, prev != nullptr);
  if (GASFM_PT_BWD_R) {
    if (prev)
      hipLaunchKernelGGL(point_tail_bwd_r_kernel<true>, dim3(gsz), dim3(kThreadsR), 0, st, dout, prev, agg, N, Wp,
                         bp, ln_w, ln_b, eps, Wm, dx, dagg, part);
    else
      hipLaunchKernelGGL(point_tail_bwd_r_kernel<false>, dim3(gsz), dim3(kThreadsR), 0, st, dout, prev, agg, N, Wp,
                         bp, ln_w, ln_b, eps, Wm, dx, dagg, part);
    return launch_status("gasfm_point_tail_bwd");
  }
  if (prev)
    hipLaunchKernelGGL(point_tail_bwd_kernel<true>, dim3(gsz), dim3(kThreads8), 0, st, dout, prev, agg, N, Wp, bp,
                       ln_w, ln_b, eps, Wm, dx, dagg, part);
  else
    hipLaunchKernelGGL(point_tail_bwd_kernel<false>, dim3(gsz), dim3(kThreads8), 0, st, dout, prev, agg, N, Wp, bp,
                       ln_w, ln_b, eps, Wm, dx, dagg, part);
  return launch_status("gasfm_point_tail_bwd");
}

extern "C" int gasfm_point_hub_fwd(const float* X, int64_t N, float eps, const float* gA, const float* bA,
                                   const float* WA, float* SA, const float* WB, const float* bB, float* XL,
                                   const float* gC, const float* bC, const float* WC, const float* bWC,
                                   const float* WD, const float* bD, float* XR, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_hub_fwd: N < 0");
  const bool hc = gC != nullptr;
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(X && gA && bA && WA && SA && WB && bB && XL, "gasfm_point_hub_fwd: null pointer");
  GASFM_REQUIRE(!hc || (bC && WC && bWC && WD && bD && XR), "gasfm_point_hub_fwd: null pointer (C part)");
  GASFM_REQUIRE(aligned16(X), "gasfm_point_hub_fwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (GASFM_PT_FWD_T) {
    if (hc)
      hipLaunchKernelGGL(point_hub_fwd_t_kernel<true>, dim3(gridT(&point_hub_fwd_t_kernel<true>, N)), dim3(kThreadsT),
                         0, st, X, N, eps, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR);
    else
      hipLaunchKernelGGL(point_hub_fwd_t_kernel<false>, dim3(gridT(&point_hub_fwd_t_kernel<false>, N)),
                         dim3(kThreadsT), 0, st, X, N, eps, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR);
    return launch_status("gasfm_point_hub_fwd");
  }
  if (hc)
    hipLaunchKernelGGL(point_hub_fwd_kernel<true>, dim3(grid8(&point_hub_fwd_kernel<true>, N)), dim3(kThreads8), 0,
                       st, X, N, eps, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR);
  else
    hipLaunchKernelGGL(point_hub_fwd_kernel<false>, dim3(grid4(&point_hub_fwd_kernel<false>, N)), dim3(kThreads), 0,
                       st, X, N, eps, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR);
  return launch_status("gasfm_point_hub_fwd");
}

extern "C" int gasfm_point_tail_hub_fwd(const float* prev, const float* agg, int64_t N, const float* Wp,
                                        const float* bp, const float* ln_w, const float* ln_b, float eps,
                                        const float* Wm, const float* bm, float* out, float eps_h, const float* gA,
                                        const float* bA, const float* WA, float* SA, const float* WB,
                                        const float* bB, float* XL, const float* gC, const float* bC,
                                        const float* WC, const float* bWC, const float* WD, const float* bD,
                                        float* XR, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_tail_hub_fwd: N < 0");
  const bool hc = gC != nullptr;
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(agg && Wp && bp && ln_w && ln_b && Wm && bm && out && gA && bA && WA && SA && WB && bB && XL,
                "gasfm_point_tail_hub_fwd: null pointer");
  GASFM_REQUIRE(!hc || (bC && WC && bWC && WD && bD && XR), "gasfm_point_tail_hub_fwd: null pointer (C part)");
  GASFM_REQUIRE(aligned16(agg) && (!prev || aligned16(prev)) && aligned16(out) && aligned16(SA) && aligned16(XL) &&
                    (!hc || aligned16(XR)),
                "gasfm_point_tail_hub_fwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // 4-wave workgroups (two per CU by the 64 KB of staged weights: 2 waves per SIMD); 6-wave ones
  // (3 per SIMD at 156 VGPRs) measured 31.5 vs 18.3 us per rank-of-8 launch, 94.9 vs 72.5 at config 4
  // (profiles/r6_ab_tail_hub.txt)
#define GASFM_LAUNCH(PV, HCV)                                                                                  \
  hipLaunchKernelGGL((point_tail_hub_fwd_t_kernel<PV, HCV, 4>),                                                \
                     dim3(resident_grid(reinterpret_cast<const void*>(&point_tail_hub_fwd_t_kernel<PV, HCV, 4>), \
                                        4 * kW, 0, tiles_of(N), 4)),                                           \
                     dim3(4 * kW), 0, st, prev, agg, N, Wp, bp, ln_w, ln_b, eps, Wm, bm, out, eps_h, gA, bA, WA, \
                     SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR)
  if (prev && hc)
    GASFM_LAUNCH(true, true);
  else if (prev)
    GASFM_LAUNCH(true, false);
  else if (hc)
    GASFM_LAUNCH(false, true);
  else
    GASFM_LAUNCH(false, false);
#undef GASFM_LAUNCH
  return launch_status("gasfm_point_tail_hub_fwd");
}

extern "C" int gasfm_point_hub_bwd_c(const float* X, int64_t N, float eps, const float* gC, const float* bC,
                                     const float* WC, const float* bWC, const float* WD, const float* dXR,
                                     const float* dRes, float* dX, float* part, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_hub_bwd_c: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(X && gC && bC && WC && bWC && WD && dXR && dX && part, "gasfm_point_hub_bwd_c: null pointer");
  GASFM_REQUIRE(aligned16(X), "gasfm_point_hub_bwd_c: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool hr = dRes != nullptr;
  if (hr)
    hipLaunchKernelGGL(point_hub_bwd_c_kernel<true>, dim3((GASFM_PT_HUB_BWD_R ? hub_r_grid(N) : hub_c_grid(N, true))), dim3(kThreads8), 0, st, X, N, eps,
                       gC, bC, WC, bWC, WD, dXR, dRes, dX, part);
  else
    hipLaunchKernelGGL(point_hub_bwd_c_kernel<false>, dim3((GASFM_PT_HUB_BWD_R ? hub_r_grid(N) : hub_c_grid(N, false))), dim3(kThreads8), 0, st, X, N,
                       eps, gC, bC, WC, bWC, WD, dXR, dRes, dX, part);
  return launch_status("gasfm_point_hub_bwd_c");
}

extern "C" int gasfm_point_hub_bwd_ab(const float* X, int64_t N, float eps, const float* gA, const float* bA,
                                      const float* WA, const float* WB, const float* dSA, const float* dXL,
                                      const float* dRes, float* dX, float* part, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_hub_bwd_ab: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(X && gA && bA && WA && WB && dSA && dXL && dX && part, "gasfm_point_hub_bwd_ab: null pointer");
  GASFM_REQUIRE(aligned16(X), "gasfm_point_hub_bwd_ab: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool hr = dRes != nullptr;
  if (hr)
    hipLaunchKernelGGL(point_hub_bwd_ab_kernel<true>, dim3((GASFM_PT_HUB_BWD_R ? hub_r_grid(N) : hub_ab_grid(N, true))), dim3(kThreads8), 0, st, X, N,
                       eps, gA, bA, WA, WB, dSA, dXL, dRes, dX, part);
  else
    hipLaunchKernelGGL(point_hub_bwd_ab_kernel<false>, dim3((GASFM_PT_HUB_BWD_R ? hub_r_grid(N) : hub_ab_grid(N, false))), dim3(kThreads8), 0, st, X, N,
                       eps, gA, bA, WA, WB, dSA, dXL, dRes, dX, part);
  return launch_status("gasfm_point_hub_bwd_ab");
}

extern "C" int gasfm_point_hub_bwd(const float* X, int64_t N, float eps, const float* gA, const float* bA,
                                   const float* WA, const float* WB, const float* gC, const float* bC,
                                   const float* WC, const float* bWC, const float* WD, const float* dSA,
                                   const float* dXL, const float* dXR, const float* dRes, float* dX, float* part_a,
                                   float* part_c, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_hub_bwd: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(X && gA && bA && WA && WB && gC && bC && WC && bWC && WD && dSA && dXL && dXR && dX && part_a &&
                    part_c,
                "gasfm_point_hub_bwd: null pointer");
  GASFM_REQUIRE(aligned16(X) && aligned16(dSA) && aligned16(dXL) && aligned16(dXR),
                "gasfm_point_hub_bwd: alignment");
  GASFM_REQUIRE(dX != X && dX != dSA && dX != dXL && dX != dXR, "gasfm_point_hub_bwd: dX aliases an input");
  if (!GASFM_PT_HUB_BWD_R) {  // the two-pass form: C pass into dX, AB pass in place
    const int st = gasfm_point_hub_bwd_c(X, N, eps, gC, bC, WC, bWC, WD, dXR, dRes, dX, part_c, stream);
    if (st != GASFM_OK) return st;
    return gasfm_point_hub_bwd_ab(X, N, eps, gA, bA, WA, WB, dSA, dXL, dX, dX, part_a, stream);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int gsz = hub_r_grid(N);
  if (dRes)
    hipLaunchKernelGGL(point_hub_bwd_r_kernel<true>, dim3(gsz), dim3(kThreadsR), 0, st, X, N, eps, gA, bA, WA, WB,
                       gC, bC, WC, bWC, WD, dSA, dXL, dXR, dRes, dX, part_a, part_c);
  else
    hipLaunchKernelGGL(point_hub_bwd_r_kernel<false>, dim3(gsz), dim3(kThreadsR), 0, st, X, N, eps, gA, bA, WA, WB,
                       gC, bC, WC, bWC, WD, dSA, dXL, dXR, dRes, dX, part_a, part_c);
  return launch_status("gasfm_point_hub_bwd");
}
