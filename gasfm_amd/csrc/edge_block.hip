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
// Layout: every kernel works on 32-edge tiles held by ONE wavefront.  The
// tile is staged row-major in the wave's private LDS slice (row stride 33 /
// 65 floats: conflict-free for both the "row per lane" and the "column per
// lane" reads below), and the GEMM-shaped parts run on the f32 MFMA
// v_mfma_f32_32x32x2_f32 (exact fp32, K split as lane halves h = lane>>5):
//   tile x W     A[i][k] = T[i][2s+h],  B[k][n] = W(...)     -> C: col = lane&31,
//                                                               row = (r&3)+8(r>>2)+4h
//   T1^T x T2    A[m][k] = T1[2s+h][m], B[k][n] = T2[2s+h][n]  (reduction over edges)
// Weight-gradient partials are reduced across the workgroup's waves in LDS
// and written once per workgroup; gasfm_colsum finishes them (deterministic).
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace gasfm {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kW = 64;           // wave
constexpr int kWaves = 4;        // waves per workgroup
constexpr int kThreads = kW * kWaves;
constexpr int F = 32;            // projection feature width (n_feat_proj)
constexpr int NX = 64;           // XL width: 32 (point conv) + 32 (camera conv)
constexpr int LD33 = F + 1;
constexpr int LD65 = NX + 1;
constexpr int kMaxGrid = 1024;   // workgroups (x4 waves) for the grid-stride kernels

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Load a 32 x 32 fp32 tile (rows row0.., stride 32 in global) and, per row,
// LayerNorm + ReLU it.  Writes x_hat (normalised, pre-affine) to Xh and the
// activated relu(x_hat*g + b) to Ph (either may be null), raw values to Raw,
// and rstd per row to Rs.  Rows >= nrows are zero (x_hat = 0).
// Row r of the tile is held by the 8 lanes 8k..8k+7 (k = r%8) in step u = r/8.
template <bool LN>
__device__ __forceinline__ void load_norm_tile(const float* __restrict__ P, int64_t row0, int nrows,
                                               const float* __restrict__ gam, const float* __restrict__ bet,
                                               float eps, float* Xh, float* Ph, float* Raw, float* Rs, int lane) {
  const int c = (lane & 7) * 4;
  float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (LN) {
    g4 = *reinterpret_cast<const float4*>(gam + c);
    b4 = *reinterpret_cast<const float4*>(bet + c);
  }
  float4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (lane >> 3) + 8 * u;
    v[u] = (r < nrows) ? *reinterpret_cast<const float4*>(P + (row0 + r) * F + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (lane >> 3) + 8 * u;
    float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    if (Raw) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Raw[r * LD33 + c + k] = x[k];
    }
    float mean = 0.f, rstd = 1.f;
    if (LN) {
      float s = x[0] + x[1] + x[2] + x[3];
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      mean = s * (1.f / F);
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) q = fmaf(x[k] - mean, x[k] - mean, q);
      q += __shfl_xor(q, 1);
      q += __shfl_xor(q, 2);
      q += __shfl_xor(q, 4);
      rstd = rsqrtf(q * (1.f / F) + eps);
    }
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = LN ? (x[k] - mean) * rstd : x[k];
      if (Xh) Xh[r * LD33 + c + k] = (r < nrows) ? xh : 0.f;
      if (Ph) Ph[r * LD33 + c + k] = (r < nrows) ? (LN ? fmaxf(fmaf(xh, gg[k], bb[k]), 0.f) : xh) : 0.f;
    }
    if (Rs && (lane & 7) == 0) Rs[r] = rstd;
  }
}

// Row-major [32 x W] tile from global (stride ld) into LDS (stride W+1); rows >= nrows zero.
template <int W>
__device__ __forceinline__ void load_tile(const float* __restrict__ X, int64_t ld, int64_t row0, int nrows,
                                          float* T, int lane) {
  constexpr int V = W / 4;            // float4 per row
  constexpr int STEPS = 32 * V / kW;  // float4 per lane
#pragma unroll
  for (int u = 0; u < STEPS; ++u) {
    const int q = lane + kW * u;
    const int r = q / V, c = (q % V) * 4;
    const float4 v = (r < nrows) ? *reinterpret_cast<const float4*>(X + (row0 + r) * ld + c)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    float* d = T + r * (W + 1) + c;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}

// Sum `n` floats per lane across the workgroup's waves (LDS scratch >= kWaves*kW*n),
// wave 0 returns the totals in v.
template <int N>
__device__ __forceinline__ void wg_reduce(float (&v)[N], float* scratch, int wave, int lane) {
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) scratch[(wave * N + k) * kW + lane] = v[k];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      float s = 0.f;
      for (int w = 0; w < kWaves; ++w) s += scratch[(w * N + k) * kW + lane];
      v[k] = s;
    }
  }
}

// =====================================================================================
// edge_prologue_fwd: XL[e] = W relu(LN(P[e])) + b     (W: [64 x 32], XL row stride ldY)
// =====================================================================================
template <bool LN>
__global__ __launch_bounds__(kThreads) void edge_prologue_fwd_kernel(const float* __restrict__ P, int64_t E,
                                                                    const float* __restrict__ gam,
                                                                    const float* __restrict__ bet, float eps,
                                                                    const float* __restrict__ W,
                                                                    const float* __restrict__ b,
                                                                    float* __restrict__ Y, int64_t ldY) {
  __shared__ float lds[kWaves][32 * LD33];
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int i = lane & 31, h = lane >> 5;
  float* T = lds[wave];
  float wB[2][16];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < 16; ++s) wB[nt][s] = W[(nt * 32 + i) * F + 2 * s + h];
  const float bias0 = b[i], bias1 = b[32 + i];
  const int64_t ntiles = (E + 31) / 32;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * 32;
    const int nrows = int(E - row0 < 32 ? E - row0 : 32);
    load_norm_tile<LN>(P, row0, nrows, gam, bet, eps, nullptr, T, nullptr, nullptr, lane);
    wave_sync();
    f32x16 acc0 = zero16(), acc1 = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float a = T[i * LD33 + 2 * s + h];
      acc0 = mfma(a, wB[0][s], acc0);
      acc1 = mfma(a, wB[1][s], acc1);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = crow(r, h);
      if (row < nrows) {
        float* y = Y + (row0 + row) * ldY;
        y[i] = acc0[r] + bias0;
        y[32 + i] = acc1[r] + bias1;
      }
    }
    wave_sync();
  }
}

// =====================================================================================
// edge_epilogue_fwd: P'[e] = P[e] + (Wp [relu(LN(P[e])) | P0[e]] + bp + Sp[pt] + Sv[cam] + Sg) / 4
// Wp: [32 x ldWp] (ldWp = 34 with the init-feature skip, 32 without: P0 == null)
// =====================================================================================
__global__ __launch_bounds__(kThreads) void edge_epilogue_fwd_kernel(
    const float* __restrict__ P, const float* __restrict__ P0, const int32_t* __restrict__ cam,
    const int32_t* __restrict__ pt, int64_t E, const float* __restrict__ gam, const float* __restrict__ bet,
    float eps, const float* __restrict__ Wp, int ldWp, const float* __restrict__ bp, const float* __restrict__ Sp,
    const float* __restrict__ Sv, const float* __restrict__ Sg, float scale, float* __restrict__ Pout) {
  __shared__ float lds[kWaves][2 * 32 * LD33 + 64];
  __shared__ int32_t idx[kWaves][64];
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int i = lane & 31, h = lane >> 5;
  float* Ph = lds[wave];
  float* Raw = Ph + 32 * LD33;
  float* Q0 = Raw + 32 * LD33;
  int32_t* ix = idx[wave];
  float wB[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wB[s] = Wp[i * ldWp + 2 * s + h];
  const float w32 = P0 ? Wp[i * ldWp + 32] : 0.f, w33 = P0 ? Wp[i * ldWp + 33] : 0.f;
  const float cst = bp[i] + Sg[i];
  const int64_t ntiles = (E + 31) / 32;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * 32;
    const int nrows = int(E - row0 < 32 ? E - row0 : 32);
    load_norm_tile<true>(P, row0, nrows, gam, bet, eps, nullptr, Ph, Raw, nullptr, lane);
    if (P0) Q0[lane] = (lane < 2 * nrows) ? P0[row0 * 2 + lane] : 0.f;
    ix[lane] = (i < nrows) ? (h ? pt[row0 + i] : cam[row0 + i]) : 0;
    wave_sync();
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = mfma(Ph[i * LD33 + 2 * s + h], wB[s], acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = crow(r, h);
      if (row < nrows) {
        float y = acc[r] + cst;
        if (P0) y = fmaf(w32, Q0[2 * row], fmaf(w33, Q0[2 * row + 1], y));
        y += Sp[int64_t(ix[32 + row]) * F + i] + Sv[int64_t(ix[row]) * F + i];
        Pout[(row0 + row) * F + i] = fmaf(y, scale, Raw[row * LD33 + i]);
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
__global__ __launch_bounds__(kThreads) void edge_epilogue_bwd_kernel(
    const gasfm_work_item* __restrict__ items, int n_items, const float* __restrict__ dPo,
    const float* __restrict__ P, const float* __restrict__ P0, const float* __restrict__ gam,
    const float* __restrict__ bet, float eps, const float* __restrict__ Wp, int ldWp, float scale,
    float* __restrict__ dSv, float* __restrict__ part_dsv, float* __restrict__ dP0, float* __restrict__ part_w) {
  __shared__ float lds[kWaves][2 * 32 * LD33 + 64];
  __shared__ float red[kWaves * 18 * kW];
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int i = lane & 31, h = lane >> 5;
  float* D = lds[wave];
  float* Ph = D + 32 * LD33;
  float* Q0 = Ph + 32 * LD33;
  // Wp[:, 32:34] for dP0: lane (i,h) needs Wp[j][32+c] for j in its half -> registers
  float w2[16][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = 16 * h + k;
    w2[k][0] = P0 ? Wp[j * ldWp + 32] * scale : 0.f;
    w2[k][1] = P0 ? Wp[j * ldWp + 33] * scale : 0.f;
  }
  f32x16 accW = zero16();
  float accP0[2] = {0.f, 0.f};
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;
  for (int it = gw; it < n_items; it += nw) {
    const gasfm_work_item w = items[it];
    float dsv = 0.f;
    for (int64_t row0 = w.begin; row0 < w.end; row0 += 32) {
      const int nrows = int(w.end - row0 < 32 ? w.end - row0 : 32);
      load_tile<F>(dPo, F, row0, nrows, D, lane);
      load_norm_tile<true>(P, row0, nrows, gam, bet, eps, nullptr, Ph, nullptr, nullptr, lane);
      if (P0) Q0[lane] = (lane < 2 * nrows) ? P0[row0 * 2 + lane] : 0.f;
      wave_sync();
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int row = 2 * s + h;
        const float a = D[row * LD33 + i] * scale;
        accW = mfma(a, Ph[row * LD33 + i], accW);
        dsv += a;
        if (P0) {
          accP0[0] = fmaf(a, Q0[2 * row], accP0[0]);
          accP0[1] = fmaf(a, Q0[2 * row + 1], accP0[1]);
        }
      }
      if (P0) {  // dP0[row i] = sum_j d[i][j] * Wp[j][32:34]; lane half h takes j in [16h, 16h+16)
        float q0 = 0.f, q1 = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const float d = D[i * LD33 + 16 * h + k];
          q0 = fmaf(d, w2[k][0], q0);
          q1 = fmaf(d, w2[k][1], q1);
        }
        q0 += __shfl_xor(q0, 32);
        q1 += __shfl_xor(q1, 32);
        if (i < nrows) dP0[(row0 + i) * 2 + h] = h ? q1 : q0;
      }
      wave_sync();
    }
    dsv += __shfl_xor(dsv, 32);
    if (h == 0) {
      if (w.slot < 0)
        dSv[int64_t(w.seg) * F + i] = dsv;
      else
        part_dsv[int64_t(w.slot) * F + i] = dsv;
    }
  }
  // workgroup reduction of dWp: accW (C layout: row = out j = crow(r,h), col = feature i),
  // accP0[c]: out j = i, summed over the lane halves
  float v[18];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = accW[r];
  v[16] = accP0[0];
  v[17] = accP0[1];
  wg_reduce<18>(v, red, wave, lane);
  if (wave == 0) {
    float* out = part_w + int64_t(blockIdx.x) * 32 * ldWp;
#pragma unroll
    for (int r = 0; r < 16; ++r) out[crow(r, h) * ldWp + i] = v[r];
    if (P0) {
      const float p0 = v[16] + __shfl_xor(v[16], 32), p1 = v[17] + __shfl_xor(v[17], 32);
      if (h == 0) {
        out[i * ldWp + 32] = p0;
        out[i * ldWp + 33] = p1;
      }
    }
  }
}

// =====================================================================================
// edge_prologue_bwd: dP = LN_bwd(mask * (W^T dXL + Wp[:, :32]^T dRes*scale)) + dRes
// part layout per workgroup: [64*32 dW][64 db][32 dgamma][32 dbeta]
// =====================================================================================
template <bool LN, bool RES>
__global__ __launch_bounds__(kThreads) void edge_prologue_bwd_kernel(
    const float* __restrict__ dXL, int64_t ldX, const float* __restrict__ P, const float* __restrict__ dRes,
    int64_t E, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ W, const float* __restrict__ Wp, int ldWp, float scale, float* __restrict__ dP,
    float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int PER_WAVE = 32 * LD65 + 2 * 32 * LD33 + 96;
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int i = lane & 31, h = lane >> 5;
  float* T1 = lds + wave * PER_WAVE;  // dXL tile   32 x 65
  float* T2 = T1 + 32 * LD65;         // x_hat      32 x 33
  float* T3 = T2 + 32 * LD33;         // dRes, then G = dy*gamma
  float* Rs = T3 + 32 * LD33;         // rstd[32], S1[32], S2[32]
  float wB1[32], wB2[16];
#pragma unroll
  for (int s = 0; s < 32; ++s) wB1[s] = W[(2 * s + h) * F + i];  // B[k][j] = W[k][j]
#pragma unroll
  for (int s = 0; s < 16; ++s) wB2[s] = RES ? Wp[(2 * s + h) * ldWp + i] * scale : 0.f;
  const float gi = LN ? gam[i] : 1.f, bi = LN ? bet[i] : 0.f;
  f32x16 accW0 = zero16(), accW1 = zero16();
  float db0 = 0.f, db1 = 0.f, dg = 0.f, dbt = 0.f;
  const int64_t ntiles = (E + 31) / 32;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * 32;
    const int nrows = int(E - row0 < 32 ? E - row0 : 32);
    load_tile<NX>(dXL, ldX, row0, nrows, T1, lane);
    load_norm_tile<LN>(P, row0, nrows, gam, bet, eps, T2, nullptr, nullptr, Rs, lane);
    if (RES) load_tile<F>(dRes, F, row0, nrows, T3, lane);
    wave_sync();
    // dP_hat (C layout) = dXL W  (+ dRes Wp scale)
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = mfma(T1[i * LD65 + 2 * s + h], wB1[s], acc);
    if (RES) {
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma(T3[i * LD33 + 2 * s + h], wB2[s], acc);
    }
    // dW += dXL^T P_hat ; db += colsum(dXL)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int row = 2 * s + h;
      const float xh = T2[row * LD33 + i];
      const float ph = LN ? fmaxf(fmaf(xh, gi, bi), 0.f) : xh;
      const float a0 = T1[row * LD65 + i], a1 = T1[row * LD65 + 32 + i];
      accW0 = mfma(a0, ph, accW0);
      accW1 = mfma(a1, ph, accW1);
      db0 += a0;
      db1 += a1;
    }
    float res[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = crow(r, h);
      res[r] = RES ? T3[row * LD33 + i] : 0.f;
    }
    if (LN) {
      wave_sync();
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = crow(r, h);
        const float xh = T2[row * LD33 + i];
        const float dy = (fmaf(xh, gi, bi) > 0.f) ? acc[r] : 0.f;
        dg = fmaf(dy, xh, dg);
        dbt += dy;
        T3[row * LD33 + i] = dy * gi;
      }
      wave_sync();
      {  // row sums: lane (i, h) takes columns [16h, 16h+16) of row i
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const float g = T3[i * LD33 + 16 * h + k];
          s1 += g;
          s2 = fmaf(g, T2[i * LD33 + 16 * h + k], s2);
        }
        s1 += __shfl_xor(s1, 32);
        s2 += __shfl_xor(s2, 32);
        if (h == 0) {
          Rs[32 + i] = s1 * (1.f / F);
          Rs[64 + i] = s2 * (1.f / F);
        }
      }
      wave_sync();
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = crow(r, h);
        if (row < nrows) {
          const float g = T3[row * LD33 + i], xh = T2[row * LD33 + i];
          const float dx = Rs[row] * (g - Rs[32 + row] - xh * Rs[64 + row]);
          dP[(row0 + row) * F + i] = dx + res[r];
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = crow(r, h);
        if (row < nrows) dP[(row0 + row) * F + i] = acc[r] + res[r];
      }
    }
    wave_sync();
  }
  // workgroup reduction (LDS reused): 32 accW + 2 db + 2 (dg, dbt) floats per lane
  float v[36];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    v[r] = accW0[r];
    v[16 + r] = accW1[r];
  }
  v[32] = db0;
  v[33] = db1;
  v[34] = dg;
  v[35] = dbt;
  wg_reduce<36>(v, lds, wave, lane);
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * (NX * F + NX + 2 * F);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      out[crow(r, h) * F + i] = v[r];
      out[(32 + crow(r, h)) * F + i] = v[16 + r];
    }
    const float t0 = v[32] + __shfl_xor(v[32], 32), t1 = v[33] + __shfl_xor(v[33], 32);
    const float t2 = v[34] + __shfl_xor(v[34], 32), t3 = v[35] + __shfl_xor(v[35], 32);
    if (h == 0) {
      out[NX * F + i] = t0;
      out[NX * F + 32 + i] = t1;
      out[NX * F + NX + i] = t2;
      out[NX * F + NX + F + i] = t3;
    }
  }
}

// =====================================================================================
// segment_rowsum: out[seg] = scale * sum_{e in item} X[src_e]   (32-wide rows, optional perm)
// 8 lanes x float4 per row, 8 rows per wave, 4 row groups in flight.
// =====================================================================================
__global__ __launch_bounds__(kThreads) void segment_rowsum_kernel(const gasfm_work_item* __restrict__ items,
                                                                 int n_items, const int32_t* __restrict__ perm,
                                                                 const float* __restrict__ X, int64_t ldX,
                                                                 float scale, float* __restrict__ out,
                                                                 float* __restrict__ part) {
  const int lane = threadIdx.x & (kW - 1);
  const int row = lane >> 3, c = (lane & 7) * 4;
  const int nw = gridDim.x * kWaves;
  for (int it = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + threadIdx.x / kW); it < n_items; it += nw) {
    const gasfm_work_item w = items[it];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e0 = w.begin; e0 < w.end; e0 += 32) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 8 * u + row;
        if (e < w.end) {
          const int64_t src = perm ? perm[e] : e;
          v[u] = *reinterpret_cast<const float4*>(X + src * ldX + c);
        } else {
          v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x;
        acc.y += v[u].y;
        acc.z += v[u].z;
        acc.w += v[u].w;
      }
    }
#pragma unroll
    for (int o = 8; o < kW; o <<= 1) {
      acc.x += __shfl_xor(acc.x, o);
      acc.y += __shfl_xor(acc.y, o);
      acc.z += __shfl_xor(acc.z, o);
      acc.w += __shfl_xor(acc.w, o);
    }
    if (row == 0) {
      const float4 r = make_float4(acc.x * scale, acc.y * scale, acc.z * scale, acc.w * scale);
      float* dst = (w.slot < 0) ? out + int64_t(w.seg) * F : part + int64_t(w.slot) * F;
      *reinterpret_cast<float4*>(dst + c) = r;
    }
  }
}

int grid_tiles(int64_t E) {
  const int64_t tiles = (E + 31) / 32;
  const int64_t g = (tiles + kWaves - 1) / kWaves;
  return int(g < 1 ? 1 : (g > kMaxGrid ? kMaxGrid : g));
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_edge_part_floats(int32_t which, int64_t E, int32_t n_items) {
  // which: 0 = prologue_bwd partial row, 1 = epilogue_bwd partial row (ldWp = 34)
  const int g = which == 1 ? (n_items < kMaxGrid * kWaves ? (n_items + kWaves - 1) / kWaves : kMaxGrid)
                           : grid_tiles(E);
  const int gg = g < 1 ? 1 : g;
  return which == 0 ? gg * (NX * F + NX + 2 * F) : gg * 32 * 34;
}

extern "C" int gasfm_edge_prologue_fwd(const float* P, int64_t E, const float* ln_w, const float* ln_b,
                                       float eps, const float* W, const float* b, float* Y, int64_t ldY,
                                       void* stream) {
  GASFM_REQUIRE(E >= 0 && P && W && b && Y, "gasfm_edge_prologue_fwd: bad args");
  GASFM_REQUIRE(ldY >= NX, "gasfm_edge_prologue_fwd: ldY < 64");
  GASFM_REQUIRE(aligned16(P), "gasfm_edge_prologue_fwd: P not 16-byte aligned");
  if (E == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (ln_w)
    hipLaunchKernelGGL(edge_prologue_fwd_kernel<true>, dim3(grid_tiles(E)), dim3(kThreads), 0, st, P, E, ln_w,
                       ln_b, eps, W, b, Y, ldY);
  else
    hipLaunchKernelGGL(edge_prologue_fwd_kernel<false>, dim3(grid_tiles(E)), dim3(kThreads), 0, st, P, E, ln_w,
                       ln_b, eps, W, b, Y, ldY);
  return launch_status("gasfm_edge_prologue_fwd");
}

extern "C" int gasfm_edge_epilogue_fwd(const float* P, const float* P0, const int32_t* cam, const int32_t* pt,
                                       int64_t E, const float* ln_w, const float* ln_b, float eps, const float* Wp,
                                       int32_t ldWp, const float* bp, const float* Sp, const float* Sv,
                                       const float* Sg, float scale, float* Pout, void* stream) {
  GASFM_REQUIRE(E >= 0 && P && cam && pt && ln_w && ln_b && Wp && bp && Sp && Sv && Sg && Pout,
                "gasfm_edge_epilogue_fwd: null pointer");
  GASFM_REQUIRE((P0 && ldWp == 34) || (!P0 && ldWp == 32), "gasfm_edge_epilogue_fwd: ldWp=%d vs P0", ldWp);
  GASFM_REQUIRE(aligned16(P), "gasfm_edge_epilogue_fwd: P not 16-byte aligned");
  if (E == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(edge_epilogue_fwd_kernel, dim3(grid_tiles(E)), dim3(kThreads), 0, st, P, P0, cam, pt, E, ln_w,
                     ln_b, eps, Wp, ldWp, bp, Sp, Sv, Sg, scale, Pout);
  return launch_status("gasfm_edge_epilogue_fwd");
}

extern "C" int gasfm_edge_epilogue_bwd(const gasfm_work_item* items, int32_t n_items, const float* dPo,
                                       const float* P, const float* P0, const float* ln_w, const float* ln_b,
                                       float eps, const float* Wp, int32_t ldWp, float scale, float* dSv,
                                       float* part_dsv, float* dP0, float* part_w, void* stream) {
  GASFM_REQUIRE(items && dPo && P && ln_w && ln_b && Wp && dSv && part_w, "gasfm_edge_epilogue_bwd: null pointer");
  GASFM_REQUIRE((P0 && dP0 && ldWp == 34) || (!P0 && ldWp == 32), "gasfm_edge_epilogue_bwd: ldWp=%d vs P0",
                ldWp);
  if (n_items <= 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = n_items < kMaxGrid * kWaves ? (n_items + kWaves - 1) / kWaves : kMaxGrid;
  hipLaunchKernelGGL(edge_epilogue_bwd_kernel, dim3(g), dim3(kThreads), 0, st, items, n_items, dPo, P, P0, ln_w,
                     ln_b, eps, Wp, ldWp, scale, dSv, part_dsv, dP0, part_w);
  return launch_status("gasfm_edge_epilogue_bwd");
}

extern "C" int gasfm_edge_prologue_bwd(const float* dXL, int64_t ldX, const float* P, const float* dRes, int64_t E,
                                       const float* ln_w, const float* ln_b, float eps, const float* W,
                                       const float* Wp, int32_t ldWp, float scale, float* dP, float* part,
                                       void* stream) {
  GASFM_REQUIRE(dXL && P && W && dP && part && ldX >= NX, "gasfm_edge_prologue_bwd: bad args");
  GASFM_REQUIRE(!dRes || Wp, "gasfm_edge_prologue_bwd: dRes needs Wp");
  if (E == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = size_t(kWaves) * (32 * LD65 + 2 * 32 * LD33 + 96) * sizeof(float);
  const int g = grid_tiles(E);
  const bool ln = ln_w != nullptr, res = dRes != nullptr;
#define GASFM_LAUNCH(LNV, RESV)                                                                                 \
  hipLaunchKernelGGL((edge_prologue_bwd_kernel<LNV, RESV>), dim3(g), dim3(kThreads), lds, st, dXL, ldX, P, dRes, \
                     E, ln_w, ln_b, eps, W, Wp, ldWp, scale, dP, part)
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
  const int waves = n_items < 8192 ? n_items : 8192;
  hipLaunchKernelGGL(segment_rowsum_kernel, dim3((waves + kWaves - 1) / kWaves), dim3(kThreads), 0, st, items,
                     n_items, perm, X, ldX, scale, out, part);
  return launch_status("gasfm_segment_rowsum");
}
