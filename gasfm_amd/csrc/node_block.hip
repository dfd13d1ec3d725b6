// Fused LayerNorm -> ReLU -> Linear (-> + x) over the 64-wide scene-point rows, gfx950.
//
// The point side of every GASFM block (n ~ 200k rows x n_feat_scenepoint = 64) runs three
// such chains (reference code/models/layers.py):
//   state projection   Lin_64->32(relu(LN(x_prev)))           layers.py:48-56 via :403-404
//   pre-MLP + skip     x + Lin_64->64(relu(LN(x)))            layers.py:449-456
//   proj-update term   Lin_64->32,nobias(relu(LN(x)))         layers.py:928-935
// which aten runs as LayerNorm, clamp, GEMM (+ add) forward and GEMM, threshold_backward,
// LayerNorm backward (3 kernels), bias reduce (+ add) backward, each re-reading the 51 MB
// point tensor.  Here one kernel reads x once and writes y; one backward kernel reads
// (dy, x) once and writes dx plus per-workgroup [dW | db | dgamma | dbeta] partials that
// gasfm_colsum finishes in a fixed order (deterministic, no atomics).
//
// Tiles are 16 rows x 64: a 16-lane group holds one row (float4 per lane), so the LayerNorm
// statistics are 4 xor-shuffles; the GEMMs run on v_mfma_f32_16x16x4_f32 against weights
// staged once per workgroup in LDS (row stride 80 / 48 floats).  LayerNorm statistics are
// recomputed in the backward pass (x is re-read anyway; no mean/rstd tensors are stored).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

using namespace tile;

constexpr int FI = 64;           // input width (n_feat_scenepoint)
constexpr int LDX = 66;          // LDS row stride of 64-wide tiles
constexpr int LDWB = 80;         // LDS row stride of the 64-column weights in the backward pass

template <int FO>
struct Fwd {
  static constexpr int LDW = FO == 64 ? 80 : 48;  // staged W^T [64 x FO]
};

// 16 x 64 tile of X: lane l loads row (l>>4) + 4u (u < 4), columns 4(l&15)..+3.  Writes
// x_hat (Xh), relu(x_hat*gamma + beta) (Ph), raw x (Raw) and rstd (Rs); each optional.
// Rows >= nrows are zeros (x_hat and the activation included).
__device__ __forceinline__ void load_ln64(const float* __restrict__ X, int64_t row0, int nrows,
                                          const float* __restrict__ gam, const float* __restrict__ bet, float eps,
                                          float* Xh, float* Ph, float* Raw, float* Rs, int lane) {
  const int c = (lane & 15) * 4;
  float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (Ph) {
    g4 = *reinterpret_cast<const float4*>(gam + c);
    b4 = *reinterpret_cast<const float4*>(bet + c);
  }
  float4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (lane >> 4) + 4 * u;
    v[u] = *reinterpret_cast<const float4*>(X + (row0 + (r < nrows ? r : 0)) * FI + c);  // see load_tile
    if (r >= nrows) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (lane >> 4) + 4 * u;
    const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    if (Raw) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Raw[r * LDX + c + k] = x[k];
    }
    const float mean = sum16(x[0] + x[1] + x[2] + x[3]) * (1.f / FI);
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) q = fmaf(x[k] - mean, x[k] - mean, q);
    const float rstd = rsq_normal(sum16(q) * (1.f / FI) + eps);
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
    const bool live = r < nrows;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (x[k] - mean) * rstd;
      if (Xh) Xh[r * LDX + c + k] = live ? xh : 0.f;
      if (Ph) Ph[r * LDX + c + k] = live ? fmaxf(fmaf(xh, gg[k], bb[k]), 0.f) : 0.f;
    }
    if (Rs && (lane & 15) == 0) Rs[r] = rstd;
  }
}

// Y[i] = W relu(LN(X[i])) + b (+ X[i] when RES)       W: [FO x 64], Y row stride ldY
template <int FO, bool RES>
__global__ __launch_bounds__(kThreads) void node_fwd_kernel(const float* __restrict__ X, int64_t N,
                                                           const float* __restrict__ gam,
                                                           const float* __restrict__ bet, float eps,
                                                           const float* __restrict__ W,
                                                           const float* __restrict__ b, float* __restrict__ Y,
                                                           int64_t ldY) {
  constexpr int LDW = Fwd<FO>::LDW;
  constexpr int NT = FO / 16;
  __shared__ float Wt[FI * LDW];  // Wt[k][n] = W[n][k]
  __shared__ float tiles[kWaves][(RES ? 2 : 1) * TR * LDX];
  {
    tile::Stage<FO * FI, kThreads> sw;
    sw.load([&](int q) { return W[q]; });
    sw.store([&](int q, float v) { Wt[(q % FI) * LDW + q / FI] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T = tiles[wave];
  float* Raw = RES ? T + TR * LDX : nullptr;
  float bias[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bias[nt] = b ? b[nt * 16 + c] : 0.f;
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    load_ln64(X, row0, nrows, gam, bet, eps, nullptr, T, Raw, nullptr, lane);
    wave_sync();
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = zero4();
#pragma unroll
    for (int s = 0; s < FI / 4; ++s) {
      const float a = T[c * LDX + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16(a, Wt[(4 * s + g) * LDW + nt * 16 + c], acc[nt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      if (e < nrows) {
        float* y = Y + (row0 + e) * ldY;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          float o = acc[nt][r] + bias[nt];
          if (RES) o += Raw[e * LDX + nt * 16 + c];
          y[nt * 16 + c] = o;
        }
      }
    }
    wave_sync();
  }
}

// dX = LN_bwd(mask * (dY W)) (+ dY when RES); per-workgroup partials
// part: [FO*64 dW][FO db][64 dgamma][64 dbeta]
template <int FO, bool RES>
__global__ __launch_bounds__(kThreads) void node_bwd_kernel(const float* __restrict__ dY,
                                                           const float* __restrict__ X, int64_t N,
                                                           const float* __restrict__ gam,
                                                           const float* __restrict__ bet, float eps,
                                                           const float* __restrict__ W, float* __restrict__ dX,
                                                           float* __restrict__ part) {
  constexpr int LDY = FO + 2;
  constexpr int MT = FO / 16;
  constexpr int PW = TR * LDY + TR * LDX + TR;
  constexpr int NRED = MT * 16 + MT + 8;
  constexpr int LDS = FO * LDWB + kWaves * PW;
  static_assert(NRED * kW <= LDS, "reduction scratch");
  __shared__ float lds[LDS];
  float* Wl = lds;  // Wl[k][j] = W[k][j]: B operand of dY W
  {
    tile::Stage<FO * FI, kThreads> sw;
    sw.load([&](int q) { return W[q]; });
    sw.store([&](int q, float v) { Wl[(q / FI) * LDWB + q % FI] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T1 = lds + FO * LDWB + wave * PW;  // dY     16 x FO
  float* T2 = T1 + TR * LDY;                // x_hat  16 x 64
  float* Rs = T2 + TR * LDX;                // rstd   16
  float gi[4], bi[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    gi[nt] = gam[nt * 16 + c];
    bi[nt] = bet[nt * 16 + c];
  }
  f32x4 accW[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) accW[mt][nt] = zero4();
  float db[MT], dg[4], dbt[4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) db[mt] = 0.f;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) dg[nt] = dbt[nt] = 0.f;
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = int64_t(blockIdx.x) * kWaves + wave, nw = int64_t(gridDim.x) * kWaves;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    load_tile<FO, LDY>(dY, FO, row0, nrows, T1, lane);
    load_ln64(X, row0, nrows, gam, bet, eps, T2, nullptr, nullptr, Rs, lane);
    wave_sync();
    // d relu-out (C layout: row 4g+r, column nt*16+c) = dY W
    f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < FO / 4; ++s) {
      const float a = T1[c * LDY + 4 * s + g];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(a, Wl[(4 * s + g) * LDWB + nt * 16 + c], acc[nt]);
    }
    // dW += dY^T relu(LN(x)), db += column sums of dY
#pragma unroll
    for (int s = 0; s < TR / 4; ++s) {
      const int row = 4 * s + g;
      float ph[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) ph[nt] = fmaxf(fmaf(T2[row * LDX + nt * 16 + c], gi[nt], bi[nt]), 0.f);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float a = T1[row * LDY + mt * 16 + c];
        db[mt] += a;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) accW[mt][nt] = mfma16(a, ph[nt], accW[mt][nt]);
      }
    }
    // ReLU mask + LayerNorm backward; a row's 64 columns are 16 lanes x 4 column tiles
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      float gv[4], xh[4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        xh[nt] = T2[e * LDX + nt * 16 + c];
        const float dy = (fmaf(xh[nt], gi[nt], bi[nt]) > 0.f) ? acc[nt][r] : 0.f;
        dg[nt] = fmaf(dy, xh[nt], dg[nt]);
        dbt[nt] += dy;
        gv[nt] = dy * gi[nt];
        s1 += gv[nt];
        s2 = fmaf(gv[nt], xh[nt], s2);
      }
      s1 = sum16(s1) * (1.f / FI);
      s2 = sum16(s2) * (1.f / FI);
      if (e < nrows) {
        const float rs = Rs[e];
        float* dx = dX + (row0 + e) * FI;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          float o = rs * (gv[nt] - s1 - xh[nt] * s2);
          if (RES) o += T1[e * LDY + nt * 16 + c];
          dx[nt * 16 + c] = o;
        }
      }
    }
    wave_sync();
  }
  float v[NRED];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(mt * 4 + nt) * 4 + r] = accW[mt][nt][r];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) v[MT * 16 + mt] = db[mt];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    v[MT * 17 + nt] = dg[nt];
    v[MT * 17 + 4 + nt] = dbt[nt];
  }
  wg_reduce_ordered<NRED, kWaves, LDS>(v, lds, wave, lane);
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * (FO * FI + FO + 2 * FI);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(mt * 16 + 4 * g + r) * FI + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
    float tt[MT + 8];
#pragma unroll
    for (int k = 0; k < MT + 8; ++k) tt[k] = sum_groups(v[MT * 16 + k]);
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) out[FO * FI + mt * 16 + c] = tt[mt];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        out[FO * FI + FO + nt * 16 + c] = tt[MT + nt];
        out[FO * FI + FO + FI + nt * 16 + c] = tt[MT + 4 + nt];
      }
    }
  }
}

int64_t tiles_of(int64_t N) { return (N + TR - 1) / TR; }

template <class K>
int grid_of(K kernel, int64_t N) {
  return resident_grid(reinterpret_cast<const void*>(kernel), kThreads, 0, tiles_of(N), kWaves);
}

// backward grid (= partial rows) of the variant a call uses
int bwd_grid(int64_t N, int n_out, int residual) {
  if (n_out == 32) return grid_of(&node_bwd_kernel<32, false>, N);
  return residual ? grid_of(&node_bwd_kernel<64, true>, N) : grid_of(&node_bwd_kernel<64, false>, N);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_node_part_rows(int64_t N, int32_t n_out, int32_t residual) {
  return bwd_grid(N, n_out, residual);
}

extern "C" int gasfm_node_ln_linear_fwd(const float* X, int64_t N, int32_t n_in, const float* ln_w,
                                        const float* ln_b, float eps, const float* W, const float* b, int32_t n_out,
                                        int32_t residual, float* Y, int64_t ldY, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_node_ln_linear_fwd: N < 0");
  GASFM_REQUIRE(n_in == FI && (n_out == 32 || n_out == 64), "gasfm_node_ln_linear_fwd: unsupported widths %d -> %d",
                n_in, n_out);
  GASFM_REQUIRE(!residual || n_out == n_in, "gasfm_node_ln_linear_fwd: residual needs n_out == n_in");
  GASFM_REQUIRE(ldY >= n_out, "gasfm_node_ln_linear_fwd: ldY < n_out");
  if (N == 0) return GASFM_OK;  // empty tensors may carry null data pointers
  GASFM_REQUIRE(X && ln_w && ln_b && W && Y, "gasfm_node_ln_linear_fwd: null pointer");
  GASFM_REQUIRE(aligned16(X) && aligned16(ln_w) && aligned16(ln_b), "gasfm_node_ln_linear_fwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n_out == 32)
    hipLaunchKernelGGL((node_fwd_kernel<32, false>), dim3(grid_of(&node_fwd_kernel<32, false>, N)), dim3(kThreads), 0, st, X, N, ln_w, ln_b, eps, W, b, Y,
                       ldY);
  else if (residual)
    hipLaunchKernelGGL((node_fwd_kernel<64, true>), dim3(grid_of(&node_fwd_kernel<64, true>, N)), dim3(kThreads), 0, st, X, N, ln_w, ln_b, eps, W, b, Y,
                       ldY);
  else
    hipLaunchKernelGGL((node_fwd_kernel<64, false>), dim3(grid_of(&node_fwd_kernel<64, false>, N)), dim3(kThreads), 0, st, X, N, ln_w, ln_b, eps, W, b, Y,
                       ldY);
  return launch_status("gasfm_node_ln_linear_fwd");
}

extern "C" int gasfm_node_ln_linear_bwd(const float* dY, const float* X, int64_t N, int32_t n_in, const float* ln_w,
                                        const float* ln_b, float eps, const float* W, int32_t n_out,
                                        int32_t residual, float* dX, float* part, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_node_ln_linear_bwd: N < 0");
  GASFM_REQUIRE(n_in == FI && (n_out == 32 || n_out == 64), "gasfm_node_ln_linear_bwd: unsupported widths %d -> %d",
                n_in, n_out);
  GASFM_REQUIRE(!residual || n_out == n_in, "gasfm_node_ln_linear_bwd: residual needs n_out == n_in");
  if (N == 0) return GASFM_OK;  // empty tensors may carry null data pointers
  GASFM_REQUIRE(dY && X && ln_w && ln_b && W && dX && part, "gasfm_node_ln_linear_bwd: null pointer");
  GASFM_REQUIRE(aligned16(dY) && aligned16(X), "gasfm_node_ln_linear_bwd: alignment");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = bwd_grid(N, n_out, residual);
  if (n_out == 32)
    hipLaunchKernelGGL((node_bwd_kernel<32, false>), dim3(g), dim3(kThreads), 0, st, dY, X, N, ln_w, ln_b, eps, W,
                       dX, part);
  else if (residual)
    hipLaunchKernelGGL((node_bwd_kernel<64, true>), dim3(g), dim3(kThreads), 0, st, dY, X, N, ln_w, ln_b, eps, W, dX,
                       part);
  else
    hipLaunchKernelGGL((node_bwd_kernel<64, false>), dim3(g), dim3(kThreads), 0, st, dY, X, N, ln_w, ln_b, eps, W,
                       dX, part);
  return launch_status("gasfm_node_ln_linear_bwd");
}
