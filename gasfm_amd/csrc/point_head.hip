// The scene-point head of GraphAttnSfMNet as fused row-tile kernels, gfx950.
//
// Reference (code/models/graph_attn_sfm.py:170-174, layers.py:10-44 with norm=False, two hidden
// layers -- the configuration's n_hidden_layers):
//   pts3D = [scenepoint_head(relu(p))^T ; 1],
//   scenepoint_head = Linear(64,64) ReLU Linear(64,64) ReLU Linear(64,3),  p = final point features.
// aten runs it as three ReLUs over [n x 64] (51 MB each at config 4), three GEMMs, a transpose and a
// concatenation, and in the backward three ReLU masks, three GEMM pairs and three tall bias sums.
// Here:
//   point_head_fwd     one pass over p: relu, both hidden layers (v_mfma_f32_16x16x4_f32 against
//                      weights staged in LDS), the 3-wide output layer, and pts3D [4, n] written
//                      directly (rows 0-2 the coordinates, row 3 the ones);
//   point_head_bwd_b   the second and third layers' weight / bias gradients;
//   point_head_bwd_a   dp and the first layer's weight / bias gradients.
// Both backward kernels recompute the forward from p (one 51 MB read each instead of writing and
// re-reading two activations); two kernels rather than one because one would hold 148 weight-
// gradient accumulators per lane.  Weight gradients leave as per-workgroup partial rows (ordered
// workgroup reduction) for gasfm_colsum: deterministic, no atomics.
//
// Tile conventions are point_block.hip's (tile.hpp): wave = 16-row tile, MFMA A[i = lane&15][k =
// lane>>4], B[k][j = lane&15], C[row = 4 (lane>>4) + r][col = lane&15].  Activation tiles and the
// weights (natural [out][in] layout) both use row stride 66 (== 2 mod 32): A reads T[i][k] and the
// forward's transposed weight reads W[j][k] are conflict-free, the backward's W[k][j] reads 2-way.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tile.hpp"

namespace gasfm {
namespace {

using namespace tile;

constexpr int FP = 64, FO = 3;
constexpr int L66 = 66, L17 = 17;
constexpr int kWavesH = 8, kThreadsH = kWavesH * kW;
constexpr int TS = TR * L66;                          // one activation tile
constexpr int PART_A = FP * FP + FP;                  // dW1 | db1
constexpr int PART_B = FP * FP + FO * FP + FP + FO;   // dW2 | dW3 | db2 | db3

// [NO x FP] weight into LDS rows of stride L66; rows [NO, NOP) zero
template <int NO, int NOP>
__device__ __forceinline__ void stage_w(const float* __restrict__ W, float* Ws) {
  Stage<NO * FP, kThreadsH> s;
  s.load([&](int q) { return W[q]; });
  s.store([&](int q, float v) { Ws[(q / FP) * L66 + q % FP] = v; });
  if constexpr (NOP > NO) {
    for (int q = threadIdx.x; q < (NOP - NO) * FP; q += kThreadsH) Ws[(NO + q / FP) * L66 + q % FP] = 0.f;
  }
}

// acc[nt] (C layout, 16 x 64) = A (16 x 64 LDS tile, relu'd on read when RELU_A) . B, where
// B[k][j] = W[j][k] (TRANS: x W^T, a forward layer) or W[k][j] (dy W, a backward layer)
template <bool RELU_A, bool TRANS>
__device__ __forceinline__ void mm64(const float* A, const float* W, f32x4 (&acc)[4], int c, int g) {
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = zero4();
#pragma unroll
  for (int s = 0; s < FP / 4; ++s) {
    const int k = 4 * s + g;
    float a = A[c * L66 + k];
    if (RELU_A) a = fmaxf(a, 0.f);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float b = TRANS ? W[(nt * 16 + c) * L66 + k] : W[k * L66 + nt * 16 + c];
      acc[nt] = mfma16(a, b, acc[nt]);
    }
  }
}

// C layout + bias -> LDS tile, relu'd when RELU
template <bool RELU>
__device__ __forceinline__ void c_to_lds(const f32x4 (&acc)[4], const float (&b)[4], float* T, int c, int g) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float v = acc[nt][r] + b[nt];
      T[(4 * g + r) * L66 + nt * 16 + c] = RELU ? fmaxf(v, 0.f) : v;
    }
}

// masked gradient (C layout) -> LDS tile D: D = acc where Y > 0, else 0 (D may be Y: each element
// is read and written by the same lane)
__device__ __forceinline__ void mask_to_lds(const f32x4 (&acc)[4], const float* Y, float* D, int c, int g) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int o = (4 * g + r) * L66 + nt * 16 + c;
      D[o] = Y[o] > 0.f ? acc[nt][r] : 0.f;
    }
}

__device__ __forceinline__ void load_relu_p(const float* __restrict__ P, int64_t row0, int nrows, float* T0,
                                            int lane) {
  float4 v[4];
  rows_load<FP>(P, FP, row0, nrows, v, lane);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    v[u] = make_float4(fmaxf(v[u].x, 0.f), fmaxf(v[u].y, 0.f), fmaxf(v[u].z, 0.f), fmaxf(v[u].w, 0.f));
  rows_to_lds<FP, L66>(T0, v, lane);
}

// The backward kernels' forward recomputation: T0 = relu(p), T1 = y1, T2 = y2 (pre-activations).
__device__ __forceinline__ void recompute(const float* __restrict__ P, int64_t row0, int nrows, float* T0, float* T1,
                                          float* T2, const float* W1s, const float* W2s, const float (&b1)[4],
                                          const float (&b2)[4], int lane, int c, int g) {
  load_relu_p(P, row0, nrows, T0, lane);
  wave_sync();
  f32x4 acc[4];
  mm64<false, true>(T0, W1s, acc, c, g);
  c_to_lds<false>(acc, b1, T1, c, g);
  wave_sync();
  mm64<true, true>(T1, W2s, acc, c, g);
  c_to_lds<false>(acc, b2, T2, c, g);
  wave_sync();
}

// dY3 rows [row0, row0 + 16) of dpts3D (rows 0-2 of the [4, n] gradient) as a 16 x 16 tile of row
// stride L17 (odd: both the A read D[i][k] and the row read D[row][c] are conflict-free); columns >= 3
// zero.  Rows past nrows zero.
__device__ __forceinline__ void load_dy3(const float* __restrict__ dout, int64_t N, int64_t row0, int nrows, float* D3,
                                         int lane) {
  const int e = lane & 15, j = lane >> 4;
  D3[e * L17 + j] = (j < FO && e < nrows) ? dout[int64_t(j) * N + row0 + e] : 0.f;
#pragma unroll
  for (int k = 4 + j; k < 16; k += 4) D3[e * L17 + k] = 0.f;
}

// dh2 = dY3 (16 x 3) . W3 (3 x 64): one k-step (k = 3 zero in both operands)
__device__ __forceinline__ void dh_from_dy3(const float* D3, const float* W3s, f32x4 (&acc)[4], int c, int g) {
  const float a = D3[c * L17 + g];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(a, W3s[g * L66 + nt * 16 + c], zero4());
}

// dW[mt*16 + i][nt*16 + j] += sum_rows D[row][mt*16 + i] Hin[row][nt*16 + j] (Hin = relu(Y) when RELU,
// else Y); db[mt] += this lane's share of the column sums of D
template <bool RELU>
__device__ __forceinline__ void acc_dw(const float* D, const float* Y, f32x4 (&dW)[4][4], float (&db)[4], int c, int g) {
#pragma unroll
  for (int s = 0; s < TR / 4; ++s) {
    const int row = 4 * s + g;
    float h[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float y = Y[row * L66 + nt * 16 + c];
      h[nt] = RELU ? fmaxf(y, 0.f) : y;
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const float a = D[row * L66 + mt * 16 + c];
      db[mt] += a;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dW[mt][nt] = mfma16(a, h[nt], dW[mt][nt]);
    }
  }
}

// dW [64 x 64] (C layout, rows = output features) to a partial row
__device__ __forceinline__ void store_dw(const float* v, float* out, int c, int g) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) out[(mt * 16 + 4 * g + r) * FP + nt * 16 + c] = v[(mt * 4 + nt) * 4 + r];
}

// ------------------------------------------------------------------------------------------ fwd
__global__ __launch_bounds__(kThreadsH) void point_head_fwd_kernel(const float* __restrict__ P, int64_t N,
                                                                   const float* __restrict__ W1,
                                                                   const float* __restrict__ b1,
                                                                   const float* __restrict__ W2,
                                                                   const float* __restrict__ b2,
                                                                   const float* __restrict__ W3,
                                                                   const float* __restrict__ b3,
                                                                   float* __restrict__ out) {
  constexpr int PW = 2 * TS;
  __shared__ float W1s[FP * L66], W2s[FP * L66], W3s[16 * L66];
  __shared__ float tiles[kWavesH * PW];
  stage_w<FP, FP>(W1, W1s);
  stage_w<FP, FP>(W2, W2s);
  stage_w<FO, 16>(W3, W3s);
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T0 = tiles + wave * PW;
  float* T1 = T0 + TS;
  float bv1[4], bv2[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bv1[nt] = b1[nt * 16 + c];
    bv2[nt] = b2[nt * 16 + c];
  }
  const float bv3 = c < FO ? b3[c] : 0.f;
  const int64_t ntiles = (N + TR - 1) / TR;
  for (int64_t t = int64_t(blockIdx.x) * kWavesH + wave; t < ntiles; t += int64_t(gridDim.x) * kWavesH) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    load_relu_p(P, row0, nrows, T0, lane);
    wave_sync();
    f32x4 acc[4];
    mm64<false, true>(T0, W1s, acc, c, g);
    c_to_lds<true>(acc, bv1, T1, c, g);  // relu(y1)
    wave_sync();
    mm64<false, true>(T1, W2s, acc, c, g);
    wave_sync();
    c_to_lds<true>(acc, bv2, T0, c, g);  // relu(y2)
    wave_sync();
    f32x4 o3 = zero4();
#pragma unroll
    for (int s = 0; s < FP / 4; ++s) o3 = mfma16(T0[c * L66 + 4 * s + g], W3s[c * L66 + 4 * s + g], o3);
    // o3[r] = output feature c of row 4g + r; column 3 (W3s row 3 is zero) becomes the ones row
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = 4 * g + r;
      if (e < nrows && c <= FO) out[int64_t(c) * N + row0 + e] = c < FO ? o3[r] + bv3 : 1.f;
    }
    wave_sync();
  }
}

// ------------------------------------------------------------------------------------------ bwd
constexpr int PWB = 3 * TS + TR * L17;  // T0 | T1 | T2 | D3 per wave

// dW3 += dY3^T relu(y2), db3;  dW2 += dy2^T relu(y1), db2   with dy2 = (dY3 W3) * (y2 > 0)
__global__ __launch_bounds__(kThreadsH) void point_head_bwd_b_kernel(
    const float* __restrict__ P, int64_t N, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ W3,
    const float* __restrict__ dout, float* __restrict__ part) {
  __shared__ float W1s[FP * L66], W2s[FP * L66], W3s[4 * L66];
  __shared__ float tiles[kWavesH * PWB];
  stage_w<FP, FP>(W1, W1s);
  stage_w<FP, FP>(W2, W2s);
  stage_w<FO, 4>(W3, W3s);
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T0 = tiles + wave * PWB;
  float* T1 = T0 + TS;
  float* T2 = T1 + TS;
  float* D3 = T2 + TS;
  float bv1[4], bv2[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bv1[nt] = b1[nt * 16 + c];
    bv2[nt] = b2[nt * 16 + c];
  }
  f32x4 dW2[4][4], dW3[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    dW3[mt] = zero4();
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dW2[mt][nt] = zero4();
  }
  float db2[4] = {0.f, 0.f, 0.f, 0.f}, db3 = 0.f;
  const int64_t ntiles = (N + TR - 1) / TR;
  for (int64_t t = int64_t(blockIdx.x) * kWavesH + wave; t < ntiles; t += int64_t(gridDim.x) * kWavesH) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    recompute(P, row0, nrows, T0, T1, T2, W1s, W2s, bv1, bv2, lane, c, g);
    load_dy3(dout, N, row0, nrows, D3, lane);
    wave_sync();
    // dW3[j][k] (C rows j = 4g + r, only j < 3 real): A[j][row] = dY3[row][j], B[row][k] = relu(y2)
#pragma unroll
    for (int s = 0; s < TR / 4; ++s) {
      const int row = 4 * s + g;
      const float a = D3[row * L17 + c];
      db3 += a;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dW3[nt] = mfma16(a, fmaxf(T2[row * L66 + nt * 16 + c], 0.f), dW3[nt]);
    }
    f32x4 acc[4];
    dh_from_dy3(D3, W3s, acc, c, g);
    wave_sync();
    mask_to_lds(acc, T2, T2, c, g);  // dy2, in place
    wave_sync();
    acc_dw<true>(T2, T1, dW2, db2, c, g);
    wave_sync();
  }
  constexpr int NRED = 64 + 16 + 4 + 1;
  float v[NRED];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(mt * 4 + nt) * 4 + r] = dW2[mt][nt][r];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[64 + nt * 4 + r] = dW3[nt][r];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[80 + k] = db2[k];
  v[84] = db3;
  wg_reduce_ordered<NRED, kWavesH, kWavesH * PWB>(v, tiles, wave, lane);
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * PART_B;
    store_dw(v, out, c, g);
    if (g == 0) {
#pragma unroll
      for (int r = 0; r < FO; ++r)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) out[FP * FP + r * FP + nt * 16 + c] = v[64 + nt * 4 + r];
    }
    float tt[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) tt[k] = sum_groups(v[80 + k]);
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) out[FP * FP + FO * FP + k * 16 + c] = tt[k];
      if (c < FO) out[FP * FP + FO * FP + FP + c] = tt[4];
    }
  }
}

// dp = (dy1 W1) * (p > 0), dy1 = (dy2 W2) * (y1 > 0);  dW1 += dy1^T relu(p), db1
__global__ __launch_bounds__(kThreadsH) void point_head_bwd_a_kernel(
    const float* __restrict__ P, int64_t N, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ W3,
    const float* __restrict__ dout, float* __restrict__ dP, float* __restrict__ part) {
  __shared__ float W1s[FP * L66], W2s[FP * L66], W3s[4 * L66];
  __shared__ float tiles[kWavesH * PWB];
  stage_w<FP, FP>(W1, W1s);
  stage_w<FP, FP>(W2, W2s);
  stage_w<FO, 4>(W3, W3s);
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T0 = tiles + wave * PWB;
  float* T1 = T0 + TS;
  float* T2 = T1 + TS;
  float* D3 = T2 + TS;
  float bv1[4], bv2[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bv1[nt] = b1[nt * 16 + c];
    bv2[nt] = b2[nt * 16 + c];
  }
  f32x4 dW1[4][4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dW1[mt][nt] = zero4();
  float db1[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ntiles = (N + TR - 1) / TR;
  for (int64_t t = int64_t(blockIdx.x) * kWavesH + wave; t < ntiles; t += int64_t(gridDim.x) * kWavesH) {
    const int64_t row0 = t * TR;
    const int nrows = int(N - row0 < TR ? N - row0 : TR);
    recompute(P, row0, nrows, T0, T1, T2, W1s, W2s, bv1, bv2, lane, c, g);
    load_dy3(dout, N, row0, nrows, D3, lane);
    wave_sync();
    f32x4 acc[4];
    dh_from_dy3(D3, W3s, acc, c, g);
    mask_to_lds(acc, T2, T2, c, g);  // dy2 (zero on rows past nrows: dY3 is)
    wave_sync();
    mm64<false, false>(T2, W2s, acc, c, g);  // dh1 = dy2 W2
    wave_sync();
    mask_to_lds(acc, T1, T1, c, g);  // dy1
    wave_sync();
    acc_dw<false>(T1, T0, dW1, db1, c, g);   // T0 holds relu(p)
    mm64<false, false>(T1, W1s, acc, c, g);  // dh0 = dy1 W1
    wave_sync();
    mask_to_lds(acc, T0, T0, c, g);  // dp: relu(p) > 0 iff p > 0
    wave_sync();
    float4 vo[4];
    rows_from_lds<FP, L66>(T0, vo, lane);
    rows_store<FP>(dP, FP, row0, nrows, vo, lane);
    wave_sync();
  }
  constexpr int NRED = 64 + 4;
  float v[NRED];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(mt * 4 + nt) * 4 + r] = dW1[mt][nt][r];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[64 + k] = db1[k];
  wg_reduce_ordered<NRED, kWavesH, kWavesH * PWB>(v, tiles, wave, lane);
  if (wave == 0) {
    float* out = part + int64_t(blockIdx.x) * PART_A;
    store_dw(v, out, c, g);
    float tt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tt[k] = sum_groups(v[64 + k]);
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) out[FP * FP + k * 16 + c] = tt[k];
    }
  }
}

template <class K>
int grid_h(K kernel, int64_t N) {
  return resident_grid(reinterpret_cast<const void*>(kernel), kThreadsH, 0, (N + TR - 1) / TR, kWavesH);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

// Partial-row shape of the backward's weight gradients: which = 0 pass A (dW1 | db1), 1 pass B
// (dW2 | dW3 | db2 | db3).  Returns the row count (0 when N <= 0), *cols the row width.
extern "C" int32_t gasfm_point_head_part_shape(int64_t N, int32_t which, int32_t* cols) {
  if (cols) *cols = which ? PART_B : PART_A;
  if (N <= 0) return 0;
  return which ? grid_h(&point_head_bwd_b_kernel, N) : grid_h(&point_head_bwd_a_kernel, N);
}

extern "C" int gasfm_point_head_fwd(const float* P, int64_t N, const float* W1, const float* b1, const float* W2,
                                    const float* b2, const float* W3, const float* b3, float* out, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_head_fwd: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(P && W1 && b1 && W2 && b2 && W3 && b3 && out && aligned16(P), "gasfm_point_head_fwd: bad args");
  hipLaunchKernelGGL(point_head_fwd_kernel, dim3(grid_h(&point_head_fwd_kernel, N)), dim3(kThreadsH), 0,
                     reinterpret_cast<hipStream_t>(stream), P, N, W1, b1, W2, b2, W3, b3, out);
  return launch_status("gasfm_point_head_fwd");
}

extern "C" int gasfm_point_head_bwd(const float* P, int64_t N, const float* W1, const float* b1, const float* W2,
                                    const float* b2, const float* W3, const float* dout, float* dP, float* part_a,
                                    float* part_b, void* stream) {
  GASFM_REQUIRE(N >= 0, "gasfm_point_head_bwd: N < 0");
  if (N == 0) return GASFM_OK;
  GASFM_REQUIRE(P && W1 && b1 && W2 && b2 && W3 && dout && dP && part_a && part_b && aligned16(P) && aligned16(dP),
                "gasfm_point_head_bwd: bad args");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(point_head_bwd_b_kernel, dim3(grid_h(&point_head_bwd_b_kernel, N)), dim3(kThreadsH), 0, st, P,
                     N, W1, b1, W2, b2, W3, dout, part_b);
  const int s = launch_status("gasfm_point_head_bwd_b");
  if (s != GASFM_OK) return s;
  hipLaunchKernelGGL(point_head_bwd_a_kernel, dim3(grid_h(&point_head_bwd_a_kernel, N)), dim3(kThreadsH), 0, st, P,
                     N, W1, b1, W2, b2, W3, dout, dP, part_a);
  return launch_status("gasfm_point_head_bwd_a");
}
