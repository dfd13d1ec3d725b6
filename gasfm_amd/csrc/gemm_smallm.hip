// fp32 MFMA GEMMs for the camera-side D x D products when the row count is small, gfx950.
//
// A camera-sharded rank (gasfm_amd/distributed.py) owns m / W view rows: 125 at config 4 on 8
// GPUs.  Its Proj2View MLP and graph_conv_view2global.lin_l products (code/models/layers.py:292-320,
// 352-358, 506-511) are then 125 x 1024 x 1024: 0.27 GFLOP, which hipBLASLt runs in ~11.5 us (one
// 32 x 16 output tile per workgroup, a 1024-long K loop per wave).  Here every wave owns a 16 x 32
// output tile and an eighth of K (128: 64 MFMAs), so 8 x 32 tiles x 8 K-slices = 2,048 waves
// (two per SIMD); the K-slices of a tile are the eight waves of one workgroup and are summed
// through LDS in wave order (deterministic).  Operands are read straight into the
// v_mfma_f32_16x16x4_f32 operand layouts (k index of step (u, j) = 16 u + 4 g + j for lane
// (g = l >> 4, c = l & 15)): float4 loads along a row's contiguous k where the operand is
// k-contiguous, 64-B row segments of scalar loads where it is not.  No LDS staging, no barrier
// in the K loop.
//
//   mode 0  C[M,N] = A[M,K] W[N,K]^T (+ bias[N]) (+ Cin[M,N])   y = x W^T (+ b) (+ skip)
//   mode 1  C[M,N] = A[M,K] W[K,N]                               dx = dy W
//   mode 2  C[I,J] = A[K,I]^T B[K,J]                             dW = dy^T x  (K = rows, small)
// Modes 0 / 1 need K % (16 x 8 K-slices) == 0 and N % 32 == 0 (M arbitrary); mode 2 needs
// I % 16 == 0, J % 128 == 0 and K <= 256 (rows past K read as 0).  Exact fp32 products, fp32 sums in a fixed
// order.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

typedef float f32x4s __attribute__((ext_vector_type(4)));
constexpr int kWs = 64, kTM = 16, kTN = 32, kWavesS = 4, kThreadsS = kWavesS * kWs;
#ifndef GASFM_SMALLM_KSPLIT
#define GASFM_SMALLM_KSPLIT 8  // K slices (waves) per output tile in modes 0 / 1
#endif
constexpr int kSplit = GASFM_SMALLM_KSPLIT, kThreadsR = kSplit * kWs;

__device__ __forceinline__ f32x4s mfma4(float a, float b, f32x4s c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// modes 0 / 1: one workgroup per 16 x 32 tile, wave w takes K range [w K/S, (w+1) K/S), S = kSplit
template <int MODE, int KQ>  // KQ: K / 4 / 16 (u steps per wave)
__global__ __launch_bounds__(kThreadsR) void gemm_sm_rows_kernel(int M, int N, int K, const float* __restrict__ A,
                                                                 int64_t lda, const float* __restrict__ W,
                                                                 int64_t ldw, const float* __restrict__ bias,
                                                                 const float* Cin, int64_t ldCin, float* C,
                                                                 int64_t ldC) {
  __shared__ float red[kSplit][2][kWs * 4];
  const int lane = threadIdx.x & (kWs - 1), wave = threadIdx.x / kWs, c = lane & 15, g = lane >> 4;
  const int ntn = N / kTN;
  const int row0 = (blockIdx.x / ntn) * kTM, col0 = (blockIdx.x % ntn) * kTN;
  const int k0 = wave * (K / kSplit);
  const int ra = row0 + c < M ? row0 + c : M - 1;  // clamped: rows past M are computed and not stored
  const float* ap = A + int64_t(ra) * lda + k0 + 4 * g;
  float4 av[KQ];
#pragma unroll
  for (int u = 0; u < KQ; ++u) av[u] = *reinterpret_cast<const float4*>(ap + 16 * u);
  f32x4s acc[2] = {f32x4s{0.f, 0.f, 0.f, 0.f}, f32x4s{0.f, 0.f, 0.f, 0.f}};
  if (MODE == 0) {
    float4 bv[2][KQ];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float* bp = W + int64_t(col0 + 16 * t + c) * ldw + k0 + 4 * g;
#pragma unroll
      for (int u = 0; u < KQ; ++u) bv[t][u] = *reinterpret_cast<const float4*>(bp + 16 * u);
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first MFMA (one wave per SIMD: VGPRs are free)
#pragma unroll
    for (int u = 0; u < KQ; ++u) {
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma4(av[u].x, bv[t][u].x, acc[t]);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma4(av[u].y, bv[t][u].y, acc[t]);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma4(av[u].z, bv[t][u].z, acc[t]);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma4(av[u].w, bv[t][u].w, acc[t]);
    }
  } else {
    float bv[KQ][2][4];
#pragma unroll
    for (int u = 0; u < KQ; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* bp = W + int64_t(k0 + 16 * u + 4 * g + j) * ldw + col0 + c;
        bv[u][0][j] = bp[0];
        bv[u][1][j] = bp[16];
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < KQ; ++u) {
      const float a4[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma4(a4[j], bv[u][t][j], acc[t]);
    }
  }
  // the K-slices summed in wave order
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][t][r * kWs + lane] = acc[t][r];
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = col0 + 16 * t + c;
    const float b = bias ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      float v = red[0][t][r * kWs + lane];
#pragma unroll
      for (int w = 1; w < kSplit; ++w) v += red[w][t][r * kWs + lane];
      if (row < M) {
        v += b;
        if (Cin) v += Cin[int64_t(row) * ldCin + col];
        C[int64_t(row) * ldC + col] = v;
      }
    }
  }
}

// mode 2: C[I,J] = A[K,I]^T B[K,J]; one wave per 16 x 32 tile, a workgroup = 4 tiles along J; every
// operand load issued before the first MFMA (KU = ceil(K / 16) u-steps, rows past K read as 0)
template <int KU>
__global__ __launch_bounds__(kThreadsS) void gemm_sm_wgrad_kernel(int I, int J, int K, const float* __restrict__ A,
                                                                  int64_t lda, const float* __restrict__ B,
                                                                  int64_t ldb, float* __restrict__ C, int64_t ldC) {
  const int lane = threadIdx.x & (kWs - 1), wave = threadIdx.x / kWs, c = lane & 15, g = lane >> 4;
  const int nwj = J / (kTN * kWavesS);
  const int i0 = (blockIdx.x / nwj) * kTM, j0 = ((blockIdx.x % nwj) * kWavesS + wave) * kTN;
  float a4[KU][4], b4[KU][2][4];
#pragma unroll
  for (int u = 0; u < KU; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * u + 4 * g + j;
      const int kk = k < K ? k : K - 1;  // clamped address, A zeroed where consumed
      a4[u][j] = A[int64_t(kk) * lda + i0 + c];
      b4[u][0][j] = B[int64_t(kk) * ldb + j0 + c];
      b4[u][1][j] = B[int64_t(kk) * ldb + j0 + 16 + c];
    }
  __builtin_amdgcn_sched_barrier(0);
  f32x4s acc[2] = {f32x4s{0.f, 0.f, 0.f, 0.f}, f32x4s{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int u = 0; u < KU; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = 16 * u + 4 * g + j < K ? a4[u][j] : 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma4(a, b4[u][t][j], acc[t]);
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) C[int64_t(i0 + 4 * g + r) * ldC + j0 + 16 * t + c] = acc[t][r];
}

template <int MODE>
int launch_rows(int M, int N, int K, const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias,
                const float* Cin, int64_t ldCin, float* C, int64_t ldC, hipStream_t st) {
  const dim3 grid(unsigned(((M + kTM - 1) / kTM) * (N / kTN)));
  switch (K / kSplit / 16) {
    case 16:
      hipLaunchKernelGGL((gemm_sm_rows_kernel<MODE, 16>), grid, dim3(kThreadsR), 0, st, M, N, K, A, lda, W, ldw, bias,
                         Cin, ldCin, C, ldC);
      break;
    case 8:
      hipLaunchKernelGGL((gemm_sm_rows_kernel<MODE, 8>), grid, dim3(kThreadsR), 0, st, M, N, K, A, lda, W, ldw, bias,
                         Cin, ldCin, C, ldC);
      break;
    case 4:
      hipLaunchKernelGGL((gemm_sm_rows_kernel<MODE, 4>), grid, dim3(kThreadsR), 0, st, M, N, K, A, lda, W, ldw, bias,
                         Cin, ldCin, C, ldC);
      break;
    case 2:
      hipLaunchKernelGGL((gemm_sm_rows_kernel<MODE, 2>), grid, dim3(kThreadsR), 0, st, M, N, K, A, lda, W, ldw, bias,
                         Cin, ldCin, C, ldC);
      break;
    case 1:
      hipLaunchKernelGGL((gemm_sm_rows_kernel<MODE, 1>), grid, dim3(kThreadsR), 0, st, M, N, K, A, lda, W, ldw, bias,
                         Cin, ldCin, C, ldC);
      break;
    default:
      return GASFM_ERR_INVALID;
  }
  return GASFM_OK;
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

// 1 when gasfm_gemm_f32_smallm takes (mode, M, N, K)
extern "C" int32_t gasfm_gemm_f32_smallm_ok(int32_t mode, int32_t M, int32_t N, int32_t K) {
  if (M < 0 || N <= 0 || K <= 0) return 0;
  if (mode == 0 || mode == 1) {
    const int q = K / kSplit / 16;
    return K % (16 * kSplit) == 0 && N % kTN == 0 && (q == 1 || q == 2 || q == 4 || q == 8 || q == 16);
  }
  if (mode == 2) return M % kTM == 0 && N % (kTN * kWavesS) == 0 && K <= 256;  // (I = M, J = N)
  return 0;
}

extern "C" int gasfm_gemm_f32_smallm(int32_t mode, int32_t M, int32_t N, int32_t K, const float* A, int64_t lda,
                                     const float* B, int64_t ldb, const float* bias, const float* Cin, int64_t ldCin,
                                     float* C, int64_t ldC, void* stream) {
  GASFM_REQUIRE(gasfm_gemm_f32_smallm_ok(mode, M, N, K), "gasfm_gemm_f32_smallm: mode=%d M=%d N=%d K=%d", mode, M, N,
                K);
  if (M == 0) return GASFM_OK;
  GASFM_REQUIRE(A && B && C, "gasfm_gemm_f32_smallm: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (mode == 0) {
    GASFM_REQUIRE(aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0,
                  "gasfm_gemm_f32_smallm: mode 0 reads float4 runs of A and W rows");
    const int st0 = launch_rows<0>(M, N, K, A, lda, B, ldb, bias, Cin, ldCin, C, ldC, st);
    if (st0 != GASFM_OK) return st0;
  } else if (mode == 1) {
    GASFM_REQUIRE(aligned16(A) && lda % 4 == 0, "gasfm_gemm_f32_smallm: mode 1 reads float4 runs of A rows");
    GASFM_REQUIRE(!bias && !Cin, "gasfm_gemm_f32_smallm: mode 1 has no epilogue");
    const int st1 = launch_rows<1>(M, N, K, A, lda, B, ldb, nullptr, nullptr, 0, C, ldC, st);
    if (st1 != GASFM_OK) return st1;
  } else {
    GASFM_REQUIRE(!bias && !Cin, "gasfm_gemm_f32_smallm: mode 2 has no epilogue");
    const dim3 grid(unsigned((M / kTM) * (N / (kTN * kWavesS))));
    const int ku = (K + 15) / 16;
#define GASFM_WG(KU_)                                                                                          \
  hipLaunchKernelGGL(gemm_sm_wgrad_kernel<KU_>, grid, dim3(kThreadsS), 0, st, M, N, K, A, lda, B, ldb, C, ldC)
    if (ku <= 1)
      GASFM_WG(1);
    else if (ku <= 2)
      GASFM_WG(2);
    else if (ku <= 4)
      GASFM_WG(4);
    else if (ku <= 8)
      GASFM_WG(8);
    else
      GASFM_WG(16);
#undef GASFM_WG
  }
  return launch_status("gasfm_gemm_f32_smallm");
}
