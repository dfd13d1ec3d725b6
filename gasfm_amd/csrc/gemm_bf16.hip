// bf16 MFMA GEMM with fp32 operands, fp32 accumulation and a fused epilogue, for gfx950.
//
//   C[M,N] = A[M,K] . B[K,N] (+ Cin[M,N]) (+ bias[N])
//   A(i,k) = A[i*sAm + k*sAk], B(k,j) = B[k*sBk + j*sBn]: one of each pair must be 1, so the
//   same kernel runs the three products of a Linear layer on row-major fp32 tensors:
//     forward   y  = x W^T (+ b, + skip)   A = x [M,K] (k-contiguous), B = W^T (k-contiguous)
//     input     dx = dy W                  A = dy (k-contiguous),       B = W (n-contiguous)
//     weight    dW = dy^T x                A = dy^T (m-contiguous),     B = x (n-contiguous)
//
// BASELINE config 5's "bf16 projections on MFMA" for the dense per-camera layers of the reference
// (code/models/layers.py:292-320, 352-358: Proj2View's 1024-wide MLP; graph_conv_view2global.lin_l
// at layers.py:506-511).  Operands are read as fp32 (the parameters and activations stay fp32),
// rounded to bf16 (round to nearest even, v_cvt_pk_bf16_f32) while being staged into LDS,
// multiplied on v_mfma_f32_16x16x32_bf16 (products exact in fp32) and summed in fp32: the result
// equals the fp32 accumulation of the bf16-rounded operands up to summation order.
//
// Tiling: 64 x 64 output tile per 256-thread workgroup (4 waves, 2 x 2, each 32 x 32 = 2 x 2
// MFMA blocks), K in steps of 32.  The kernel is bound by the latency of re-reading the fp32
// operand panels from L2 / MALL, not by MFMA (2.1 GFLOP of a 1000 x 1024 x 1024 product is
// ~1 us at the dense bf16 peak), so:
//   - kStages K tiles are in flight per thread in REGISTERS (a ring of kStages x 4 float4; the
//     loop is unrolled over the ring so every slot index is static) -- the oldest is converted
//     and written to LDS each step while the newer ones fly;
//   - LDS holds two bf16 tiles (rows padded to 40 bf16: the 16-byte fragment reads of 16 rows
//     cover all 64 banks once), one barrier per K step;
//   - m-/n-contiguous operands (the weight-gradient product) load float4s along the row index
//     for two adjacent k and write bf16 pairs (one dword per row) into the same [row][k] layout;
//   - tiles are mapped XCD-aware: workgroup b runs on XCD b % 8, and the eight XCDs take
//     contiguous ranges of a grouped tile order (4 M-tiles x 8 N-tiles for m = 1000 x 1024), so
//     each XCD's L2 holds only the operand panels its own tiles read.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

#ifndef GASFM_GEMM_STAGES
#define GASFM_GEMM_STAGES 3  // K tiles in flight per thread (A/B knob)
#endif
#ifndef GASFM_GEMM_BK
#define GASFM_GEMM_BK 64  // K step: 32 or 64 (A/B knob)
#endif
constexpr int BM = 64, BN = 64, BK = GASFM_GEMM_BK, LDK = BK + 8, kThreadsG = 256, kStages = GASFM_GEMM_STAGES;
constexpr int kLd = BM * BK / 4 / kThreadsG;  // float4 loads per thread per operand tile (2 or 4)
static_assert(BK == 32 || BK == 64, "BK");
constexpr int kXcd = 8, kGroupM = 4;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4g __attribute__((ext_vector_type(4)));
typedef float f32x2g __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2g __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {  // RNE, v_cvt_pk_bf16_f32
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2g{lo, hi}), bf16x2g));
}

// One 64 x 32 operand tile of "rows" row0 .. row0+63 (m for A, n for B) and k0 .. k0+31, as two
// float4 loads per thread.  Out-of-range float4s (the contiguous extent is a multiple of 4,
// checked on the host, so a float4 is all-in or all-out) read a clamped in-range address and are
// zeroed when stored: no per-load branch.
//   RowContig == false: contiguous along k: thread i -> rows i/8 and i/8 + 32, k = 4 (i % 8)
//   RowContig == true:  contiguous along the rows: thread i -> rows 4 (i % 16) .. +3 at
//                       k = 2 (i / 16) and k + 1
// Element offsets are int32 (the host checks every operand spans < 2^31 elements) and the row
// part is computed once: a load costs one multiply-add (none when k is the unit stride).
template <bool RowContig>
struct Tile {
  const float* X;  // deliberately not __restrict__: with it, the operands count as invariant
                   // memory and the compiler sinks the prefetch loads down to their use one ring
                   // round later (a full-latency wait per K step)
  int s_k, K, kmax;
  int roff[kLd], kk[kLd];
  bool rok[kLd];
  __device__ __forceinline__ static void coord(int u, int& r, int& k) {
    const int i = threadIdx.x;
    if constexpr (!RowContig) {
      r = (i + kThreadsG * u) / (BK / 4);
      k = ((i + kThreadsG * u) % (BK / 4)) * 4;
    } else {  // float4 pairs (k, k + 1): u = 2 p + h
      r = (i % 16) * 4;
      k = (i / 16) * 2 + (u & 1) + 32 * (u >> 1);
    }
  }
  __device__ __forceinline__ Tile(const float* X_, int64_t s_row, int64_t s_k_, int rows, int K_, int row0)
      : X(X_), s_k(int(s_k_)), K(K_), kmax(RowContig ? K_ - 1 : K_ - 4) {
#pragma unroll
    for (int u = 0; u < kLd; ++u) {
      int r, k;
      coord(u, r, k);
      const int gr = row0 + r;
      rok[u] = gr < rows;
      roff[u] = (rok[u] ? gr : rows - (RowContig ? 4 : 1)) * int(s_row);
      kk[u] = k;
    }
  }
  __device__ __forceinline__ void load(f32x4g (&v)[kLd], int k0) const {
#pragma unroll
    for (int u = 0; u < kLd; ++u) {
      const int k = k0 + kk[u] < kmax ? k0 + kk[u] : kmax;
      v[u] = *reinterpret_cast<const f32x4g*>(X + (roff[u] + k * s_k));
    }
  }
  __device__ __forceinline__ void store(f32x4g (&v)[kLd], uint16_t* __restrict__ T, int k0) const {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int u = 0; u < kLd; ++u) {  // zero out-of-range float4s with a mask (a branch would drain vmcnt)
      const uint32_t mk = (rok[u] && k0 + kk[u] < K) ? ~0u : 0u;
      v[u] = __builtin_bit_cast(f32x4g, __builtin_bit_cast(u32x4, v[u]) & mk);
    }
    if constexpr (!RowContig) {
#pragma unroll
      for (int u = 0; u < kLd; ++u) {
        int r, k;
        coord(u, r, k);
        *reinterpret_cast<uint2*>(T + r * LDK + k) = make_uint2(pack_bf16(v[u][0], v[u][1]), pack_bf16(v[u][2], v[u][3]));
      }
    } else {
#pragma unroll
      for (int p = 0; p < kLd / 2; ++p) {
        int r, k;
        coord(2 * p, r, k);
        uint32_t* row = reinterpret_cast<uint32_t*>(T + r * LDK + k);  // k even: dword aligned
#pragma unroll
        for (int j = 0; j < 4; ++j) row[j * LDK / 2] = pack_bf16(v[2 * p][j], v[2 * p + 1][j]);
      }
    }
  }
};

template <bool AM, bool BN_>  // AM: A contiguous along m; BN_: B contiguous along n
__global__ __launch_bounds__(kThreadsG) void gemm_bf16_kernel(int M, int N, int K, const float* A,
                                                              int64_t sAm, int64_t sAk, const float* B,
                                                              int64_t sBk, int64_t sBn, const float* __restrict__ Cin,
                                                              int64_t ldCin, const float* __restrict__ bias,
                                                              float* __restrict__ C, int64_t ldC) {
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN * LDK];
  // XCD-aware tile order: grouped (kGroupM M-tiles x all N-tiles per group), and the workgroups
  // of XCD x (b % 8 == x) take the x-th contiguous eighth of that order when it divides evenly
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN, nt = ntm * ntn;
  int lt = blockIdx.x;
  if (nt % kXcd == 0) lt = (lt % kXcd) * (nt / kXcd) + lt / kXcd;
  const int gsz = kGroupM * ntn, g = lt / gsz, gm0 = g * kGroupM;
  const int gm = ntm - gm0 < kGroupM ? ntm - gm0 : kGroupM;
  const int tm = gm0 + (lt % gsz) % gm, tn = (lt % gsz) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x4g acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4g{0.f, 0.f, 0.f, 0.f};
  const int nk = (K + BK - 1) / BK;
  // register ring: slot s holds K tile t with t % kStages == s.  Tiles past the end re-read the
  // last one (in range, L2-resident) so every step issues the same loads.
  f32x4g ra[kStages][kLd], rb[kStages][kLd];  // native vectors: HIP's float4 struct blocks SROA here
  const Tile<AM> ta(A, sAm, sAk, M, K, m0);
  const Tile<BN_> tb(B, sBn, sBk, N, K, n0);  // B(k, j) as [n][k]: "row" = n
  auto issue = [&](int t, f32x4g (&a)[kLd], f32x4g (&b)[kLd]) {
    const int k0 = (t < nk ? t : nk - 1) * BK;
    ta.load(a, k0);
    tb.load(b, k0);
  };
  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < kStages; ++s) issue(s, ra[s], rb[s]);
  }
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  // one K step: tile t (register slot s) -> LDS buffer t & 1, refill the slot with tile
  // t + kStages, one barrier, 4 MFMAs per wave.  Buffer t & 1 is rewritten at step t + 2, after
  // every wave has passed step t + 1's barrier, i.e. finished step t's MFMAs.
  auto step = [&](int t, f32x4g (&a)[kLd], f32x4g (&b)[kLd], bool refill) {
    uint16_t* as = As[t & 1];
    uint16_t* bs = Bs[t & 1];
    // scheduling fence: otherwise the scheduler hoists every slot's bf16 conversion (it halves
    // the live registers) to the top of the ring round, which waits for ALL slots' loads there
    __builtin_amdgcn_sched_barrier(0);
    ta.store(a, as, t * BK);
    tb.store(b, bs, t * BK);
    if (refill) issue(t + kStages, a, b);
    __syncthreads();
#pragma unroll
    for (int kq = 0; kq < BK; kq += 32) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(as + (wm + 16 * i + fr) * LDK + kq + fk);
        bfr[i] = *reinterpret_cast<const bf16x8*>(bs + (wn + 16 * i + fr) * LDK + kq + fk);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // whole rounds of the ring: straight-line bodies, so the compiler's vmcnt waits only for the
  // oldest slot; then the < kStages remaining tiles without refills
  int t0 = 0;
  for (; t0 + kStages <= nk; t0 += kStages) {
#pragma unroll
    for (int s = 0; s < kStages; ++s) step(t0 + s, ra[s], rb[s], true);
  }
#pragma unroll
  for (int s = 0; s < kStages; ++s)
    if (t0 + s < nk) step(t0 + s, ra[s], rb[s], false);
  // epilogue: C layout col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + 16 * j + (lane & 15);
      if (col >= N) continue;
      const float b = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + (lane >> 4) * 4 + r;
        if (row < M) {
          float v = acc[i][j][r] + b;
          if (Cin) v += Cin[int64_t(row) * ldCin + col];
          C[int64_t(row) * ldC + col] = v;
        }
      }
    }
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_gemm_bf16(int32_t M, int32_t N, int32_t K, const float* A, int64_t sAm, int64_t sAk,
                               const float* B, int64_t sBk, int64_t sBn, const float* Cin, int64_t ldCin,
                               const float* bias, float* C, int64_t ldC, void* stream) {
  GASFM_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gasfm_gemm_bf16: M=%d N=%d K=%d", M, N, K);
  if (M == 0 || N == 0) return GASFM_OK;
  GASFM_REQUIRE(C && (K == 0 || (A && B)), "gasfm_gemm_bf16: null pointer");
  const bool am = K > 0 && sAm == 1, bn = K > 0 && sBn == 1;
  if (K > 0) {
    GASFM_REQUIRE((am || sAk == 1) && (bn || sBk == 1), "gasfm_gemm_bf16: A and B need a unit stride");
    // vector loads along the contiguous index: that extent and the other stride multiples of 4
    GASFM_REQUIRE((am ? M % 4 == 0 && sAk % 4 == 0 : K % 4 == 0 && sAm % 4 == 0) && aligned16(A),
                  "gasfm_gemm_bf16: A needs 16-byte aligned float4 runs along its contiguous index");
    GASFM_REQUIRE((bn ? N % 4 == 0 && sBk % 4 == 0 : K % 4 == 0 && sBn % 4 == 0) && aligned16(B),
                  "gasfm_gemm_bf16: B needs 16-byte aligned float4 runs along its contiguous index");
  }
  GASFM_REQUIRE(ldC >= N && (!Cin || ldCin >= N), "gasfm_gemm_bf16: ldC / ldCin < N");
  if (K > 0) {  // the kernel addresses A and B with int32 element offsets
    const int64_t spanA = int64_t(M - 1) * sAm + int64_t(K - 1) * sAk;
    const int64_t spanB = int64_t(K - 1) * sBk + int64_t(N - 1) * sBn;
    GASFM_REQUIRE(sAm >= 0 && sAk >= 0 && sBk >= 0 && sBn >= 0 && spanA < (int64_t(1) << 31) - 4 &&
                      spanB < (int64_t(1) << 31) - 4,
                  "gasfm_gemm_bf16: operands must span < 2^31 elements with non-negative strides");
  }
  const dim3 grid(((N + BN - 1) / BN) * ((M + BM - 1) / BM));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (am && bn)
    hipLaunchKernelGGL((gemm_bf16_kernel<true, true>), grid, dim3(kThreadsG), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  else if (am)
    hipLaunchKernelGGL((gemm_bf16_kernel<true, false>), grid, dim3(kThreadsG), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  else if (bn)
    hipLaunchKernelGGL((gemm_bf16_kernel<false, true>), grid, dim3(kThreadsG), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<false, false>), grid, dim3(kThreadsG), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  return launch_status("gasfm_gemm_bf16");
}
