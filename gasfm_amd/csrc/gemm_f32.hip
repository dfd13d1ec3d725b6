// fp32 MFMA GEMM with a fused epilogue for the camera-side D x D products, gfx950.
//
//   C[M,N] = A[M,K] . B[K,N] (+ Cin[M,N]) (+ bias[N])
//   A(i,k) = A[i*sAm + k*sAk], B(k,j) = B[k*sBk + j*sBn]: one of each pair must be 1 (the three
//   products of a Linear layer on row-major fp32 tensors: y = x W^T, dx = dy W, dW = dy^T x).
//
// The reference's Proj2View MLP and graph_conv_view2global.lin_l (code/models/layers.py:292-320,
// 352-358, 506-511) are m x 1024 x 1024 products: m = 1000 cameras on one GPU, m = 125 rows per
// rank when the camera rows are sharded over 8 GPUs (gasfm_amd/distributed.py).  hipBLASLt runs
// the 125-row product in 11.5 us (24 TF/s: 32 workgroups of 64 x 64 on a 256-CU chip); here:
//   - operands read as fp32 float4 runs along their contiguous index, staged through LDS
//     (rows padded to BK + 4 floats: the 16 x 4 fragment reads of a v_mfma_f32_16x16x4_f32 hit
//     64 distinct banks), a register ring of kStages K tiles in flight per thread;
//   - exact fp32 products on v_mfma_f32_16x16x4_f32 (same rounding as a k-ordered fma chain per
//     4-step), fp32 sums in a fixed order: deterministic;
//   - M x N <= 256k: 32 x 32 per workgroup with the K steps dealt round-robin to its 4 waves and
//     their four 32 x 32 partials summed in wave order through LDS at the end;
//   - larger (round 6, gemm_f32_d_kernel below): 64 x 64 per workgroup of 8 waves, operand tiles
//     global -> LDS directly (global_load_lds, XOR-swizzled images), 64-wide K chunks in a 3-deep
//     ring, one ds_read_b128 per four MFMA operands.  tools/gemm_bench.py at m = 1000 (MI355X,
//     back-to-back launches): 27.3 / 27.4 / 26.9 us for x W^T / dy W / dy^T x against the round-3
//     register-staged 64 x 64 kernel's 34.0 / 39.3 / 42.5 us and hipBLASLt's 25.9 / 25.2 / 27.9 us
//     (profiles/r6_gemm_f32.txt); hipBLASLt stays the model's default at m = 1000 (view_block.py);
//   - XCD-aware tile order as in gemm_bf16.hip.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int BK = 32, LDK = BK + 4, kThreadsF = 256, kStagesF = 3, kXcdF = 8, kGroupMF = 4;

typedef float f32x4f __attribute__((ext_vector_type(4)));

// One R x BK operand tile (rows row0 .., k0 ..): float4 runs along the contiguous index.
//   RowContig == false: k-contiguous, thread-float4 q -> row q / 8, k = 4 (q % 8)
//   RowContig == true:  row-contiguous, q -> rows 4 (q % (R/4)) .. +3, k = q / (R/4)
// Out-of-range float4s read a clamped in-range address and are zeroed when stored.
template <int R, bool RowContig>
struct TileF {
  static constexpr int kLd = R * BK / 4 / kThreadsF;
  const float* X;  // not __restrict__ (see gemm_bf16.hip: keeps the prefetch loads where they are)
  int s_k, K, kmax;
  int roff[kLd], kk[kLd];
  bool rok[kLd];
  __device__ __forceinline__ static void coord(int u, int& r, int& k) {
    const int q = threadIdx.x + kThreadsF * u;
    if constexpr (!RowContig) {
      r = q / (BK / 4);
      k = (q % (BK / 4)) * 4;
    } else {
      r = (q % (R / 4)) * 4;
      k = q / (R / 4);
    }
  }
  __device__ __forceinline__ TileF(const float* X_, int64_t s_row, int64_t s_k_, int rows, int K_, int row0)
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
  __device__ __forceinline__ void load(f32x4f (&v)[kLd], int k0) const {
#pragma unroll
    for (int u = 0; u < kLd; ++u) {
      const int k = k0 + kk[u] < kmax ? k0 + kk[u] : kmax;
      v[u] = *reinterpret_cast<const f32x4f*>(X + (roff[u] + k * s_k));
    }
  }
  __device__ __forceinline__ void store(f32x4f (&v)[kLd], float* __restrict__ T, int k0) const {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int u = 0; u < kLd; ++u) {  // mask instead of a branch (a branch would drain vmcnt)
      const uint32_t mk = (rok[u] && k0 + kk[u] < K) ? ~0u : 0u;
      v[u] = __builtin_bit_cast(f32x4f, __builtin_bit_cast(u32x4, v[u]) & mk);
      int r, k;
      coord(u, r, k);
      if constexpr (!RowContig) {
        *reinterpret_cast<f32x4f*>(T + r * LDK + k) = v[u];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) T[(r + j) * LDK + k] = v[u][j];
      }
    }
  }
};

// BM x BN tile per workgroup; 4 waves = (BM/32) x (BN/32) x KW, each accumulating 32 x 32 (2 x 2
// blocks of 16 x 16) over the K quads kq with kq % KW == its k-lane.
template <int BM, int BN, int KW, bool AM, bool BNC>
__global__ __launch_bounds__(kThreadsF) void gemm_f32_kernel(int M, int N, int K, const float* A, int64_t sAm,
                                                             int64_t sAk, const float* B, int64_t sBk, int64_t sBn,
                                                             const float* Cin, int64_t ldCin,
                                                             const float* __restrict__ bias, float* C, int64_t ldC) {
  static_assert((BM / 32) * (BN / 32) * KW == kThreadsF / 64, "4 waves per workgroup");
  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * LDK];
  float* const As0 = lds;                  // [2][BM * LDK]
  float* const Bs0 = lds + 2 * BM * LDK;   // [2][BN * LDK]
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN, nt = ntm * ntn;
  int lt = blockIdx.x;
  if (nt % kXcdF == 0) lt = (lt % kXcdF) * (nt / kXcdF) + lt / kXcdF;
  const int gsz = kGroupMF * ntn, g = lt / gsz, gm0 = g * kGroupMF;
  const int gm = ntm - gm0 < kGroupMF ? ntm - gm0 : kGroupMF;
  const int tm = gm0 + (lt % gsz) % gm, tn = (lt % gsz) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kw = wave % KW, wt = wave / KW;
  const int wm = (wt / (BN / 32)) * 32, wn = (wt % (BN / 32)) * 32;
  f32x4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4f{0.f, 0.f, 0.f, 0.f};
  using TA = TileF<BM, AM>;
  using TB = TileF<BN, BNC>;
  const int nk = (K + BK - 1) / BK;
  f32x4f ra[kStagesF][TA::kLd], rb[kStagesF][TB::kLd];
  const TA ta(A, sAm, sAk, M, K, m0);
  const TB tb(B, sBn, sBk, N, K, n0);  // B(k, j) as [n][k]
  auto issue = [&](int t, f32x4f (&a)[TA::kLd], f32x4f (&b)[TB::kLd]) {
    const int k0 = (t < nk ? t : nk - 1) * BK;
    ta.load(a, k0);
    tb.load(b, k0);
  };
  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < kStagesF; ++s) issue(s, ra[s], rb[s]);
  }
  const int fr = lane & 15, fq = lane >> 4;
  auto step = [&](int t, f32x4f (&a)[TA::kLd], f32x4f (&b)[TB::kLd], bool refill) {
    float* as = As0 + (t & 1) * BM * LDK;
    float* bs = Bs0 + (t & 1) * BN * LDK;
    __builtin_amdgcn_sched_barrier(0);
    ta.store(a, as, t * BK);
    tb.store(b, bs, t * BK);
    if (refill) issue(t + kStagesF, a, b);
    __syncthreads();
#pragma unroll
    for (int kq = kw; kq < BK / 4; kq += KW) {
      float af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = as[(wm + 16 * i + fr) * LDK + 4 * kq + fq];
        bf[i] = bs[(wn + 16 * i + fr) * LDK + 4 * kq + fq];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };
  int t0 = 0;
  for (; t0 + kStagesF <= nk; t0 += kStagesF) {
#pragma unroll
    for (int s = 0; s < kStagesF; ++s) step(t0 + s, ra[s], rb[s], true);
  }
#pragma unroll
  for (int s = 0; s < kStagesF; ++s)
    if (t0 + s < nk) step(t0 + s, ra[s], rb[s], false);
  if constexpr (KW > 1) {
    // the KW k-lane partials of each 32 x 32 block, summed in k-lane order through LDS (free
    // after the last step's barrier; (KW - 1) partials x 64 lanes x 16 floats)
    __syncthreads();
    float* red = lds;
    static_assert((KW - 1) * 64 * 16 <= 2 * (BM + BN) * LDK, "reduction scratch");
    if (kw > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[((kw - 1) * 16 + (i * 2 + j) * 4 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int q = 1; q < KW; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += red[((q - 1) * 16 + (i * 2 + j) * 4 + r) * 64 + lane];
  }
  // epilogue: C layout col = lane & 15, row = (lane >> 4) * 4 + r (Cin may alias C: each
  // element is read, then written, by the same lane)
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

// The large-tile path (M x N > 256k: the m = 1000 camera products; round 6).  64 x 64 per
// workgroup of NWV = 8 waves: wave w owns the 32 x 32 quadrant w % 4 and the k split w / 4 of every
// chunk (the two waves of a quadrant share a SIMD); the splits are summed through LDS at the end.
// The operand tiles go global -> LDS with global_load_lds
// (16 B per lane, no VGPR staging, no ds_write), in a ring of DS stages (DS - 1 K chunks in flight),
// one barrier per chunk.  The lanes' load order is the LDS image, so the layouts are chosen by
// which global 16-byte chunk each lane fetches:
//   k-contiguous operand (x, W of x W^T): [64 rows][8 chunks of 4 k], chunk kc of row r at slot
//     kc ^ (r & 7) (8 consecutive rows' b128 reads of one kc hit 8 distinct bank quads); a lane's
//     four k of a 16x16x4 quad step are ONE ds_read_b128 (k = 8 fq + 4 kh + t as in the q kernel);
//   row-contiguous operand (W of dy W, dy^T of dy^T x): [32 k][16 chunks of 4 rows], chunk c of
//     k row kr at slot c ^ (((kr >> 3) & 1) << 2) (the two k rows 8 apart that lanes 0-15 and
//     16-31 read in one pass land 16 banks apart); one ds_read_b32 per MFMA operand.
template <bool AM, bool BNC, int DS, int KB, int NWV>
__global__ __launch_bounds__(64 * NWV) void gemm_f32_d_kernel(int M, int N, int K, const float* A, int64_t sAm,
                                                         int64_t sAk, const float* B, int64_t sBk, int64_t sBn,
                                                         const float* Cin, int64_t ldCin,
                                                         const float* __restrict__ bias, float* C, int64_t ldC) {
  typedef __attribute__((address_space(3))) void* lds_vp;
  typedef const __attribute__((address_space(1))) void* glb_vp;
  constexpr int BM = 64, BN = 64, TILE = 64 * KB;  // floats per operand tile
  constexpr int CPR = KB / 4, NL = KB * 16 / (NWV * 64);  // 16-B chunks per k row; loads per operand per wave
  constexpr int KS = NWV / 4, NH = KB / (16 * KS);  // k splits (waves per quadrant); 16-wide k groups per wave
  constexpr int SW = KB / 4;  // k distance between the lanes fq and fq + 1 (row-contiguous swizzle bit)
  __shared__ __attribute__((aligned(16))) float lds[DS * 2 * TILE];
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN, nt = ntm * ntn;
  int lt = blockIdx.x;
  if (nt % kXcdF == 0) lt = (lt % kXcdF) * (nt / kXcdF) + lt / kXcdF;
  const int gsz = kGroupMF * ntn, g = lt / gsz, gm0 = g * kGroupMF;
  const int gm = ntm - gm0 < kGroupMF ? ntm - gm0 : kGroupMF;
  const int tm = gm0 + (lt % gsz) % gm, tn = (lt % gsz) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kh = wave >> 2, q = wave & 3;  // k split, quadrant
  const int wm = (q >> 1) * 32, wn = (q & 1) * 32;
  // this lane's fetch: (tile row, k offset within the chunk) of the 16 bytes it loads, per operand
  // load l (0 .. NL - 1) of this lane: (tile row, k offset within the chunk) of its 16 bytes
  auto coords = [&](bool rowc, int l, int& r, int& k) {
    if (!rowc) {  // k-contiguous: [64 rows][CPR slots], slot holds chunk slot ^ (row & 7)
      const int idx = (wave * NL + l) * 64 + lane;
      r = idx / CPR;
      k = 4 * ((idx % CPR) ^ (r & 7));
    } else {      // row-contiguous: [KB k rows][16 slots of 4 rows], slot holds chunk slot ^ swz(k)
      const int idx = (wave * NL + l) * 64 + lane;
      k = idx / 16;
      r = 4 * ((idx % 16) ^ (((k / SW) & 1) << 2));
    }
  };
  int ra[NL], ka[NL], rb[NL], kb[NL];
  int64_t aoff[NL], boff[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    coords(AM, l, ra[l], ka[l]);
    coords(BNC, l, rb[l], kb[l]);
    // out-of-range rows / k read a clamped in-range address: their products only reach C entries
    // that are never stored (rows >= M, cols >= N) or multiply a zeroed partner (k >= K, below)
    aoff[l] = int64_t(m0 + ra[l] < M ? m0 + ra[l] : M - (AM ? 4 : 1)) * sAm;
    boff[l] = int64_t(n0 + rb[l] < N ? n0 + rb[l] : N - (BNC ? 4 : 1)) * sBn;
  }
  const int kmaxA = AM ? K - 1 : K - 4, kmaxB = BNC ? K - 1 : K - 4;
  const int nk = (K + KB - 1) / KB;
  auto issue = [&](int t) {
    const int tt = t < nk ? t : nk - 1;  // past the end: re-read the last chunk (never consumed)
    const int k0 = tt * KB;
    float* sa = lds + (t % DS) * 2 * TILE;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int kA = k0 + ka[l] < kmaxA ? k0 + ka[l] : kmaxA, kB = k0 + kb[l] < kmaxB ? k0 + kb[l] : kmaxB;
      __builtin_amdgcn_global_load_lds((glb_vp)(A + (aoff[l] + int64_t(kA) * sAk)),
                                       (lds_vp)(sa + (wave * NL + l) * 256), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((glb_vp)(B + (boff[l] + int64_t(kB) * sBk)),
                                       (lds_vp)(sa + TILE + (wave * NL + l) * 256), 16, 0, 0);
    }
  };
  f32x4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < DS - 1; ++s) issue(s);
  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    // chunk t landed for this wave (DS - 2 younger chunks may still fly), then for every wave
    // (a bare s_barrier: __syncthreads' release fence would add vmcnt(0), draining the ring)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NL * (DS - 2)) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + DS - 1);  // into the slot chunk t - 1 used: every wave is past it (the barrier)
    const float* sa = lds + (t % DS) * 2 * TILE;
    const float* sb = sa + TILE;
    const bool kdead = (t + 1) * KB > K;  // the last chunk of a K that is not a multiple of KB
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int kc = NH * (KS * fq + kh) + h;  // this lane's k chunk
      f32x4f af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm + 16 * i + fr;
        if constexpr (!AM) {
          af[i] = *reinterpret_cast<const f32x4f*>(sa + r * KB + 4 * (kc ^ (r & 7)));
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kr = 4 * kc + u;
            af[i][u] = sa[kr * 64 + 4 * ((r >> 2) ^ (((kr / SW) & 1) << 2)) + (r & 3)];
          }
        }
        const int c = wn + 16 * i + fr;
        if constexpr (!BNC) {
          bf[i] = *reinterpret_cast<const f32x4f*>(sb + c * KB + 4 * (kc ^ (c & 7)));
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kr = 4 * kc + u;
            bf[i][u] = sb[kr * 64 + 4 * ((c >> 2) ^ (((kr / SW) & 1) << 2)) + (c & 3)];
          }
        }
      }
      if (kdead) {  // zero A's k >= K (clamped reads hold real values)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = t * KB + 4 * kc + u < K;
#pragma unroll
          for (int i = 0; i < 2; ++i) af[i][u] = ok ? af[i][u] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][u], bf[j][u], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-read chunks past the end
  __syncthreads();
  // the KS k splits of each quadrant, summed in split order through LDS (free after the loop)
  if (kh > 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) lds[(((kh - 1) * 4 + q) * 16 + (i * 2 + j) * 4 + r) * 64 + lane] = acc[i][j][r];
  }
  __syncthreads();
  if (kh > 0) return;
#pragma unroll
  for (int x = 1; x < KS; ++x)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += lds[(((x - 1) * 4 + q) * 16 + (i * 2 + j) * 4 + r) * 64 + lane];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + 16 * j + (lane & 15);
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + (lane >> 4) * 4 + r;
        if (row < M) {
          float v = acc[i][j][r] + bv;
          if (Cin) v += Cin[int64_t(row) * ldCin + col];
          C[int64_t(row) * ldC + col] = v;
        }
      }
    }
}

template <int DS, int KB, int NWV>
void launch_f32_d(bool am, bool bn, int M, int N, int K, const float* A, int64_t sAm, int64_t sAk, const float* B,
                  int64_t sBk, int64_t sBn, const float* Cin, int64_t ldCin, const float* bias, float* C,
                  int64_t ldC, hipStream_t st) {
  const dim3 grid(((N + 63) / 64) * ((M + 63) / 64));
  if (am && bn)
    hipLaunchKernelGGL((gemm_f32_d_kernel<true, true, DS, KB, NWV>), grid, dim3(64 * NWV), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  else if (am)
    hipLaunchKernelGGL((gemm_f32_d_kernel<true, false, DS, KB, NWV>), grid, dim3(64 * NWV), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  else if (bn)
    hipLaunchKernelGGL((gemm_f32_d_kernel<false, true, DS, KB, NWV>), grid, dim3(64 * NWV), 0, st, M, N, K, A, sAm, sAk, B, sBk,
                       sBn, Cin, ldCin, bias, C, ldC);
  else
    hipLaunchKernelGGL((gemm_f32_d_kernel<false, false, DS, KB, NWV>), grid, dim3(64 * NWV), 0, st, M, N, K, A, sAm, sAk, B,
                       sBk, sBn, Cin, ldCin, bias, C, ldC);
}

template <int BM, int BN, int KW>
void launch_f32(bool am, bool bn, int M, int N, int K, const float* A, int64_t sAm, int64_t sAk, const float* B,
                int64_t sBk, int64_t sBn, const float* Cin, int64_t ldCin, const float* bias, float* C, int64_t ldC,
                hipStream_t st) {
  const dim3 grid(((N + BN - 1) / BN) * ((M + BM - 1) / BM));
  if (am && bn)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, KW, true, true>), grid, dim3(kThreadsF), 0, st, M, N, K, A, sAm, sAk,
                       B, sBk, sBn, Cin, ldCin, bias, C, ldC);
  else if (am)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, KW, true, false>), grid, dim3(kThreadsF), 0, st, M, N, K, A, sAm,
                       sAk, B, sBk, sBn, Cin, ldCin, bias, C, ldC);
  else if (bn)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, KW, false, true>), grid, dim3(kThreadsF), 0, st, M, N, K, A, sAm,
                       sAk, B, sBk, sBn, Cin, ldCin, bias, C, ldC);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, KW, false, false>), grid, dim3(kThreadsF), 0, st, M, N, K, A, sAm,
                       sAk, B, sBk, sBn, Cin, ldCin, bias, C, ldC);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_gemm_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t sAm, int64_t sAk,
                              const float* B, int64_t sBk, int64_t sBn, const float* Cin, int64_t ldCin,
                              const float* bias, float* C, int64_t ldC, void* stream) {
  GASFM_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gasfm_gemm_f32: M=%d N=%d K=%d", M, N, K);
  if (M == 0 || N == 0) return GASFM_OK;
  GASFM_REQUIRE(C && (K == 0 || (A && B)), "gasfm_gemm_f32: null pointer");
  const bool am = K > 0 && sAm == 1, bn = K > 0 && sBn == 1;
  if (K > 0) {
    GASFM_REQUIRE((am || sAk == 1) && (bn || sBk == 1), "gasfm_gemm_f32: A and B need a unit stride");
    GASFM_REQUIRE((am ? M % 4 == 0 && sAk % 4 == 0 : K % 4 == 0 && sAm % 4 == 0) && aligned16(A),
                  "gasfm_gemm_f32: A needs 16-byte aligned float4 runs along its contiguous index");
    GASFM_REQUIRE((bn ? N % 4 == 0 && sBk % 4 == 0 : K % 4 == 0 && sBn % 4 == 0) && aligned16(B),
                  "gasfm_gemm_f32: B needs 16-byte aligned float4 runs along its contiguous index");
    const int64_t spanA = int64_t(M - 1) * sAm + int64_t(K - 1) * sAk;
    const int64_t spanB = int64_t(K - 1) * sBk + int64_t(N - 1) * sBn;
    GASFM_REQUIRE(sAm >= 0 && sAk >= 0 && sBk >= 0 && sBn >= 0 && spanA < (int64_t(1) << 31) - 4 &&
                      spanB < (int64_t(1) << 31) - 4,
                  "gasfm_gemm_f32: operands must span < 2^31 elements with non-negative strides");
  }
  GASFM_REQUIRE(ldC >= N && (!Cin || ldCin >= N), "gasfm_gemm_f32: ldC / ldCin < N");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (int64_t(M) * N <= 256 * 1024)  // e.g. a camera shard's 125 x 1024: the 32 x 32, K-split tile
    launch_f32<32, 32, 4>(am, bn, M, N, K, A, sAm, sAk, B, sBk, sBn, Cin, ldCin, bias, C, ldC, st);
  else
    launch_f32_d<3, 64, 8>(am, bn, M, N, K, A, sAm, sAk, B, sBk, sBn, Cin, ldCin, bias, C, ldC, st);
  return launch_status("gasfm_gemm_f32");
}
