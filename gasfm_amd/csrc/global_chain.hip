// hipcc-flags: -mllvm --amdgpu-sched-strategy=max-ilp
// (round 6: the rank-0-of-8 proxy 7.19-7.20 -> 7.16 ms on one box, profiles/r6_ab_sched_files.txt; the
// other kernel files measured within noise or slower under max-ilp)
// The global node's chain of one GASFM block -- a single row of G = 2048 features -- forward and
// backward in four launches each way, gfx950.
//
// Per block (code/models/layers.py):
//   F1  x1  = W1 xcat + b1 (+ prev)              proj_view_and_scenepoint2global + skip  :527-528, 590-592
//   F2  g   = x1 + W2 relu(LN_M(x1)) + b2        norm_pre_mlp, mlp, skip                 :594-603
//   F3  SG  = WA relu(LN_A(g))                   lin_global of the projection update      :928-935
//       xv  = WB relu(LN_B(g)) + bWB             next block's norm_and_proj_global2view   :497-505
//       xp  = WC relu(LN_C(g)) + bWC             next block's norm_and_proj_global2scenepoint :512-520
//   F4  XRv = WD xv + bD,  XRp = WE xp + bE      the next block's two GATv2 lin_r rows (PyG)
// (the last block's chain ends at F3 with SG only).  BASELINE config 5 (round 5): with bf16 weight
// shadows (gasfm_gchain.W*h) every GEMV streams half the weight bytes (fp32 accumulation; the
// weight gradients stay fp32: dW = dy x h reads no weight).  Round 3 ran this as gvec launches with a
// one-workgroup "finish" kernel after every backward GEMV (12 launches per block, ~100 us); here:
//
//   gnode_fwd   one wave per output row; the wave's W row is requested FIRST, into registers,
//               and the workgroup's LayerNorm of the input row (recomputed by every workgroup)
//               runs while it is in flight.
//   gnode_bwd   a workgroup per (problem, 32-column slab of K, chunk of 32*RPT rows of N):
//                 dW[rows, slab] = dy[rows] (x) h[slab]   (h = relu(LN(x)) or x)
//                 dh[slab]       = sum over rows of dy[n] W[n, slab]
//               chunk partials of dh are handed to the slab's last-arriving workgroup (write-
//               through stores, one relaxed agent-scope ticket per slab: reduce.hip's hand-off),
//               which sums them in chunk order: dh leaves FINAL, no finish launch.  The LayerNorm
//               backward that follows a level (F3's LN_A/B/C into dg, F2's LN_M into dx1) is split
//               by where its operands are: the slab's last arriver, holding the final dh of its 32
//               columns, writes gv = relu'(.) gamma dh, the gamma / beta gradients of those columns
//               and their two row-sum partials (sum gv, sum gv xh); the NEXT level's workgroups sum
//               the partials in slab order (the same order in every workgroup) and finish dy for
//               their own chunk of rows in a prologue that overlaps their W slab loads.  No
//               launch-wide ticket and no one-workgroup tail (round 4's first version ran the
//               LayerNorm backward in the level's last workgroup: ~9 us of the 18 us B2 / B3).
//   Every phase issues all of its global loads before the first use (clamped addresses): a load
//   behind a branch or behind a store to a possibly-aliasing pointer costs a full round trip.
// No float atomics; every sum has a fixed order: deterministic, identical on every rank.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kFT = 256;              // forward: 4 waves, one output row each
constexpr int kBT = 256;              // backward: 8 float4 column lanes x 32 row lanes
constexpr int kSW = 32;               // backward slab width (columns of K)
constexpr int kMaxK = 2048;           // widest row (G)
constexpr int kPer = kMaxK / 256;     // row values per thread in the full-row prologues
constexpr int kMaxProb = 3;
constexpr int kMaxRaw = 3;
constexpr int kMaxRows = GASFM_GCHAIN_MAX_ROWS;  // global rows of a union batch per launch

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// NV sums over a 256-thread workgroup in one barrier round, fixed order; results to every thread
template <int NV>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[wave * NV + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = scratch[k] + scratch[NV + k] + scratch[2 * NV + k] + scratch[3 * NV + k];
}

// 4 consecutive weights from the bf16 shadow (8-byte load) or the fp32 row (16-byte load)
template <bool BF>
__device__ __forceinline__ float4 w4(const float* W, const uint16_t* Wh, int64_t off) {
  if (BF) {
    const uint2 t = *reinterpret_cast<const uint2*>(Wh + off);
    return make_float4(__uint_as_float(t.x << 16), __uint_as_float(t.x & 0xffff0000u), __uint_as_float(t.y << 16),
                       __uint_as_float(t.y & 0xffff0000u));
  }
  return *reinterpret_cast<const float4*>(W + off);
}

// mean / rstd of a row held as kPer strided values per thread (j = tid + 256 u; 0 past K)
__device__ __forceinline__ void row_stats(const float (&xv)[kPer], int K, float eps, float* scratch, float& mean,
                                          float& rstd) {
  float s[1] = {0.f};
#pragma unroll
  for (int u = 0; u < kPer; ++u) s[0] += xv[u];
  block_sums<1>(s, scratch);
  mean = s[0] / K;
  float q[1] = {0.f};
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int j = int(threadIdx.x) + 256 * u;
    const float d = j < K ? xv[u] - mean : 0.f;
    q[0] = fmaf(d, d, q[0]);
  }
  block_sums<1>(q, scratch);
  rstd = rsq_normal(q[0] / K + eps);
}

__device__ __forceinline__ void load_row(const float* __restrict__ x, int K, float (&xv)[kPer]) {
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int j = int(threadIdx.x) + 256 * u;
    xv[u] = j < K ? x[j] : 0.f;
  }
}

template <int NP>
__device__ __forceinline__ int find_prob(const int (&blk0)[NP], int nprob) {
  int pi = 0;
  while (pi + 1 < nprob && int(blockIdx.x) >= blk0[pi + 1]) ++pi;
  return pi;
}

// ---------------------------------------------------------------------------------- forward
struct GnFwdProb {
  const float* x;    // [K] input row
  const float* gam;  // [K] LayerNorm (null: h = x)
  const float* bet;
  const float* W;    // [N, K]
  const float* b;    // [N] or null
  const float* res;  // [N] or null
  float* y;          // [N]
  int K, N, blk0;
  float eps;
  const uint16_t* Wh;  // bf16 shadow of W (null: W)
  int rows;            // rows of x / res / y ([rows, K], [rows, N], [rows, N]); 1 for the one-scene chain
};
struct GnFwdArgs {
  GnFwdProb p[kMaxProb];
  int nprob;
};

// R: the rows of a union batch's global nodes (one per scene, batch.SceneBatch / static_batch), up
// to R per launch (p.rows of them); each workgroup streams its W rows once for all of them.
template <int KI, bool BF, int R>  // float4 per lane of a W row: K <= 256 KI; BF: the bf16 shadows (every problem's)
__global__ __launch_bounds__(kFT) void gnode_fwd_kernel(GnFwdArgs a) {
  __shared__ __attribute__((aligned(16))) float h[kMaxK];
  __shared__ float scratch[8];
  int blk0[kMaxProb];
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) blk0[q] = a.p[q].blk0;
  const GnFwdProb& p = a.p[find_prob(blk0, a.nprob)];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = p.K;
  const int rows = R == 1 ? 1 : p.rows;
  const int i = (int(blockIdx.x) - p.blk0) * (kFT / 64) + wave;
  const int ic = i < p.N ? i : p.N - 1;
  // every load of the kernel first: the wave's W row, the input row and its LayerNorm affine
  // (clamped in-range addresses; values past K are zeroed where consumed)
  float4 w[KI];
#pragma unroll
  for (int u = 0; u < KI; ++u) {
    const int j = 4 * lane + 256 * u;
    w[u] = w4<BF>(p.W, p.Wh, int64_t(ic) * K + (j < K ? j : 0));
  }
  const bool ln = p.gam != nullptr;
  const float* gp = ln ? p.gam : p.x;
  const float* bp = ln ? p.bet : p.x;
  float xv[kPer], gv[kPer], bv[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int j = int(threadIdx.x) + 256 * u, jc = j < K ? j : 0;
    xv[u] = p.x[jc];
    gv[u] = gp[jc];
    bv[u] = bp[jc];
  }
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = 0.f;
    if (r >= rows) continue;  // uniform
    if (r > 0) {
      __syncthreads();  // row r - 1's h consumed
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int j = int(threadIdx.x) + 256 * u;
        xv[u] = p.x[int64_t(r) * K + (j < K ? j : 0)];
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u)
      if (int(threadIdx.x) + 256 * u >= K) xv[u] = 0.f;
    if (ln) {
      float mean, rstd;
      row_stats(xv, K, p.eps, scratch, mean, rstd);
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int j = int(threadIdx.x) + 256 * u;
        h[j] = j < K ? fmaxf(fmaf((xv[u] - mean) * rstd, gv[u], bv[u]), 0.f) : 0.f;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kPer; ++u) h[int(threadIdx.x) + 256 * u] = xv[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KI; ++u) {
      const int j = 4 * lane + 256 * u;
      if (j < kMaxK) {
        const float4 hv = *reinterpret_cast<const float4*>(h + j);  // 0 past K
        acc[r] = fmaf(w[u].x, hv.x, fmaf(w[u].y, hv.y, fmaf(w[u].z, hv.z, fmaf(w[u].w, hv.w, acc[r]))));
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r >= rows) continue;
    const float v = wave_sum(acc[r]);
    if (lane == 0 && i < p.N)
      p.y[int64_t(r) * p.N + i] = v + (p.b ? p.b[i] : 0.f) + (p.res ? p.res[int64_t(r) * p.N + i] : 0.f);
  }
}

int launch_fwd(GnFwdArgs& a, hipStream_t st) {
  int blocks = 0, kmax = 0;
  for (int q = 0; q < a.nprob; ++q) {
    a.p[q].blk0 = blocks;
    blocks += (a.p[q].N + 3) / 4;
    kmax = a.p[q].K > kmax ? a.p[q].K : kmax;
  }
  for (int q = a.nprob; q < kMaxProb; ++q) a.p[q].blk0 = blocks;
  bool bf = true;  // the bf16 kernels when every problem has its shadow (no per-load branch)
  for (int q = 0; q < a.nprob; ++q) bf = bf && a.p[q].Wh != nullptr;
  const int rows = a.p[0].rows;
  auto go = [&](auto k32, auto k16, auto m32, auto m16) {
    const auto kern = rows > 1 ? (bf ? m16 : m32) : (bf ? k16 : k32);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kFT), 0, st, a);
  };
  constexpr int RM = kMaxRows;
  if (kmax <= 256)
    go(&gnode_fwd_kernel<1, false, 1>, &gnode_fwd_kernel<1, true, 1>, &gnode_fwd_kernel<1, false, RM>,
       &gnode_fwd_kernel<1, true, RM>);
  else if (kmax <= 1024)
    go(&gnode_fwd_kernel<4, false, 1>, &gnode_fwd_kernel<4, true, 1>, &gnode_fwd_kernel<4, false, RM>,
       &gnode_fwd_kernel<4, true, RM>);
  else if (kmax <= 1280)
    go(&gnode_fwd_kernel<5, false, 1>, &gnode_fwd_kernel<5, true, 1>, &gnode_fwd_kernel<5, false, RM>,
       &gnode_fwd_kernel<5, true, RM>);
  else
    go(&gnode_fwd_kernel<8, false, 1>, &gnode_fwd_kernel<8, true, 1>, &gnode_fwd_kernel<8, false, RM>,
       &gnode_fwd_kernel<8, true, RM>);
  return launch_status("gasfm_gchain_fwd");
}

// --------------------------------------------------------------------------------- backward
struct GnBwdProb {
  const float* dy;   // [N] output gradient (final; unused when the launch has a prologue)
  const float* x;    // [K] forward input row
  const float* gam;  // [K] LayerNorm of x (null: h = x)
  const float* bet;
  const float* W;    // [N, K]
  float* dW;         // [N, K]
  float* db;         // [N] or null (= dy, written by the slab-0 workgroups)
  float* dh;         // [K] W^T dy, or with lnfin gv = relu'(.) gam (W^T dy) (final)
  float* ws;         // [chunks, K] chunk partials
  uint32_t* cnt;     // [slabs] self-resetting tickets
  int K, N, blk0, slabs, chunks;
  float eps;
  // lnfin: the slab's last arriver also runs its columns' share of the LayerNorm backward of x:
  // gv (into dh), dgam / dbet, and the two row-sum partials (sum gv, sum gv xh) into lnp[slab]
  float* dgam;
  float* dbet;
  float* lnp;        // [slabs][2]
  float* stats;      // (mean, rstd) of x, written by slab 0 (null: not needed)
  int lnfin;
  const uint16_t* Wh;  // bf16 shadow of W (null: W)
  // rows > 1 (a union batch's global nodes): dy / x / dh are [rows, N] / [rows, K] / [rows, K],
  // ws [chunks, rows, K], lnp [rows, slabs, 2], stats [rows, 2]; dW, db, dgam, dbet sum the rows
  int rows;
};
// The launch's prologue (the previous level's LayerNorm backward, finished per row here):
//   dy[n] = dres[n] + sum_q rstd (gv_q[n] - S1_q / F - xh[n] S2_q / F),  xh = (x - mean) rstd,
//   S1_q / S2_q = the previous level's lnp rows summed in slab order (same order in every workgroup)
struct GnPro {
  const float* gv[kMaxRaw];
  const float* lnp[kMaxRaw];
  const float* stats;  // (mean, rstd) of x
  const float* x;
  const float* dres;   // or null
  float* out;          // or null: dy rows written by the slab-0 workgroups (d prev)
  int nq, F, slabs;     // rows > 1: gv / x / dres / out are [rows, F], lnp [rows, slabs, 2], stats [rows, 2]
};
struct GnBwdArgs {
  GnBwdProb p[kMaxProb];
  GnPro pro;
  int nprob;
};

__device__ __forceinline__ void st_sc1(float* p, float4 v) {
  uint64_t a, b;
  __builtin_memcpy(&a, &v.x, 8);
  __builtin_memcpy(&b, &v.z, 8);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p) + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int RPT, bool BF, int R>  // rows per thread: a chunk is 32 RPT rows; BF: the bf16 shadows;
                                     // R: global rows per launch (p.rows of them)
__global__ __launch_bounds__(kBT) void gnode_bwd_kernel(GnBwdArgs a) {
  static_assert(32 * RPT == kBT, "one dy row per thread");
  __shared__ float dys[R][32 * RPT];
  __shared__ float4 red[kBT];
  __shared__ float scratch[4 * 2 * kMaxRaw * R + 8];
  __shared__ uint32_t flag;
  int blk0[kMaxProb];
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) blk0[q] = a.p[q].blk0;
  const int pi = find_prob(blk0, a.nprob);
  const GnBwdProb& p = a.p[pi];
  const int rows = R == 1 ? 1 : p.rows;
  const int local = int(blockIdx.x) - p.blk0;
  const int slab = local % p.slabs, chunk = local / p.slabs;
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int K = p.K, N = p.N;
  const int col = slab * kSW + 4 * cl;
  const int row0 = chunk * 32 * RPT;
  const int nrow = row0 + int(threadIdx.x), nrc = nrow < N ? nrow : N - 1;  // this thread's dy row
  const GnPro& pr = a.pro;
  const bool pro = pr.nq > 0;
  // 1. every load first: the prologue's operands (they gate dy), the workgroup's W slab rows, the
  // input rows (+ affine)
  float dres[R], xr[R], gvr[R][kMaxRaw], lp[R * 2 * kMaxRaw], st0[R], st1[R], dyv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    dres[r] = xr[r] = st0[r] = st1[r] = dyv[r] = 0.f;
#pragma unroll
    for (int q = 0; q < kMaxRaw; ++q) {
      gvr[r][q] = 0.f;
      lp[(r * kMaxRaw + q) * 2] = lp[(r * kMaxRaw + q) * 2 + 1] = 0.f;
    }
    if (r >= rows) continue;
    if (pro) {
      const int64_t ro = int64_t(r) * pr.F;
      dres[r] = pr.dres ? pr.dres[ro + nrc] : 0.f;
      xr[r] = pr.x[ro + nrc];
      st0[r] = pr.stats[2 * r];
      st1[r] = pr.stats[2 * r + 1];
      const int tc = int(threadIdx.x) < pr.slabs ? int(threadIdx.x) : 0;
#pragma unroll
      for (int q = 0; q < kMaxRaw; ++q) {
        const bool on = q < pr.nq;
        gvr[r][q] = on ? pr.gv[q][ro + nrc] : 0.f;
        const int64_t lo = (int64_t(r) * pr.slabs + tc) * 2;
        lp[(r * kMaxRaw + q) * 2] = on ? pr.lnp[q][lo] : 0.f;
        lp[(r * kMaxRaw + q) * 2 + 1] = on ? pr.lnp[q][lo + 1] : 0.f;
      }
    } else {
      dyv[r] = p.dy[int64_t(r) * N + nrc];
    }
  }
  float4 w[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int n = row0 + rl + 32 * k;
    w[k] = w4<BF>(p.W, p.Wh, int64_t(n < N ? n : N - 1) * K + col);
  }
  float4 x4[R];
#pragma unroll
  for (int r = 0; r < R; ++r) x4[r] = *reinterpret_cast<const float4*>(p.x + int64_t(r < rows ? r : 0) * K + col);
  const bool ln = p.gam != nullptr;
  float4 g4 = x4[0], b4 = x4[0];
  float xv[kPer];
  if (ln) {
    g4 = *reinterpret_cast<const float4*>(p.gam + col);
    b4 = *reinterpret_cast<const float4*>(p.bet + col);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int j = int(threadIdx.x) + 256 * u;
      xv[u] = p.x[j < K ? j : 0];
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u)
      if (int(threadIdx.x) + 256 * u >= K) xv[u] = 0.f;
  }
  // 2. dy of the chunk's rows
  if (pro) {
    if (int(threadIdx.x) >= pr.slabs) {
#pragma unroll
      for (int k = 0; k < R * 2 * kMaxRaw; ++k) lp[k] = 0.f;
    }
    block_sums<R * 2 * kMaxRaw>(lp, scratch);
    const float invF = 1.f / pr.F;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r >= rows) continue;
      const float xh = (xr[r] - st0[r]) * st1[r];
      float d = dres[r];
#pragma unroll
      for (int q = 0; q < kMaxRaw; ++q)
        if (q < pr.nq)
          d += st1[r] * (gvr[r][q] - lp[(r * kMaxRaw + q) * 2] * invF - xh * lp[(r * kMaxRaw + q) * 2 + 1] * invF);
      dyv[r] = d;
      if (slab == 0 && pr.out && nrow < N) pr.out[int64_t(r) * pr.F + nrow] = d;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) dys[r][threadIdx.x] = (nrow < N && r < rows) ? dyv[r] : 0.f;
  // 3. h over the thread's 4 slab columns, per row
  float4 h4[R], xh4[R];
  float mean[R], rstd[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    h4[r] = xh4[r] = x4[r];
    mean[r] = rstd[r] = 0.f;
    if (ln && r < rows) {
      if (r > 0) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
          const int j = int(threadIdx.x) + 256 * u;
          xv[u] = j < K ? p.x[int64_t(r) * K + j] : 0.f;
        }
      }
      __syncthreads();  // the prologue's / the previous row's block_sums scratch before row_stats reuses it
      row_stats(xv, K, p.eps, scratch, mean[r], rstd[r]);
      const float4 xx = x4[r];
      xh4[r] = make_float4((xx.x - mean[r]) * rstd[r], (xx.y - mean[r]) * rstd[r], (xx.z - mean[r]) * rstd[r],
                           (xx.w - mean[r]) * rstd[r]);
      h4[r] = make_float4(fmaxf(fmaf(xh4[r].x, g4.x, b4.x), 0.f), fmaxf(fmaf(xh4[r].y, g4.y, b4.y), 0.f),
                          fmaxf(fmaf(xh4[r].z, g4.z, b4.z), 0.f), fmaxf(fmaf(xh4[r].w, g4.w, b4.w), 0.f));
    }
  }
  __syncthreads();  // dys
  auto store_dw = [&]() {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int n = row0 + rl + 32 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= rows) continue;
        const float d = dys[r][rl + 32 * k];
        v.x = fmaf(d, h4[r].x, v.x);
        v.y = fmaf(d, h4[r].y, v.y);
        v.z = fmaf(d, h4[r].z, v.z);
        v.w = fmaf(d, h4[r].w, v.w);
      }
      if (n < N) *reinterpret_cast<float4*>(p.dW + int64_t(n) * K + col) = v;
    }
    if (p.db && slab == 0 && nrow < N) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (r < rows) v += dys[r][threadIdx.x];
      p.db[nrow] = v;
    }
  };
  // 4. + 5. this thread's share of dh per row (the dW rows are stored last: a ticket's s_waitcnt
  // vmcnt(0) would otherwise wait for them too), the 32 row lanes summed in lane order
  float4 tot[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    tot[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r >= rows) continue;
    float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const float d = dys[r][rl + 32 * k];  // 0 past N
      sv.x = fmaf(d, w[k].x, sv.x);
      sv.y = fmaf(d, w[k].y, sv.y);
      sv.z = fmaf(d, w[k].z, sv.z);
      sv.w = fmaf(d, w[k].w, sv.w);
    }
    if (r > 0) __syncthreads();  // red of row r - 1 read
    red[threadIdx.x] = sv;
    __syncthreads();
    if (threadIdx.x < 8) {
#pragma unroll 8
      for (int l = 0; l < 32; ++l) {
        const float4 v = red[l * 8 + threadIdx.x];
        tot[r].x += v.x;
        tot[r].y += v.y;
        tot[r].z += v.z;
        tot[r].w += v.w;
      }
    }
  }
  if (p.chunks > 1) {
    // 6. the chunk partials to the slab's last arriver (write-through stores, one ticket)
    if (threadIdx.x < 8) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (r < rows) st_sc1(p.ws + (int64_t(chunk) * rows + r) * K + col, tot[r]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t t = __hip_atomic_fetch_add(p.cnt + slab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = t == uint32_t(p.chunks - 1) ? 1u : 0u;
    }
    __syncthreads();
    if (flag == 0u) {
      store_dw();
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (threadIdx.x < 8) {
      constexpr int MAXC = 16;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= rows) continue;
        float4 v[MAXC];
#pragma unroll
        for (int ch = 0; ch < MAXC; ++ch) {
          const float* q = p.ws + (int64_t(ch < p.chunks ? ch : 0) * rows + r) * K + col;
          v[ch] = make_float4(ld_sc1(q), ld_sc1(q + 1), ld_sc1(q + 2), ld_sc1(q + 3));
        }
        tot[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int ch = 0; ch < MAXC; ++ch)
          if (ch < p.chunks) {
            tot[r].x += v[ch].x;
            tot[r].y += v[ch].y;
            tot[r].z += v[ch].z;
            tot[r].w += v[ch].w;
          }
      }
    }
    if (threadIdx.x == 0) __hip_atomic_store(p.cnt + slab, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // 7. the slab's final dh, or its columns of the LayerNorm backward of x
  if (threadIdx.x < 8) {
    if (p.lnfin) {
      const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
      const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
      float dg[4] = {0.f, 0.f, 0.f, 0.f}, db[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= rows) continue;
        const float t4[4] = {tot[r].x, tot[r].y, tot[r].z, tot[r].w};
        const float xh[4] = {xh4[r].x, xh4[r].y, xh4[r].z, xh4[r].w};
        float d[4], gv[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = fmaf(xh[k], gg[k], bb[k]) > 0.f ? t4[k] : 0.f;
          gv[k] = d[k] * gg[k];
          s1 += gv[k];
          s2 = fmaf(gv[k], xh[k], s2);
          dg[k] = fmaf(d[k], xh[k], dg[k]);
          db[k] += d[k];
        }
        *reinterpret_cast<float4*>(p.dh + int64_t(r) * K + col) = make_float4(gv[0], gv[1], gv[2], gv[3]);
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
          s1 += __shfl_xor(s1, o);
          s2 += __shfl_xor(s2, o);
        }
        if (threadIdx.x == 0) {
          p.lnp[(int64_t(r) * p.slabs + slab) * 2] = s1;
          p.lnp[(int64_t(r) * p.slabs + slab) * 2 + 1] = s2;
          if (slab == 0 && p.stats) {
            p.stats[2 * r] = mean[r];
            p.stats[2 * r + 1] = rstd[r];
          }
        }
      }
      *reinterpret_cast<float4*>(p.dgam + col) = make_float4(dg[0], dg[1], dg[2], dg[3]);
      *reinterpret_cast<float4*>(p.dbet + col) = make_float4(db[0], db[1], db[2], db[3]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (r < rows) *reinterpret_cast<float4*>(p.dh + int64_t(r) * K + col) = tot[r];
    }
  }
  store_dw();
}

// The same level on rows > 1 global rows (a union batch's global nodes), arranged for register
// pressure: the per-row dy go to LDS as soon as they are formed, the previous level's row-sum
// partials are summed by every wave for itself (lane l holds slab l: slabs <= 64; the same lanes
// and order as block_sums' wave 0, so bitwise the one-row result), the LayerNorm statistics of all
// rows take two workgroup sum rounds, and h / xh are recomputed where they are used.
template <int RPT, bool BF, int R>
__global__ __launch_bounds__(kBT) void gnode_bwd_rows_kernel(GnBwdArgs a) {
  static_assert(32 * RPT == kBT, "one dy row per thread");
  __shared__ float dys[R][32 * RPT];
  __shared__ float4 red[R][kBT];
  __shared__ float4 tots[R][8];
  __shared__ float scratch[4 * R + 8];
  __shared__ uint32_t flag;
  int blk0[kMaxProb];
#pragma unroll
  for (int q = 0; q < kMaxProb; ++q) blk0[q] = a.p[q].blk0;
  const int pi = find_prob(blk0, a.nprob);
  const GnBwdProb& p = a.p[pi];
  const int rows = p.rows;
  const int local = int(blockIdx.x) - p.blk0;
  const int slab = local % p.slabs, chunk = local / p.slabs;
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3, lane = threadIdx.x & 63;
  const int K = p.K, N = p.N;
  const int col = slab * kSW + 4 * cl;
  const int row0 = chunk * 32 * RPT;
  const int nrow = row0 + int(threadIdx.x), nrc = nrow < N ? nrow : N - 1;  // this thread's dy row
  const GnPro& pr = a.pro;
  const bool pro = pr.nq > 0;
  // 1. the workgroup's W slab rows first (the longest loads), then dy of every row into LDS
  float4 w[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int n = row0 + rl + 32 * k;
    w[k] = w4<BF>(p.W, p.Wh, int64_t(n < N ? n : N - 1) * K + col);
  }
  const float invF = pro ? 1.f / pr.F : 0.f;
  for (int r = 0; r < rows; ++r) {
    float d;
    if (pro) {
      const int64_t ro = int64_t(r) * pr.F;
      const int tl = lane < pr.slabs ? lane : 0;
      float gq[kMaxRaw], l1[kMaxRaw], l2[kMaxRaw];
#pragma unroll
      for (int q = 0; q < kMaxRaw; ++q) {
        const bool on = q < pr.nq;
        gq[q] = on ? pr.gv[q][ro + nrc] : 0.f;
        const int64_t lo = (int64_t(r) * pr.slabs + tl) * 2;
        l1[q] = on && lane < pr.slabs ? pr.lnp[q][lo] : 0.f;
        l2[q] = on && lane < pr.slabs ? pr.lnp[q][lo + 1] : 0.f;
      }
      d = pr.dres ? pr.dres[ro + nrc] : 0.f;
      const float m0 = pr.stats[2 * r], r0 = pr.stats[2 * r + 1];
      const float xh = (pr.x[ro + nrc] - m0) * r0;
#pragma unroll
      for (int q = 0; q < kMaxRaw; ++q) {
        const float s1 = wave_sum(l1[q]), s2 = wave_sum(l2[q]);
        if (q < pr.nq) d += r0 * (gq[q] - s1 * invF - xh * s2 * invF);
      }
      if (slab == 0 && pr.out && nrow < N) pr.out[ro + nrow] = d;
    } else {
      d = p.dy[int64_t(r) * N + nrc];
    }
    dys[r][threadIdx.x] = nrow < N ? d : 0.f;
  }
  // 2. the LayerNorm statistics of the input rows (two workgroup sum rounds for all of them)
  const bool ln = p.gam != nullptr;
  float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f), b4 = g4;
  float mean[R], rstd[R];
#pragma unroll
  for (int r = 0; r < R; ++r) mean[r] = rstd[r] = 0.f;
  if (ln) {
    g4 = *reinterpret_cast<const float4*>(p.gam + col);
    b4 = *reinterpret_cast<const float4*>(p.bet + col);
    float sx[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      sx[r] = 0.f;
      if (r < rows)
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
          const int j = int(threadIdx.x) + 256 * u;
          sx[r] += j < K ? p.x[int64_t(r) * K + j] : 0.f;
        }
    }
    block_sums<R>(sx, scratch);
#pragma unroll
    for (int r = 0; r < R; ++r) mean[r] = sx[r] / K;
    float sq[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      sq[r] = 0.f;
      if (r < rows)
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
          const int j = int(threadIdx.x) + 256 * u;
          const float dd = j < K ? p.x[int64_t(r) * K + j] - mean[r] : 0.f;
          sq[r] = fmaf(dd, dd, sq[r]);
        }
    }
    block_sums<R>(sq, scratch);
#pragma unroll
    for (int r = 0; r < R; ++r) rstd[r] = rsq_normal(sq[r] / K + p.eps);
  }
  __syncthreads();  // dys
  // 3. per row: this thread's share of dh; then 8 threads per row sum that row's 32 row lanes in
  // lane order (all rows at once: one barrier)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r >= rows) continue;
    float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const float d = dys[r][rl + 32 * k];  // 0 past N
      sv.x = fmaf(d, w[k].x, sv.x);
      sv.y = fmaf(d, w[k].y, sv.y);
      sv.z = fmaf(d, w[k].z, sv.z);
      sv.w = fmaf(d, w[k].w, sv.w);
    }
    red[r][threadIdx.x] = sv;
  }
  __syncthreads();
  const int tr = threadIdx.x >> 3;  // the row (r, column lane cl) of the threads < 8 rows
  const bool rowlane = int(threadIdx.x) < 8 * rows;
  if (rowlane) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int l = 0; l < 32; ++l) {
      const float4 v = red[tr][l * 8 + cl];
      t.x += v.x;
      t.y += v.y;
      t.z += v.z;
      t.w += v.w;
    }
    tots[tr][cl] = t;
  }
  auto hrow = [&](int r, float4& xh, float4& h) {
    const float4 x4 = *reinterpret_cast<const float4*>(p.x + int64_t(r) * K + col);
    if (!ln) {
      xh = h = x4;
      return;
    }
    xh = make_float4((x4.x - mean[r]) * rstd[r], (x4.y - mean[r]) * rstd[r], (x4.z - mean[r]) * rstd[r],
                     (x4.w - mean[r]) * rstd[r]);
    h = make_float4(fmaxf(fmaf(xh.x, g4.x, b4.x), 0.f), fmaxf(fmaf(xh.y, g4.y, b4.y), 0.f),
                    fmaxf(fmaf(xh.z, g4.z, b4.z), 0.f), fmaxf(fmaf(xh.w, g4.w, b4.w), 0.f));
  };
  auto store_dw = [&]() {
    float4 hs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float4 xh;
      hs[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < rows) hrow(r, xh, hs[r]);
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int n = row0 + rl + 32 * k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= rows) continue;
        const float d = dys[r][rl + 32 * k];
        v.x = fmaf(d, hs[r].x, v.x);
        v.y = fmaf(d, hs[r].y, v.y);
        v.z = fmaf(d, hs[r].z, v.z);
        v.w = fmaf(d, hs[r].w, v.w);
      }
      if (n < N) *reinterpret_cast<float4*>(p.dW + int64_t(n) * K + col) = v;
    }
    if (p.db && slab == 0 && nrow < N) {
      float v = 0.f;
      for (int r = 0; r < rows; ++r) v += dys[r][threadIdx.x];
      p.db[nrow] = v;
    }
  };
  if (p.chunks > 1) {
    // 4. the chunk partials to the slab's last arriver (write-through stores, one ticket)
    if (rowlane) st_sc1(p.ws + (int64_t(chunk) * rows + tr) * K + col, tots[tr][cl]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t t = __hip_atomic_fetch_add(p.cnt + slab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = t == uint32_t(p.chunks - 1) ? 1u : 0u;
    }
    __syncthreads();
    if (flag == 0u) {
      store_dw();
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (rowlane) {
      constexpr int MAXC = 16;
      float4 v[MAXC];
#pragma unroll
      for (int ch = 0; ch < MAXC; ++ch) {
        const float* q = p.ws + (int64_t(ch < p.chunks ? ch : 0) * rows + tr) * K + col;
        v[ch] = make_float4(ld_sc1(q), ld_sc1(q + 1), ld_sc1(q + 2), ld_sc1(q + 3));
      }
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int ch = 0; ch < MAXC; ++ch)
        if (ch < p.chunks) {
          t.x += v[ch].x;
          t.y += v[ch].y;
          t.z += v[ch].z;
          t.w += v[ch].w;
        }
      tots[tr][cl] = t;
    }
    if (threadIdx.x == 0) __hip_atomic_store(p.cnt + slab, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // 5. the slab's final dh, or its columns of the LayerNorm backward of x: 8 threads per row
  if (p.lnfin) {
    float4 dgr = make_float4(0.f, 0.f, 0.f, 0.f), dbr = dgr;
    if (rowlane) {
      float4 xh4, h4;
      hrow(tr, xh4, h4);
      const float4 tt = tots[tr][cl];
      const float t4[4] = {tt.x, tt.y, tt.z, tt.w};
      const float xh[4] = {xh4.x, xh4.y, xh4.z, xh4.w};
      const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
      const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
      float d[4], gv[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        d[k] = fmaf(xh[k], gg[k], bb[k]) > 0.f ? t4[k] : 0.f;
        gv[k] = d[k] * gg[k];
        s1 += gv[k];
        s2 = fmaf(gv[k], xh[k], s2);
      }
      dgr = make_float4(d[0] * xh[0], d[1] * xh[1], d[2] * xh[2], d[3] * xh[3]);
      dbr = make_float4(d[0], d[1], d[2], d[3]);
      *reinterpret_cast<float4*>(p.dh + int64_t(tr) * K + col) = make_float4(gv[0], gv[1], gv[2], gv[3]);
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {  // the row's 8 column lanes (consecutive lanes of one wave)
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
      }
      if (cl == 0) {
        p.lnp[(int64_t(tr) * p.slabs + slab) * 2] = s1;
        p.lnp[(int64_t(tr) * p.slabs + slab) * 2 + 1] = s2;
        if (slab == 0 && p.stats) {
          p.stats[2 * tr] = mean[tr];
          p.stats[2 * tr + 1] = rstd[tr];
        }
      }
    }
    // gamma / beta gradients: the rows' column partials summed in row order
    __syncthreads();  // red's dh partials consumed (step 3)
    if (rowlane) {
      red[tr][cl] = dgr;
      red[tr][8 + cl] = dbr;
    }
    __syncthreads();
    if (threadIdx.x < 8) {
      float4 dg = make_float4(0.f, 0.f, 0.f, 0.f), db = dg;
      for (int r = 0; r < rows; ++r) {
        const float4 a4 = red[r][threadIdx.x], b4v = red[r][8 + threadIdx.x];
        dg.x += a4.x;
        dg.y += a4.y;
        dg.z += a4.z;
        dg.w += a4.w;
        db.x += b4v.x;
        db.y += b4v.y;
        db.z += b4v.z;
        db.w += b4v.w;
      }
      *reinterpret_cast<float4*>(p.dgam + col) = dg;
      *reinterpret_cast<float4*>(p.dbet + col) = db;
    }
  } else if (rowlane) {
    *reinterpret_cast<float4*>(p.dh + int64_t(tr) * K + col) = tots[tr][cl];
  }
  store_dw();
}

constexpr int kRPT = 8;  // 256 rows per chunk

int chunks_of(int N) { return (N + 32 * kRPT - 1) / (32 * kRPT); }

// fills blk0 / slabs / chunks / ws / cnt / rows of the level's problems; ws and cnt advance
int launch_bwd(GnBwdArgs& a, int rows, float*& ws, uint32_t*& cnt, hipStream_t st, const char* where) {
  int blocks = 0;
  for (int q = 0; q < a.nprob; ++q) {
    GnBwdProb& p = a.p[q];
    p.blk0 = blocks;
    p.slabs = p.K / kSW;
    p.chunks = chunks_of(p.N);
    p.ws = ws;
    p.cnt = cnt;
    p.rows = rows;
    ws += int64_t(p.chunks) * rows * p.K;
    cnt += p.slabs;
    blocks += p.slabs * p.chunks;
  }
  for (int q = a.nprob; q < kMaxProb; ++q) a.p[q].blk0 = blocks;
  bool bf = true;
  for (int q = 0; q < a.nprob; ++q) bf = bf && a.p[q].Wh != nullptr;
  const auto kern = rows > 1 ? (bf ? &gnode_bwd_rows_kernel<kRPT, true, kMaxRows>
                                    : &gnode_bwd_rows_kernel<kRPT, false, kMaxRows>)
                             : (bf ? &gnode_bwd_kernel<kRPT, true, 1> : &gnode_bwd_kernel<kRPT, false, 1>);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBT), 0, st, a);
  return launch_status(where);
}

int rows_of(const gasfm_gchain* c) { return c->rows > 1 ? c->rows : 1; }

bool hub_on(const gasfm_gchain* c) { return c->NB > 0; }

}  // namespace
}  // namespace gasfm

using namespace gasfm;

static int gchain_check(const gasfm_gchain* c) {
  GASFM_REQUIRE(c, "gasfm_gchain: null parameters");
  GASFM_REQUIRE(c->G > 0 && c->G <= kMaxK && c->G % kSW == 0 && c->Kc > 0 && c->Kc <= kMaxK && c->Kc % kSW == 0 &&
                    c->NA > 0 && c->NA <= kMaxK,
                "gasfm_gchain: G=%d Kc=%d NA=%d (multiples of %d, <= %d)", c->G, c->Kc, c->NA, kSW, kMaxK);
  GASFM_REQUIRE(c->W1 && c->b1 && c->gM && c->bM && c->W2 && c->b2 && c->gA && c->bA && c->WA,
                "gasfm_gchain: null weight");
  if (c->NB > 0) {
    GASFM_REQUIRE(c->NB <= kMaxK && c->NB % kSW == 0 && c->NC > 0 && c->NC <= kMaxK && c->NC % kSW == 0 &&
                      c->ND > 0 && c->ND <= kMaxK && c->NE > 0 && c->NE <= kMaxK,
                  "gasfm_gchain: NB=%d NC=%d ND=%d NE=%d", c->NB, c->NC, c->ND, c->NE);
    GASFM_REQUIRE(c->gB && c->bB && c->WB && c->bWB && c->gC && c->bC && c->WC && c->bWC && c->WD && c->bD && c->WE &&
                      c->bE,
                  "gasfm_gchain: null hub weight");
  }
  GASFM_REQUIRE(c->rows >= 0 && c->rows <= kMaxRows, "gasfm_gchain: rows=%d (<= %d)", c->rows, kMaxRows);
  const void* ws[] = {c->W1, c->W2, c->WA, c->WB, c->WC, c->WD, c->WE};
  for (const void* p : ws) GASFM_REQUIRE(!p || aligned16(p), "gasfm_gchain: weights must be 16-byte aligned");
  const void* wh[] = {c->W1h, c->W2h, c->WAh, c->WBh, c->WCh, c->WDh, c->WEh};
  for (const void* p : wh)
    GASFM_REQUIRE(!p || reinterpret_cast<uintptr_t>(p) % 8 == 0, "gasfm_gchain: bf16 shadows must be 8-byte aligned");
  return GASFM_OK;
}

extern "C" int64_t gasfm_gchain_scratch_floats(const gasfm_gchain* c) {
  if (!c) return 0;
  // vectors: dh_D, dh_E, gv_A, gv_B, gv_C, gv_2; LayerNorm row-sum partials and statistics; chunk
  // partials of every level (each level its own range)
  const int64_t R = rows_of(c);
  const int64_t vec = int64_t(c->NB) + c->NC + 4 * int64_t(c->G);
  const int64_t lnp = 4 * 2 * int64_t(c->G / kSW) + 8;
  const int64_t l1 = int64_t(chunks_of(c->ND)) * c->NB + int64_t(chunks_of(c->NE)) * c->NC;
  const int64_t l2 = int64_t(chunks_of(c->NA) + chunks_of(c->NB) + chunks_of(c->NC)) * c->G;
  const int64_t l3 = int64_t(chunks_of(c->G)) * c->G;
  const int64_t l4 = int64_t(chunks_of(c->G)) * c->Kc;
  return R * (vec + lnp + l1 + l2 + l3 + l4 + c->G) + 64;
}

extern "C" int32_t gasfm_gchain_counters(const gasfm_gchain* c) {
  if (!c) return 0;
  return (c->NB + c->NC + 4 * c->G + c->Kc) / kSW + 8;  // per-slab tickets
}

extern "C" int gasfm_gchain_fwd(const gasfm_gchain* c, const float* xcat, const float* prev, float* x1, float* g,
                                float* sg, float* xv, float* xp, float* xrv, float* xrp, void* stream) {
  const int s0 = gchain_check(c);
  if (s0 != GASFM_OK) return s0;
  GASFM_REQUIRE(xcat && x1 && g && sg && (!hub_on(c) || (xv && xp && xrv && xrp)), "gasfm_gchain_fwd: null output");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int R = rows_of(c);
  GnFwdArgs a{};
  a.nprob = 1;
  a.p[0] = GnFwdProb{xcat, nullptr, nullptr, c->W1, c->b1, prev, x1, c->Kc, c->G, 0, 0.f, c->W1h, R};
  int s = launch_fwd(a, st);
  if (s != GASFM_OK) return s;
  a.p[0] = GnFwdProb{x1, c->gM, c->bM, c->W2, c->b2, x1, g, c->G, c->G, 0, c->eps_m, c->W2h, R};
  s = launch_fwd(a, st);
  if (s != GASFM_OK) return s;
  a.p[0] = GnFwdProb{g, c->gA, c->bA, c->WA, nullptr, nullptr, sg, c->G, c->NA, 0, c->eps_h, c->WAh, R};
  if (hub_on(c)) {
    a.nprob = 3;
    a.p[1] = GnFwdProb{g, c->gB, c->bB, c->WB, c->bWB, nullptr, xv, c->G, c->NB, 0, c->eps_h, c->WBh, R};
    a.p[2] = GnFwdProb{g, c->gC, c->bC, c->WC, c->bWC, nullptr, xp, c->G, c->NC, 0, c->eps_h, c->WCh, R};
  }
  s = launch_fwd(a, st);
  if (s != GASFM_OK || !hub_on(c)) return s;
  a.nprob = 2;
  a.p[0] = GnFwdProb{xv, nullptr, nullptr, c->WD, c->bD, nullptr, xrv, c->NB, c->ND, 0, 0.f, c->WDh, R};
  a.p[1] = GnFwdProb{xp, nullptr, nullptr, c->WE, c->bE, nullptr, xrp, c->NC, c->NE, 0, 0.f, c->WEh, R};
  return launch_fwd(a, st);
}

extern "C" int gasfm_gchain_bwd(const gasfm_gchain* c, const float* xcat, const float* x1, const float* g,
                                const float* xv, const float* xp, const float* dskip, const float* dsg,
                                const float* dxrv, const float* dxrp, float* dxcat, float* dprev,
                                const gasfm_gchain_grads* d, float* scratch, uint32_t* counters, void* stream) {
  const int s0 = gchain_check(c);
  if (s0 != GASFM_OK) return s0;
  GASFM_REQUIRE(d && xcat && x1 && g && dsg && dxcat && scratch && counters, "gasfm_gchain_bwd: null pointer");
  GASFM_REQUIRE(d->dW1 && d->db1 && d->dgM && d->dbM && d->dW2 && d->db2 && d->dgA && d->dbA && d->dWA,
                "gasfm_gchain_bwd: null gradient");
  const bool hub = hub_on(c);
  if (hub)
    GASFM_REQUIRE(xv && xp && dxrv && dxrp && d->dgB && d->dbB && d->dWB && d->dbWB && d->dgC && d->dbC && d->dWC &&
                      d->dbWC && d->dWD && d->dbD && d->dWE && d->dbE,
                  "gasfm_gchain_bwd: null hub pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int slabsG = c->G / kSW;
  const int R = rows_of(c);  // every vector below is [R, len]
  float* dhD = scratch;
  float* dhE = dhD + int64_t(R) * c->NB;
  float* gvA = dhE + int64_t(R) * c->NC;
  float* gvB = gvA + int64_t(R) * c->G;
  float* gvC = gvB + int64_t(R) * c->G;
  float* gv2 = gvC + int64_t(R) * c->G;
  float* lnA = gv2 + int64_t(R) * c->G;  // [R][slabsG][2] each
  float* lnB = lnA + 2 * R * slabsG;
  float* lnC = lnB + 2 * R * slabsG;
  float* ln2 = lnC + 2 * R * slabsG;
  float* stg = ln2 + 2 * R * slabsG;  // [R][2] (mean, rstd) of g, then of x1
  float* st1 = stg + 2 * R;
  float* dgr = st1 + 2 * R + 4;  // [R][G] dg per row (B3's dy; with one row it equals db2)
  float* ws = dgr + int64_t(R) * c->G;
  uint32_t* cnt = counters;
  int s;
  if (hub) {  // B1: the two lin_r rows
    GnBwdArgs a{};
    a.nprob = 2;
    a.p[0] = GnBwdProb{dxrv, xv, nullptr, nullptr, c->WD, d->dWD, d->dbD, dhD};
    a.p[0].K = c->NB, a.p[0].N = c->ND, a.p[0].Wh = c->WDh;
    a.p[1] = GnBwdProb{dxrp, xp, nullptr, nullptr, c->WE, d->dWE, d->dbE, dhE};
    a.p[1].K = c->NC, a.p[1].N = c->NE, a.p[1].Wh = c->WEh;
    s = launch_bwd(a, R, ws, cnt, st, "gasfm_gchain_bwd(lin_r)");
    if (s != GASFM_OK) return s;
  }
  {  // B2: the LayerNorm -> Linear consumers of g; each slab's last arriver runs its columns of
     // their LayerNorm backwards (gv, gamma / beta gradients, row-sum partials)
    GnBwdArgs a{};
    a.nprob = hub ? 3 : 1;
    auto lnprob = [&](const float* dy, const float* gam, const float* bet, const float* W, const uint16_t* Wh,
                      float* dW, float* db, int N, float* gv, float* dgam, float* dbet, float* lnp, float* stats) {
      GnBwdProb p{dy, g, gam, bet, W, dW, db, gv};
      p.K = c->G, p.N = N, p.eps = c->eps_h, p.Wh = Wh;
      p.dgam = dgam, p.dbet = dbet, p.lnp = lnp, p.stats = stats, p.lnfin = 1;
      return p;
    };
    a.p[0] = lnprob(dsg, c->gA, c->bA, c->WA, c->WAh, d->dWA, nullptr, c->NA, gvA, d->dgA, d->dbA, lnA, stg);
    if (hub) {
      a.p[1] = lnprob(dhD, c->gB, c->bB, c->WB, c->WBh, d->dWB, d->dbWB, c->NB, gvB, d->dgB, d->dbB, lnB, nullptr);
      a.p[2] = lnprob(dhE, c->gC, c->bC, c->WC, c->WCh, d->dWC, d->dbWC, c->NC, gvC, d->dgC, d->dbC, lnC, nullptr);
    }
    s = launch_bwd(a, R, ws, cnt, st, "gasfm_gchain_bwd(hub)");
    if (s != GASFM_OK) return s;
  }
  {  // B3: the MLP Linear on dg (= dskip + the hub LayerNorms' backward, finished per row in the
     // prologue; written to db2, which IS dg); the slab last arrivers run LN_M's columns
    GnBwdArgs a{};
    a.nprob = 1;
    GnBwdProb& p = a.p[0];
    p = GnBwdProb{nullptr, x1, c->gM, c->bM, c->W2, d->dW2, d->db2, gv2};
    p.K = c->G, p.N = c->G, p.eps = c->eps_m, p.Wh = c->W2h;
    p.dgam = d->dgM, p.dbet = d->dbM, p.lnp = ln2, p.stats = st1, p.lnfin = 1;
    GnPro& pr = a.pro;
    pr.nq = hub ? 3 : 1;
    pr.gv[0] = gvA, pr.lnp[0] = lnA;
    pr.gv[1] = gvB, pr.lnp[1] = lnB;
    pr.gv[2] = gvC, pr.lnp[2] = lnC;
    pr.stats = stg, pr.x = g, pr.dres = dskip, pr.out = R > 1 ? dgr : nullptr, pr.F = c->G, pr.slabs = slabsG;
    s = launch_bwd(a, R, ws, cnt, st, "gasfm_gchain_bwd(mlp)");
    if (s != GASFM_OK) return s;
  }
  // B4: proj_view_and_scenepoint2global on dx1 = dg + LN_M backward (prologue; = d b1 = d prev)
  GnBwdArgs a{};
  a.nprob = 1;
  a.p[0] = GnBwdProb{nullptr, xcat, nullptr, nullptr, c->W1, d->dW1, d->db1, dxcat};
  a.p[0].K = c->Kc, a.p[0].N = c->G, a.p[0].Wh = c->W1h;
  GnPro& pr = a.pro;
  pr.nq = 1;
  pr.gv[0] = gv2, pr.lnp[0] = ln2;
  pr.stats = st1, pr.x = x1, pr.dres = R > 1 ? dgr : d->db2, pr.out = dprev, pr.F = c->G, pr.slabs = slabsG;
  return launch_bwd(a, R, ws, cnt, st, "gasfm_gchain_bwd(proj)");
}
