// The GATv2 attention onto the single global node -- the view->global and points->global convs of a
// GASFM block (code/models/layers.py:550-556, 566-572; PyG GATv2Conv, one target) -- forward and
// backward, BOTH sources in one launch each way, gfx950.
//
// Round 3 ran each conv as a work-item attention kernel plus one or two ordered combine launches
// (points -> global: ~4k short pieces, a two-level combine) and, backward, a kernel plus a colsum:
// ~6 launches each way per block, each a few us of latency.  Here a workgroup takes a chunk of
// sources (8 views, 256 points; round 4), keeps an online softmax state (max, sum, acc) per head and
// writes it to a slot; the problem's LAST-arriving workgroup (write-through stores, one relaxed
// agent-scope ticket: reduce.hip's hand-off) merges the slots -- max, then the rescaled sums,
// parallel over slots with a fixed association order -- and writes the output + statistics, or
// on a sharded rank the packed partial row [acc HC | max H | sum H] its exchange sends.
//   views  (C = 256): thread t holds features 4t..4t+3 of the source row; head = wave
//   points (C = 16):  16 threads per source (float4 each), 16 sources in flight per workgroup;
//                     the 16 source lanes' states are merged in LDS, in lane order
// Backward recomputes each source's logit and alpha from the saved statistics and writes its dXL
// row; dXR and datt are slot sums merged the same way.  No float atomics: deterministic, and
// identical on every rank.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kT = 256;
constexpr int H = 4;
// sources per workgroup (round 4 retune: 64 / 2048 left 15 workgroups on a rank of 8 walking their
// chunks one step at a time, 53 + 81 us per block; the slots are now read back by plain batched
// loads, so more, shorter chunks cost little at the merge)
#ifndef GASFM_GATT_CHUNK_V
#define GASFM_GATT_CHUNK_V 8
#endif
#ifndef GASFM_GATT_CHUNK_P
#define GASFM_GATT_CHUNK_P 256
#endif
constexpr int kChunkV = GASFM_GATT_CHUNK_V;  // sources per workgroup, C = 256
constexpr int kChunkP = GASFM_GATT_CHUNK_P;  // sources per workgroup, C = 16
constexpr int kMaxProb = 2;
// slots per first-level group: a whole config-4 scene's 200k points are 782 chunks, which one
// workgroup merged in ~25 us; 25 groups of 32 merge in parallel, then 25 group rows
constexpr int kGroup = 32;

struct GaProb {
  const float* XL;
  int64_t ldXL;
  const int32_t* src;
  const float* XR;
  const float* att;
  const float* bias;
  float* out;
  float* smax;
  float* ssum;
  float* part;
  const float* gout;
  float* dXL;
  int64_t ldDXL;
  float* dXR;
  float* datt;
  float* slots;    // [nblk, slot floats]
  uint32_t* cnt;   // the problem's ticket
  int64_t sl;      // forward slot stride
  int S, HC, C, blk0, nblk;
  // two-level merge (nblk > kGroup): groups of kGroup consecutive slots are merged by their own
  // last arriver into group rows (same layout), and the last group merges the group rows
  float* gslots;   // [ngroups, slot floats]
  uint32_t* gcnt;  // [ngroups] tickets
  int ngroups;
};
struct GaArgs {
  GaProb p[kMaxProb];
  int nprob;
  float slope;
};

__device__ __forceinline__ float leaky(float z, float slope) { return z > 0.f ? z : z * slope; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ int find_prob(const GaArgs& a) {
  return (a.nprob > 1 && int(blockIdx.x) >= a.p[1].blk0) ? 1 : 0;
}

__device__ __forceinline__ int src_row(const GaProb& p, int j) { return p.src ? p.src[j] : j; }

__device__ __forceinline__ void st_sc1(float* q, float v) {
  __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// true for the problem's last-arriving workgroup (after its slot was stored write-through)
__device__ __forceinline__ bool last_arrival(uint32_t* cnt, int n, uint32_t* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = t == uint32_t(n - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (*flag == 0u) return false;
  // agent-scope acquire: this CU's L1 holds no stale slot lines, so the merges read the slots with
  // plain (batched, vector) loads instead of one relaxed atomic load per value
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// ------------------------------------------------------------------------------------ merge
// the last arriver of a problem: slots [nblk][HC + 2H] (acc | max | sum) -> M, S per head, then
// the rescaled acc; writes the final output (+ bias) and statistics, or the packed partial row
__device__ void merge_fwd(const GaProb& p, float* sc) {
  __shared__ float MH[H], SH[H];
  __shared__ float accg[4][64];
  const int64_t L = p.sl;  // slot stride (HC + 2H; the gathered send blocks' stride when merging ranks)
  const int n = p.nblk;
  // 1. max per head: thread (k = tid >> 2, h = tid & 3) over slots k, k + 64, ...
  {
    const int h = threadIdx.x & 3;
    float m = -INFINITY;
    for (int k = threadIdx.x >> 2; k < n; k += kT / 4) m = fmaxf(m, p.slots[int64_t(k) * L + p.HC + h]);
#pragma unroll
    for (int o = 32; o >= 4; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    __syncthreads();
    if ((threadIdx.x & 63) < 4) sc[(threadIdx.x >> 6) * 4 + h] = m;
    __syncthreads();
    if (threadIdx.x < H)
      MH[threadIdx.x] = fmaxf(fmaxf(sc[threadIdx.x], sc[4 + threadIdx.x]), fmaxf(sc[8 + threadIdx.x], sc[12 + threadIdx.x]));
    __syncthreads();
  }
  // 2. sum per head, rescaled
  {
    const int h = threadIdx.x & 3;
    const float M = MH[h];
    float s = 0.f;
    for (int k = threadIdx.x >> 2; k < n; k += kT / 4) {
      const float* q = p.slots + int64_t(k) * L + p.HC;
      const float mk = q[h], sk = q[H + h];
      s += mk == -INFINITY ? 0.f : sk * __expf(mk - M);
    }
#pragma unroll
    for (int o = 32; o >= 4; o >>= 1) s += __shfl_xor(s, o);
    __syncthreads();
    if ((threadIdx.x & 63) < 4) sc[(threadIdx.x >> 6) * 4 + h] = s;
    __syncthreads();
    if (threadIdx.x < H)
      SH[threadIdx.x] = (sc[threadIdx.x] + sc[4 + threadIdx.x]) + (sc[8 + threadIdx.x] + sc[12 + threadIdx.x]);
    __syncthreads();
  }
  // 3. acc per feature: C = 256: thread t features 4t..4t+3 over every slot; C = 16: 64 features x
  // 4 slot groups (k = grp, grp + 4, ..), the groups added in order
  auto finish = [&](int f, float a) {
    const int h = f / p.C;
    if (p.part) {  // write-through: a group row is merged by another workgroup in this launch
      st_sc1(p.part + f, a);
      if (f < H) {
        st_sc1(p.part + p.HC + f, MH[f]);
        st_sc1(p.part + p.HC + H + f, SH[f]);
      }
    } else {
      p.out[f] = a / (SH[h] + 1e-16f) + p.bias[f];
      if (f < H) {
        p.smax[f] = MH[f];
        p.ssum[f] = SH[f];
      }
    }
  };
  if (p.C == 256) {
    const int f0 = 4 * threadIdx.x, h = f0 / 256;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int k = 0; k < n; ++k) {
      const float* q = p.slots + int64_t(k) * L;
      const float mk = q[p.HC + h];
      const float w = mk == -INFINITY ? 0.f : __expf(mk - MH[h]);
      const float4 v = *reinterpret_cast<const float4*>(q + f0);  // L % 4 == 0
      a.x = fmaf(v.x, w, a.x);
      a.y = fmaf(v.y, w, a.y);
      a.z = fmaf(v.z, w, a.z);
      a.w = fmaf(v.w, w, a.w);
    }
    finish(f0, a.x);
    finish(f0 + 1, a.y);
    finish(f0 + 2, a.z);
    finish(f0 + 3, a.w);
  } else {
    const int f = threadIdx.x & 63, grp = threadIdx.x >> 6, h = f / p.C;
    float a = 0.f;
    if (f < p.HC)
#pragma unroll 8
      for (int k = grp; k < n; k += 4) {
        const float* q = p.slots + int64_t(k) * L;
        const float mk = q[p.HC + h];
        a = fmaf(q[f], mk == -INFINITY ? 0.f : __expf(mk - MH[h]), a);
      }
    accg[grp][f] = a;
    __syncthreads();
    if (threadIdx.x < p.HC) finish(threadIdx.x, (accg[0][f] + accg[1][f]) + (accg[2][f] + accg[3][f]));
  }
}

// after a workgroup's slot is stored: the merge, by the problem's last arriver (one level), or by
// the group's last arriver into the group row and then the last group's into the output
__device__ void done_fwd(const GaProb& p, int blk, uint32_t* flag, float* sc) {
  if (p.ngroups <= 1) {
    if (last_arrival(p.cnt, p.nblk, flag)) {
      merge_fwd(p, sc);
      if (threadIdx.x == 0) __hip_atomic_store(p.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int g = blk / kGroup, n0 = g * kGroup;
  const int ng = p.nblk - n0 < kGroup ? p.nblk - n0 : kGroup;
  if (!last_arrival(p.gcnt + g, ng, flag)) return;
  GaProb q = p;  // the group's slots -> its raw (packed) group row
  q.slots = p.slots + int64_t(n0) * p.sl;
  q.nblk = ng;
  q.part = p.gslots + int64_t(g) * p.sl;
  merge_fwd(q, sc);
  if (threadIdx.x == 0) __hip_atomic_store(p.gcnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (!last_arrival(p.cnt, p.ngroups, flag)) return;
  GaProb r = p;  // the group rows -> the output (or the exchange's packed row)
  r.slots = p.gslots;
  r.nblk = p.ngroups;
  merge_fwd(r, sc);
  if (threadIdx.x == 0) __hip_atomic_store(p.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// --------------------------------------------------------------------------------- forward
__device__ void fwd_views(const GaProb& p, int blk, float slope, uint32_t* flag, float* sc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f0 = 4 * threadIdx.x;  // head = wave
  const int j0 = blk * kChunkV, j1 = min(p.S, j0 + kChunkV);
  const float4 xr = *reinterpret_cast<const float4*>(p.XR + f0);
  const float4 at = *reinterpret_cast<const float4*>(p.att + f0);
  float m = -INFINITY, s = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 nx = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j0 < j1) nx = *reinterpret_cast<const float4*>(p.XL + int64_t(src_row(p, j0)) * p.ldXL + f0);
  for (int j = j0; j < j1; ++j) {
    const float4 x = nx;
    const int jn = j + 1 < j1 ? j + 1 : j;
    nx = *reinterpret_cast<const float4*>(p.XL + int64_t(src_row(p, jn)) * p.ldXL + f0);
    float e = leaky(x.x + xr.x, slope) * at.x + leaky(x.y + xr.y, slope) * at.y + leaky(x.z + xr.z, slope) * at.z +
              leaky(x.w + xr.w, slope) * at.w;
    e = wave_sum(e);
    const float mn = fmaxf(m, e);
    const float sc0 = m == -INFINITY ? 0.f : __expf(m - mn), w = __expf(e - mn);
    s = fmaf(s, sc0, w);
    acc = make_float4(fmaf(acc.x, sc0, w * x.x), fmaf(acc.y, sc0, w * x.y), fmaf(acc.z, sc0, w * x.z),
                      fmaf(acc.w, sc0, w * x.w));
    m = mn;
  }
  float* slot = p.slots + int64_t(blk) * (p.HC + 2 * H);
  st_sc1(slot + f0, acc.x);
  st_sc1(slot + f0 + 1, acc.y);
  st_sc1(slot + f0 + 2, acc.z);
  st_sc1(slot + f0 + 3, acc.w);
  if (lane == 0) {
    st_sc1(slot + p.HC + wave, m);
    st_sc1(slot + p.HC + H + wave, s);
  }
  done_fwd(p, blk, flag, sc);
}

// C = 16: thread (ql = tid >> 4: source lane, fq = tid & 15: features 4 fq.., head fq >> 2)
__device__ void fwd_points(const GaProb& p, int blk, float slope, uint32_t* flag, float* sc) {
  __shared__ float SM[16][H], SS[16][H];
  __shared__ float4 SA[16][16];
  const int ql = threadIdx.x >> 4, fq = threadIdx.x & 15, h = fq >> 2;
  const int f0 = 4 * fq;
  const int j0 = blk * kChunkP, j1 = min(p.S, j0 + kChunkP);
  const float4 xr = *reinterpret_cast<const float4*>(p.XR + f0);
  const float4 at = *reinterpret_cast<const float4*>(p.att + f0);
  float m = -INFINITY, s = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int U = 4;  // sources per step per lane, loads in flight together
  for (int jb = j0 + ql; jb < j1; jb += 16 * U) {
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jb + 16 * u;
      x[u] = *reinterpret_cast<const float4*>(p.XL + int64_t(src_row(p, j < j1 ? j : jb)) * p.ldXL + f0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float e = leaky(x[u].x + xr.x, slope) * at.x + leaky(x[u].y + xr.y, slope) * at.y +
                leaky(x[u].z + xr.z, slope) * at.z + leaky(x[u].w + xr.w, slope) * at.w;
      e += __shfl_xor(e, 1);
      e += __shfl_xor(e, 2);
      if (jb + 16 * u < j1) {
        const float mn = fmaxf(m, e);
        const float sc0 = m == -INFINITY ? 0.f : __expf(m - mn), w = __expf(e - mn);
        s = fmaf(s, sc0, w);
        acc = make_float4(fmaf(acc.x, sc0, w * x[u].x), fmaf(acc.y, sc0, w * x[u].y), fmaf(acc.z, sc0, w * x[u].z),
                          fmaf(acc.w, sc0, w * x[u].w));
        m = mn;
      }
    }
  }
  // the 16 source lanes merged in lane order
  if ((fq & 3) == 0) {
    SM[ql][h] = m;
    SS[ql][h] = s;
  }
  SA[ql][fq] = acc;
  __syncthreads();
  float* slot = p.slots + int64_t(blk) * (p.HC + 2 * H);
  if (threadIdx.x < 16) {  // thread fq: features 4 fq.., head fq >> 2
    const int hh = threadIdx.x >> 2;
    float M = -INFINITY;
#pragma unroll
    for (int q = 0; q < 16; ++q) M = fmaxf(M, SM[q][hh]);
    float S = 0.f;
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float mq = SM[q][hh];
      const float w = mq == -INFINITY ? 0.f : __expf(mq - M);
      S = fmaf(SS[q][hh], w, S);
      const float4 a = SA[q][threadIdx.x];
      A = make_float4(fmaf(a.x, w, A.x), fmaf(a.y, w, A.y), fmaf(a.z, w, A.z), fmaf(a.w, w, A.w));
    }
    const int g0 = 4 * threadIdx.x;
    st_sc1(slot + g0, A.x);
    st_sc1(slot + g0 + 1, A.y);
    st_sc1(slot + g0 + 2, A.z);
    st_sc1(slot + g0 + 3, A.w);
    if ((threadIdx.x & 3) == 0) {
      st_sc1(slot + p.HC + hh, M);
      st_sc1(slot + p.HC + H + hh, S);
    }
  }
  done_fwd(p, blk, flag, sc);
}

__global__ __launch_bounds__(kT) void gatt_fwd_kernel(GaArgs a) {
  __shared__ uint32_t flag;
  __shared__ float sc[16];
  const int pi = find_prob(a);
  const GaProb& p = a.p[pi];
  const int blk = int(blockIdx.x) - p.blk0;
  if (p.C == 256)
    fwd_views(p, blk, a.slope, &flag, sc);
  else
    fwd_points(p, blk, a.slope, &flag, sc);
}

// -------------------------------------------------------------------------------- backward
// slots [nblk][2 HC] (dXR | datt); the last arriver sums them in slot order
// final == false (first level of a two-level merge): the raw sums go to grow [2 HC] (write-through)
__device__ void merge_bwd(const GaProb& p, bool final = true, float* grow = nullptr) {
  __shared__ float acc4[4][2 * 64];
  const int L = 2 * p.HC, n = p.nblk;
  if (p.C == 256) {  // thread t: features 4t..4t+3 of both halves
    for (int half = 0; half < 2; ++half) {
      const int f0 = 4 * threadIdx.x;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
      for (int k = 0; k < n; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(p.slots + int64_t(k) * L + half * p.HC + f0);
        a.x += v.x;
        a.y += v.y;
        a.z += v.z;
        a.w += v.w;
      }
      if (!final) {
        float* d = grow + half * p.HC + f0;
        st_sc1(d, a.x);
        st_sc1(d + 1, a.y);
        st_sc1(d + 2, a.z);
        st_sc1(d + 3, a.w);
        continue;
      }
      float* d = half ? p.datt : p.dXR;
      d[f0] = a.x;
      d[f0 + 1] = a.y;
      d[f0 + 2] = a.z;
      d[f0 + 3] = a.w;
    }
    if (final)
      *reinterpret_cast<float4*>(p.datt + p.HC + 4 * threadIdx.x) =
          *reinterpret_cast<const float4*>(p.gout + 4 * threadIdx.x);
  } else {  // 2 HC = 128 values x 4 slot groups (256 threads: value v = tid & 63 (+ 64), group tid >> 6)
    const int grp = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int v = (threadIdx.x & 63) + 64 * r;
      float a = 0.f;
      if (v < L)
#pragma unroll 8
        for (int k = grp; k < n; k += 4) a += p.slots[int64_t(k) * L + v];
      acc4[grp][v] = a;
    }
    __syncthreads();
    if (threadIdx.x < L) {
      const float a = (acc4[0][threadIdx.x] + acc4[1][threadIdx.x]) + (acc4[2][threadIdx.x] + acc4[3][threadIdx.x]);
      if (!final)
        st_sc1(grow + threadIdx.x, a);
      else if (threadIdx.x < p.HC)
        p.dXR[threadIdx.x] = a;
      else
        p.datt[threadIdx.x - p.HC] = a;
    }
    if (final && threadIdx.x < p.HC) p.datt[p.HC + threadIdx.x] = p.gout[threadIdx.x];
  }
}

__device__ void done_bwd(const GaProb& p, int blk, uint32_t* flag) {
  if (p.ngroups <= 1) {
    if (last_arrival(p.cnt, p.nblk, flag)) {
      merge_bwd(p);
      if (threadIdx.x == 0) __hip_atomic_store(p.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int g = blk / kGroup, n0 = g * kGroup;
  const int ng = p.nblk - n0 < kGroup ? p.nblk - n0 : kGroup;
  if (!last_arrival(p.gcnt + g, ng, flag)) return;
  const int64_t L = 2 * int64_t(p.HC);
  GaProb q = p;
  q.slots = p.slots + int64_t(n0) * L;
  q.nblk = ng;
  merge_bwd(q, false, p.gslots + int64_t(g) * L);
  if (threadIdx.x == 0) __hip_atomic_store(p.gcnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (!last_arrival(p.cnt, p.ngroups, flag)) return;
  GaProb r = p;
  r.slots = p.gslots;
  r.nblk = p.ngroups;
  merge_bwd(r);
  if (threadIdx.x == 0) __hip_atomic_store(p.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void bwd_views(const GaProb& p, int blk, float slope, uint32_t* flag) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f0 = 4 * threadIdx.x;
  const int j0 = blk * kChunkV, j1 = min(p.S, j0 + kChunkV);
  const float4 xr = *reinterpret_cast<const float4*>(p.XR + f0);
  const float4 at = *reinterpret_cast<const float4*>(p.att + f0);
  const float4 go = *reinterpret_cast<const float4*>(p.gout + f0);
  const float4 o4 = *reinterpret_cast<const float4*>(p.out + f0);
  const float4 b4 = *reinterpret_cast<const float4*>(p.bias + f0);
  const float M = p.smax[wave], inv = 1.f / (p.ssum[wave] + 1e-16f);
  const float delta =
      wave_sum(go.x * (o4.x - b4.x) + go.y * (o4.y - b4.y) + go.z * (o4.z - b4.z) + go.w * (o4.w - b4.w));
  float4 dxr = make_float4(0.f, 0.f, 0.f, 0.f), dat = dxr;
  int jr = 0;
  float4 nx = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j0 < j1) {
    jr = src_row(p, j0);
    nx = *reinterpret_cast<const float4*>(p.XL + int64_t(jr) * p.ldXL + f0);
  }
  for (int j = j0; j < j1; ++j) {
    const float4 x = nx;
    const int row = jr;
    const int jn = j + 1 < j1 ? j + 1 : j;
    jr = src_row(p, jn);
    nx = *reinterpret_cast<const float4*>(p.XL + int64_t(jr) * p.ldXL + f0);
    const float z[4] = {x.x + xr.x, x.y + xr.y, x.z + xr.z, x.w + xr.w};
    const float a4[4] = {at.x, at.y, at.z, at.w};
    const float g4[4] = {go.x, go.y, go.z, go.w};
    const float xv[4] = {x.x, x.y, x.z, x.w};
    float e = 0.f, da = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e = fmaf(leaky(z[k], slope), a4[k], e);
      da = fmaf(g4[k], xv[k], da);
    }
    e = wave_sum(e);
    da = wave_sum(da);
    const float alpha = __expf(e - M) * inv;
    const float de = alpha * (da - delta);
    float dxl[4], dz[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dz[k] = de * a4[k] * (z[k] > 0.f ? 1.f : slope);
      dxl[k] = fmaf(alpha, g4[k], dz[k]);
    }
    *reinterpret_cast<float4*>(p.dXL + int64_t(row) * p.ldDXL + f0) = make_float4(dxl[0], dxl[1], dxl[2], dxl[3]);
    dxr = make_float4(dxr.x + dz[0], dxr.y + dz[1], dxr.z + dz[2], dxr.w + dz[3]);
    dat = make_float4(fmaf(de, leaky(z[0], slope), dat.x), fmaf(de, leaky(z[1], slope), dat.y),
                      fmaf(de, leaky(z[2], slope), dat.z), fmaf(de, leaky(z[3], slope), dat.w));
  }
  float* slot = p.slots + int64_t(blk) * 2 * p.HC;
  st_sc1(slot + f0, dxr.x);
  st_sc1(slot + f0 + 1, dxr.y);
  st_sc1(slot + f0 + 2, dxr.z);
  st_sc1(slot + f0 + 3, dxr.w);
  st_sc1(slot + p.HC + f0, dat.x);
  st_sc1(slot + p.HC + f0 + 1, dat.y);
  st_sc1(slot + p.HC + f0 + 2, dat.z);
  st_sc1(slot + p.HC + f0 + 3, dat.w);
  (void)lane;
  done_bwd(p, blk, flag);
}

__device__ void bwd_points(const GaProb& p, int blk, float slope, uint32_t* flag) {
  __shared__ float4 SX[16][16], SD[16][16];
  const int ql = threadIdx.x >> 4, fq = threadIdx.x & 15, h = fq >> 2;
  const int f0 = 4 * fq;
  const int j0 = blk * kChunkP, j1 = min(p.S, j0 + kChunkP);
  const float4 xr = *reinterpret_cast<const float4*>(p.XR + f0);
  const float4 at = *reinterpret_cast<const float4*>(p.att + f0);
  const float4 go = *reinterpret_cast<const float4*>(p.gout + f0);
  const float4 o4 = *reinterpret_cast<const float4*>(p.out + f0);
  const float4 b4 = *reinterpret_cast<const float4*>(p.bias + f0);
  const float M = p.smax[h], inv = 1.f / (p.ssum[h] + 1e-16f);
  float delta = go.x * (o4.x - b4.x) + go.y * (o4.y - b4.y) + go.z * (o4.z - b4.z) + go.w * (o4.w - b4.w);
  delta += __shfl_xor(delta, 1);
  delta += __shfl_xor(delta, 2);
  const float a4[4] = {at.x, at.y, at.z, at.w};
  const float g4[4] = {go.x, go.y, go.z, go.w};
  float4 dxr = make_float4(0.f, 0.f, 0.f, 0.f), dat = dxr;
  constexpr int U = 4;
  for (int jb = j0 + ql; jb < j1; jb += 16 * U) {
    float4 x[U];
    int rows[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jb + 16 * u;
      rows[u] = src_row(p, j < j1 ? j : jb);
      x[u] = *reinterpret_cast<const float4*>(p.XL + int64_t(rows[u]) * p.ldXL + f0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float xv[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
      float z[4], e = 0.f, da = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z[k] = xv[k] + (k == 0 ? xr.x : k == 1 ? xr.y : k == 2 ? xr.z : xr.w);
        e = fmaf(leaky(z[k], slope), a4[k], e);
        da = fmaf(g4[k], xv[k], da);
      }
      e += __shfl_xor(e, 1);
      e += __shfl_xor(e, 2);
      da += __shfl_xor(da, 1);
      da += __shfl_xor(da, 2);
      if (jb + 16 * u < j1) {
        const float alpha = __expf(e - M) * inv;
        const float de = alpha * (da - delta);
        float dxl[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float dz = de * a4[k] * (z[k] > 0.f ? 1.f : slope);
          dxl[k] = fmaf(alpha, g4[k], dz);
          if (k == 0) dxr.x += dz, dat.x = fmaf(de, leaky(z[k], slope), dat.x);
          if (k == 1) dxr.y += dz, dat.y = fmaf(de, leaky(z[k], slope), dat.y);
          if (k == 2) dxr.z += dz, dat.z = fmaf(de, leaky(z[k], slope), dat.z);
          if (k == 3) dxr.w += dz, dat.w = fmaf(de, leaky(z[k], slope), dat.w);
        }
        *reinterpret_cast<float4*>(p.dXL + int64_t(rows[u]) * p.ldDXL + f0) =
            make_float4(dxl[0], dxl[1], dxl[2], dxl[3]);
      }
    }
  }
  SX[ql][fq] = dxr;
  SD[ql][fq] = dat;
  __syncthreads();
  float* slot = p.slots + int64_t(blk) * 2 * p.HC;
  if (threadIdx.x < 32) {  // 16 threads per half: the 16 source lanes summed in lane order
    const int q = threadIdx.x & 15, half = threadIdx.x >> 4;
    float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int l = 0; l < 16; ++l) {
      const float4 v = half ? SD[l][q] : SX[l][q];
      sum = make_float4(sum.x + v.x, sum.y + v.y, sum.z + v.z, sum.w + v.w);
    }
    float* d = slot + half * p.HC + 4 * q;
    st_sc1(d, sum.x);
    st_sc1(d + 1, sum.y);
    st_sc1(d + 2, sum.z);
    st_sc1(d + 3, sum.w);
  }
  done_bwd(p, blk, flag);
}

__global__ __launch_bounds__(kT) void gatt_bwd_kernel(GaArgs a) {
  __shared__ uint32_t flag;
  const int pi = find_prob(a);
  const GaProb& p = a.p[pi];
  const int blk = int(blockIdx.x) - p.blk0;
  if (p.C == 256)
    bwd_views(p, blk, a.slope, &flag);
  else
    bwd_points(p, blk, a.slope, &flag);
}

// ---- the camera-sharded block exchange (round 5): ONE all-gather of per-rank send blocks carries
// several payloads; these unpack it.  Rank r's block (blk floats) holds at roff its chunk own rows of
// width floats (rows past the scene's m are padding) and, at soff, a partial vector of sn floats.
struct Unpack {
  const float* G;    // [W, blk] gathered send blocks
  int64_t blk, roff, soff, ld_dst;
  float* rows_dst;   // [m, width] (row stride ld_dst) or null
  float* sum_dst;    // [sn] or null: the W partial vectors summed in rank order
  int W, chunk, width, m, sn;
};

__device__ __forceinline__ int unpack_units(const Unpack& u) {
  return (u.rows_dst ? u.m * (u.width / 4) : 0) + (u.sum_dst ? u.sn / 4 : 0);
}

// float4 unit k of the unpack: a row piece, then a piece of the rank-order sum
__device__ __forceinline__ void unpack_unit(const Unpack& u, int k) {
  const int nr = u.rows_dst ? u.m * (u.width / 4) : 0;
  if (k < nr) {
    const int w4 = u.width / 4, c = k / w4, q = k % w4;
    const float4 v = *reinterpret_cast<const float4*>(u.G + int64_t(c / u.chunk) * u.blk + u.roff +
                                                      int64_t(c % u.chunk) * u.width + 4 * q);
    *reinterpret_cast<float4*>(u.rows_dst + int64_t(c) * u.ld_dst + 4 * q) = v;
    return;
  }
  const int j = k - nr;
  float4 acc = *reinterpret_cast<const float4*>(u.G + u.soff + 4 * j);
  for (int r = 1; r < u.W; ++r) {
    const float4 v = *reinterpret_cast<const float4*>(u.G + int64_t(r) * u.blk + u.soff + 4 * j);
    acc = make_float4(acc.x + v.x, acc.y + v.y, acc.z + v.z, acc.w + v.w);
  }
  *reinterpret_cast<float4*>(u.sum_dst + 4 * j) = acc;
}

__global__ __launch_bounds__(kT) void exchange_unpack_kernel(Unpack u) {
  const int k = int(blockIdx.x) * kT + int(threadIdx.x);
  if (k < unpack_units(u)) unpack_unit(u, k);
}

// the sharded forward's second half: problem blockIdx.x's W gathered partial rows -> out / stats;
// blocks past nprob unpack the exchange's row payload (the view hub's SV | XR rows)
__global__ __launch_bounds__(kT) void gatt_merge_kernel(GaArgs a, Unpack u) {
  __shared__ float sc[16];
  if (int(blockIdx.x) < a.nprob) {
    merge_fwd(a.p[blockIdx.x], sc);
    return;
  }
  const int k = (int(blockIdx.x) - a.nprob) * kT + int(threadIdx.x);
  if (k < unpack_units(u)) unpack_unit(u, k);
}

int chunk_of(int C) { return C == 256 ? kChunkV : kChunkP; }

int groups_of(int nblk) { return nblk > kGroup ? (nblk + kGroup - 1) / kGroup : 1; }

int setup(const gasfm_gatt_prob* in, int nprob, float* scratch, uint32_t* counters, bool bwd, GaArgs& a) {
  a.nprob = nprob;
  int blocks = 0;
  float* ws = scratch;
  uint32_t* cn = counters;
  for (int q = 0; q < nprob; ++q) {
    const gasfm_gatt_prob& s = in[q];
    GaProb& p = a.p[q];
    p.XL = s.XL, p.ldXL = s.ldXL, p.src = s.src, p.XR = s.XR, p.att = s.att, p.bias = s.bias;
    p.out = s.out, p.smax = s.smax, p.ssum = s.ssum, p.part = s.part;
    p.gout = s.gout, p.dXL = s.dXL, p.ldDXL = s.ldDXL, p.dXR = s.dXR, p.datt = s.datt;
    p.S = s.S, p.HC = s.HC, p.C = s.HC / H;
    p.nblk = (s.S + chunk_of(p.C) - 1) / chunk_of(p.C);
    if (p.nblk < 1) p.nblk = 1;
    p.blk0 = blocks;
    p.slots = ws;
    p.sl = p.HC + 2 * H;
    const int64_t slot = bwd ? 2 * p.HC : p.HC + 2 * H;
    ws += int64_t(p.nblk) * slot;
    p.ngroups = groups_of(p.nblk);
    p.gslots = ws;
    if (p.ngroups > 1) ws += int64_t(p.ngroups) * slot;
    p.cnt = cn++;
    p.gcnt = cn;
    if (p.ngroups > 1) cn += p.ngroups;
    blocks += p.nblk;
  }
  for (int q = nprob; q < kMaxProb; ++q) a.p[q].blk0 = blocks;
  return blocks;
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

static int gatt_check(int32_t nprob, const gasfm_gatt_prob* probs, bool bwd) {
  GASFM_REQUIRE(nprob >= 1 && nprob <= kMaxProb && probs, "gasfm_gatt: nprob=%d", nprob);
  for (int q = 0; q < nprob; ++q) {
    const gasfm_gatt_prob& p = probs[q];
    GASFM_REQUIRE(p.HC == 4 * 256 || p.HC == 4 * 16, "gasfm_gatt: problem %d HC=%d (H = 4, C in {16, 256})", q, p.HC);
    GASFM_REQUIRE(p.S >= 0 && (p.XL || p.S == 0) && p.XR && p.att && p.bias && p.ldXL % 4 == 0 && (p.ldXL >= p.HC || p.S == 0),
                  "gasfm_gatt: problem %d S=%d / pointers / ldXL", q, p.S);
    GASFM_REQUIRE(aligned16(p.XL) && aligned16(p.XR) && aligned16(p.att) && aligned16(p.bias),
                  "gasfm_gatt: problem %d alignment", q);
    if (!bwd) {
      GASFM_REQUIRE(p.part || (p.out && p.smax && p.ssum), "gasfm_gatt_fwd: problem %d outputs", q);
    } else {
      GASFM_REQUIRE(p.gout && p.out && p.smax && p.ssum && (p.dXL || p.S == 0) && p.dXR && p.datt && p.ldDXL % 4 == 0 &&
                        (aligned16(p.dXL) || p.S == 0) && aligned16(p.gout) && aligned16(p.out) && aligned16(p.datt),
                    "gasfm_gatt_bwd: problem %d pointers", q);
    }
  }
  return GASFM_OK;
}

static int64_t nblk_of(const gasfm_gatt_prob& p) {
  const int C = p.HC / H;
  const int64_t nblk = (p.S + chunk_of(C) - 1) / chunk_of(C);
  return nblk < 1 ? 1 : nblk;
}

extern "C" int64_t gasfm_gatt_scratch_floats(int32_t nprob, const gasfm_gatt_prob* probs) {
  int64_t n = 0;
  for (int q = 0; q < nprob; ++q) {
    const int64_t nblk = nblk_of(probs[q]), ng = groups_of(int(nblk));
    n += (nblk + (ng > 1 ? ng : 0)) * (2 * int64_t(probs[q].HC) + 2 * H);
  }
  return n + 16;
}

extern "C" int32_t gasfm_gatt_counters(int32_t nprob, const gasfm_gatt_prob* probs) {
  int32_t n = 0;
  for (int q = 0; q < nprob; ++q) {
    const int ng = groups_of(int(nblk_of(probs[q])));
    n += 1 + (ng > 1 ? ng : 0);
  }
  return n;
}

extern "C" int gasfm_gatt_fwd(int32_t nprob, const gasfm_gatt_prob* probs, float slope, float* scratch,
                              uint32_t* counters, void* stream) {
  const int s0 = gatt_check(nprob, probs, false);
  if (s0 != GASFM_OK) return s0;
  GASFM_REQUIRE(scratch && counters, "gasfm_gatt_fwd: scratch / counters");
  GaArgs a{};
  a.slope = slope;
  const int blocks = setup(probs, nprob, scratch, counters, false, a);
  hipLaunchKernelGGL(gatt_fwd_kernel, dim3(blocks), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream), a);
  return launch_status("gasfm_gatt_fwd");
}

static int unpack_check(const Unpack& u, const char* who) {
  GASFM_REQUIRE(u.G && u.W >= 1 && u.blk % 4 == 0 && u.roff % 4 == 0 && u.soff % 4 == 0 && u.width % 4 == 0 &&
                    u.ld_dst % 4 == 0 && u.sn % 4 == 0 && u.m >= 0 && u.chunk >= 1 && u.m <= int64_t(u.W) * u.chunk &&
                    aligned16(u.G) && aligned16(u.rows_dst) && aligned16(u.sum_dst) &&
                    (!u.rows_dst || (u.roff + int64_t(u.chunk) * u.width <= u.blk && u.ld_dst >= u.width)) &&
                    (!u.sum_dst || u.soff + u.sn <= u.blk),
                "%s: W=%d blk=%lld roff=%lld chunk=%d width=%d m=%d soff=%lld sn=%d (layout / alignment)", who, u.W,
                (long long)u.blk, (long long)u.roff, u.chunk, u.width, u.m, (long long)u.soff, u.sn);
  return GASFM_OK;
}

static Unpack make_unpack(const float* G, int32_t W, int64_t blk, int64_t roff, int32_t chunk, int32_t width, int32_t m,
                          float* rows_dst, int64_t ld_dst, int64_t soff, int32_t sn, float* sum_dst) {
  Unpack u;
  u.G = G, u.blk = blk, u.roff = roff, u.soff = soff, u.ld_dst = ld_dst;
  u.rows_dst = rows_dst, u.sum_dst = sum_dst;
  u.W = W, u.chunk = chunk, u.width = width, u.m = m, u.sn = sn;
  return u;
}

extern "C" int gasfm_exchange_unpack(const float* G, int32_t W, int64_t blk, int64_t roff, int32_t chunk,
                                     int32_t width, int32_t m, float* rows_dst, int64_t ld_dst, int64_t soff,
                                     int32_t sn, float* sum_dst, void* stream) {
  const Unpack u = make_unpack(G, W, blk, roff, chunk, width, m, rows_dst, ld_dst, soff, sn, sum_dst);
  const int s0 = unpack_check(u, "gasfm_exchange_unpack");
  if (s0 != GASFM_OK) return s0;
  const int units = (rows_dst ? m * (width / 4) : 0) + (sum_dst ? sn / 4 : 0);
  if (units == 0) return GASFM_OK;
  hipLaunchKernelGGL(exchange_unpack_kernel, dim3((units + kT - 1) / kT), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), u);
  return launch_status("gasfm_exchange_unpack");
}

static int merge_launch(int32_t nprob, const gasfm_gatt_prob* probs, int32_t nrows, int64_t stride, const Unpack& u,
                        void* stream);

extern "C" int gasfm_gatt_merge(int32_t nprob, const gasfm_gatt_prob* probs, int32_t nrows, int64_t stride,
                                void* stream) {
  Unpack u{};
  return merge_launch(nprob, probs, nrows, stride, u, stream);
}

extern "C" int gasfm_gatt_merge_unpack(int32_t nprob, const gasfm_gatt_prob* probs, int32_t nrows, int64_t stride,
                                       const float* G, int32_t W, int64_t blk, int64_t roff, int32_t chunk,
                                       int32_t width, int32_t m, float* rows_dst, int64_t ld_dst, void* stream) {
  GASFM_REQUIRE(rows_dst, "gasfm_gatt_merge_unpack: rows_dst");
  const Unpack u = make_unpack(G, W, blk, roff, chunk, width, m, rows_dst, ld_dst, 0, 0, nullptr);
  const int s0 = unpack_check(u, "gasfm_gatt_merge_unpack");
  if (s0 != GASFM_OK) return s0;
  return merge_launch(nprob, probs, nrows, stride, u, stream);
}

static int merge_launch(int32_t nprob, const gasfm_gatt_prob* probs, int32_t nrows, int64_t stride, const Unpack& u,
                        void* stream) {
  GASFM_REQUIRE(nprob >= 1 && nprob <= kMaxProb && probs && nrows >= 1, "gasfm_gatt_merge: nprob=%d nrows=%d", nprob,
                nrows);
  GaArgs a{};
  a.nprob = nprob;
  for (int q = 0; q < nprob; ++q) {
    const gasfm_gatt_prob& s = probs[q];
    GASFM_REQUIRE((s.HC == 1024 || s.HC == 64) && s.part && s.bias && s.out && s.smax && s.ssum &&
                      stride >= s.HC + 2 * H,
                  "gasfm_gatt_merge: problem %d HC=%d / pointers / stride", q, s.HC);
    GaProb& p = a.p[q];
    p.HC = s.HC, p.C = s.HC / H, p.bias = s.bias, p.out = s.out, p.smax = s.smax, p.ssum = s.ssum;
    p.part = nullptr;
    p.slots = const_cast<float*>(s.part);
    p.sl = stride;
    p.nblk = nrows;
    p.ngroups = 1;
  }
  const int units = u.G ? (u.rows_dst ? u.m * (u.width / 4) : 0) + (u.sum_dst ? u.sn / 4 : 0) : 0;
  hipLaunchKernelGGL(gatt_merge_kernel, dim3(nprob + (units + kT - 1) / kT), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), a, u);
  return launch_status("gasfm_gatt_merge");
}

extern "C" int gasfm_gatt_bwd(int32_t nprob, const gasfm_gatt_prob* probs, float slope, float* scratch,
                              uint32_t* counters, void* stream) {
  const int s0 = gatt_check(nprob, probs, true);
  if (s0 != GASFM_OK) return s0;
  GASFM_REQUIRE(scratch && counters, "gasfm_gatt_bwd: scratch / counters");
  GaArgs a{};
  a.slope = slope;
  const int blocks = setup(probs, nprob, scratch, counters, true, a);
  hipLaunchKernelGGL(gatt_bwd_kernel, dim3(blocks), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream), a);
  return launch_status("gasfm_gatt_bwd");
}
