// Fused GATv2 edge-softmax + aggregation, forward and backward, for gfx950.
//
// Replaces PyG GATv2Conv's message()/utils.softmax/scatter-'add' sequence as
// used by the reference (code/models/layers.py:329-335, 426-432, 550-556,
// 566-572): instead of materialising [E,H,C] intermediates and running
// scatter-max / scatter-sum / scatter-add with float atomics, one wavefront
// streams the edges of one destination segment (or of one piece of a long
// segment) once, computes the GATv2 logits in registers, keeps an online
// (max, sum, acc) softmax state per head and writes the destination row.
//
// Wave layout (64 lanes): every edge row of HC = H*C floats is spread over
// LPE = HC/VEC lanes holding VEC consecutive floats (16-byte loads); a wave
// holds EPR = 64/LPE edge rows side by side and U such row-groups in flight
// per step.  Per-head logits need a reduction over LPH = C/VEC lanes (or none
// when a lane holds several whole heads); the EPR row states are merged with
// xor-shuffles at the end of the item.
//
//   HC=32 (C=8, the 12/9 main blocks):    VEC 4, LPE 8,  EPR 8,  U 4 -> 32 edges/step
//   HC=4  (C=1, block 0):                 VEC 4, LPE 1,  EPR 64, U 2
//   HC=64 (C=16, scenepoint->global):     VEC 4, LPE 16, EPR 4,  U 4
//   HC=1024 (C=256, view->global):        VEC 16, LPE 64, EPR 1, U 2
// Other (H, C) combinations run the generic kernel at the bottom (still HIP).
//
// Determinism: no atomics; split segments go through ordered combine passes.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>
#include <cmath>

#include "common.hpp"
#include "lanes.hpp"

namespace gasfm {

constexpr int kWave = 64;
constexpr int kBlock = 256;

__device__ __forceinline__ float leaky(float z, float slope) { return z > 0.f ? z : z * slope; }

template <int HC_, int C_>
struct Geom {
  static constexpr int HC = HC_;
  static constexpr int C = C_;
  static constexpr int H = HC / C;
  static constexpr int VEC = (HC / kWave > 4) ? HC / kWave : 4;
  static constexpr int LPE = HC / VEC;
  static constexpr int EPR = kWave / LPE;
  static constexpr int HPL = (C >= VEC) ? 1 : VEC / C;  // heads held by one lane
  static constexpr int LPH = (C >= VEC) ? C / VEC : 1;  // lanes sharing one head
  static constexpr int CPH = (C >= VEC) ? VEC : C;      // lane floats per held head
  static constexpr int U = (VEC == 4) ? ((EPR >= 64) ? 2 : 4) : (VEC == 8 ? 2 : 1);
  static_assert(HC % VEC == 0 && kWave % LPE == 0, "bad geometry");
  static_assert(LPE * EPR == kWave, "bad geometry");
};

template <int N>
__device__ __forceinline__ void load_vec(float (&d)[N], const float* p) {
#pragma unroll
  for (int k = 0; k < N / 4; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(p + 4 * k);
    d[4 * k + 0] = v.x;
    d[4 * k + 1] = v.y;
    d[4 * k + 2] = v.z;
    d[4 * k + 3] = v.w;
  }
}

template <int N>
__device__ __forceinline__ void store_vec(float* p, const float (&d)[N]) {
#pragma unroll
  for (int k = 0; k < N / 4; ++k)
    *reinterpret_cast<float4*>(p + 4 * k) = make_float4(d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]);
}

// Sum over the LPH lanes that share a head (lanes are contiguous within an edge row).
template <int LPH>
__device__ __forceinline__ float head_sum(float v) {
  return group_sum<LPH>(v);
}

__device__ __forceinline__ float safe_scale(float m_old, float m_new) {
  // exp(m_old - m_new) with the empty-state convention (both -inf -> 0).
  return (m_new == -INFINITY) ? 0.f : __expf(m_old - m_new);
}

// Merge partner state (m2, s2, a2) into (m, s, a) for the HPL heads of a lane.
template <class G>
__device__ __forceinline__ void merge_state(float (&m)[G::HPL], float (&s)[G::HPL], float (&a)[G::VEC],
                                            const float (&m2)[G::HPL], const float (&s2)[G::HPL],
                                            const float (&a2)[G::VEC]) {
#pragma unroll
  for (int hh = 0; hh < G::HPL; ++hh) {
    const float mn = fmaxf(m[hh], m2[hh]);
    const float f1 = safe_scale(m[hh], mn), f2 = safe_scale(m2[hh], mn);
    s[hh] = s[hh] * f1 + s2[hh] * f2;
#pragma unroll
    for (int c = 0; c < G::CPH; ++c) a[hh * G::CPH + c] = a[hh * G::CPH + c] * f1 + a2[hh * G::CPH + c] * f2;
    m[hh] = mn;
  }
}

// Combine the EPR row states of a wave (xor over the row bits of the lane id).
template <class G, int O>
__device__ __forceinline__ void reduce_rows_step(float (&m)[G::HPL], float (&s)[G::HPL], float (&a)[G::VEC]) {
  if constexpr (O < kWave) {
    if constexpr (O >= G::LPE) {
      float m2[G::HPL], s2[G::HPL], a2[G::VEC];
#pragma unroll
      for (int hh = 0; hh < G::HPL; ++hh) {
        m2[hh] = xor_lane<O>(m[hh]);
        s2[hh] = xor_lane<O>(s[hh]);
      }
#pragma unroll
      for (int v = 0; v < G::VEC; ++v) a2[v] = xor_lane<O>(a[v]);
      merge_state<G>(m, s, a, m2, s2, a2);
    }
    reduce_rows_step<G, 2 * O>(m, s, a);
  }
}
template <class G>
__device__ __forceinline__ void reduce_rows(float (&m)[G::HPL], float (&s)[G::HPL], float (&a)[G::VEC]) {
  reduce_rows_step<G, 1>(m, s, a);
}

__device__ __forceinline__ int wave_id_uniform() {
  return __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) / kWave);
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
#ifndef GASFM_FWD_LOOKAHEAD
#define GASFM_FWD_LOOKAHEAD 0
#endif
#ifndef GASFM_FWD_MINWAVES
#define GASFM_FWD_MINWAVES 1
#endif
constexpr bool kFwdLookahead = GASFM_FWD_LOOKAHEAD != 0;

template <class G>
__global__ __launch_bounds__(kBlock, GASFM_FWD_MINWAVES) void attn_fwd_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, float slope, int finalize,
    float* __restrict__ out, int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  constexpr int LDP = G::HC + 2 * G::H;  // packed partial row: [acc HC | max H | sum H]
  const int lane = threadIdx.x & (kWave - 1);
  const int row = lane / G::LPE;
  const int li = lane % G::LPE;
  const int f0 = li * G::VEC;
  const int nwaves = gridDim.x * (blockDim.x / kWave);

  float attv[G::VEC];
  load_vec<G::VEC>(attv, att + f0);

  // Chunk = EPR*U consecutive edges of an item (row `row` of the wave takes u*EPR + row).
  auto load_chunk = [&](int e0, int end, float (&xl)[G::U][G::VEC], bool (&valid)[G::U]) {
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const int e = e0 + u * G::EPR + row;
      valid[u] = e < end;
      if (valid[u]) {
        const int64_t src = perm ? int64_t(perm[e]) : int64_t(e);
        load_vec<G::VEC>(xl[u], XL + src * ldXL + f0);
      } else {
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) xl[u][v] = 0.f;
      }
    }
  };

  // One-item lookahead: the next item's XR row and first chunk are requested before the
  // current item is reduced and stored, so every wave keeps loads in flight across items
  // (point segments average ~20 edges: one chunk per item).
  int it = wave_id_uniform();
  gasfm_work_item wn{0, 0, 0, -1};
  float xrn[G::VEC], xln[G::U][G::VEC];
  bool validn[G::U];
  if (kFwdLookahead && it < n_items) {
    wn = items[it];
    load_vec<G::VEC>(xrn, XR + int64_t(wn.seg) * ldXR + f0);
    load_chunk(wn.begin, wn.end, xln, validn);
  }
  for (; it < n_items; it += nwaves) {
    gasfm_work_item w;
    float xr[G::VEC], xl[G::U][G::VEC];
    bool valid[G::U];
    if constexpr (kFwdLookahead) {
      w = wn;
#pragma unroll
      for (int v = 0; v < G::VEC; ++v) xr[v] = xrn[v];
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        valid[u] = validn[u];
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) xl[u][v] = xln[u][v];
      }
      if (it + nwaves < n_items) {
        wn = items[it + nwaves];
        load_vec<G::VEC>(xrn, XR + int64_t(wn.seg) * ldXR + f0);
        load_chunk(wn.begin, wn.end, xln, validn);
      }
    } else {
      w = items[it];
      load_vec<G::VEC>(xr, XR + int64_t(w.seg) * ldXR + f0);
    }

    float m[G::HPL], s[G::HPL], acc[G::VEC];
#pragma unroll
    for (int hh = 0; hh < G::HPL; ++hh) {
      m[hh] = -INFINITY;
      s[hh] = 0.f;
    }
#pragma unroll
    for (int v = 0; v < G::VEC; ++v) acc[v] = 0.f;

    for (int e0 = w.begin; e0 < w.end; e0 += G::EPR * G::U) {
      if (!kFwdLookahead || e0 != w.begin) load_chunk(e0, w.end, xl, valid);
      // logits for the U rows, per held head
      float lg[G::U][G::HPL];
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
#pragma unroll
        for (int hh = 0; hh < G::HPL; ++hh) {
          float p = 0.f;
#pragma unroll
          for (int c = 0; c < G::CPH; ++c) {
            const int v = hh * G::CPH + c;
            p = fmaf(leaky(xl[u][v] + xr[v], slope), attv[v], p);
          }
          p = head_sum<G::LPH>(p);
          lg[u][hh] = valid[u] ? p : -INFINITY;
        }
      }
      // online softmax update with one rescale per step
#pragma unroll
      for (int hh = 0; hh < G::HPL; ++hh) {
        float cm = lg[0][hh];
#pragma unroll
        for (int u = 1; u < G::U; ++u) cm = fmaxf(cm, lg[u][hh]);
        const float mn = fmaxf(m[hh], cm);
        const float f = safe_scale(m[hh], mn);
        float ssum = s[hh] * f;
        float a[G::CPH];
#pragma unroll
        for (int c = 0; c < G::CPH; ++c) a[c] = acc[hh * G::CPH + c] * f;
#pragma unroll
        for (int u = 0; u < G::U; ++u) {
          const float p = (lg[u][hh] == -INFINITY) ? 0.f : __expf(lg[u][hh] - mn);
          ssum += p;
#pragma unroll
          for (int c = 0; c < G::CPH; ++c) a[c] = fmaf(p, xl[u][hh * G::CPH + c], a[c]);
        }
        s[hh] = ssum;
#pragma unroll
        for (int c = 0; c < G::CPH; ++c) acc[hh * G::CPH + c] = a[c];
        m[hh] = mn;
      }
    }
    reduce_rows<G>(m, s, acc);

    if (row == 0) {
      const bool head_leader = (li % G::LPH) == 0;
      const int h0 = (f0 / G::C);  // first head held by this lane
      if (w.slot < 0) {
        float o[G::VEC];
#pragma unroll
        for (int hh = 0; hh < G::HPL; ++hh) {
          const float inv = 1.f / (s[hh] + 1e-16f);
#pragma unroll
          for (int c = 0; c < G::CPH; ++c) {
            const int v = hh * G::CPH + c;
            o[v] = finalize ? fmaf(acc[v], inv, bias[f0 + v]) : acc[v];
          }
        }
        store_vec<G::VEC>(out + int64_t(w.seg) * ldOut + f0, o);
        if (head_leader) {
#pragma unroll
          for (int hh = 0; hh < G::HPL; ++hh) {
            seg_max[int64_t(w.seg) * ldStat + h0 + hh] = m[hh];
            seg_sum[int64_t(w.seg) * ldStat + h0 + hh] = s[hh];
          }
        }
      } else {
        float* pr = part + int64_t(w.slot) * LDP;
        store_vec<G::VEC>(pr + f0, acc);
        if (head_leader) {
#pragma unroll
          for (int hh = 0; hh < G::HPL; ++hh) {
            pr[G::HC + h0 + hh] = m[hh];
            pr[G::HC + G::H + h0 + hh] = s[hh];
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// forward, XL streamed in segment order (perm == NULL) with direct-to-LDS prefetch.
// Each wave owns a 5 KB LDS buffer: rows 0..31 of its item (8 lanes x 16 B per row, the image
// is the lanes' load order, global_load_lds) + the XR row.  Per item: wait, copy the buffer to
// registers, issue the NEXT item's rows into the same buffer (no VGPRs held while they fly),
// then compute.  Items are wave-uniform scalar loads and no ordinary vector load is consumed
// while the prefetch is in flight (hipcc would drain it with vmcnt(0)), except the extra
// chunks of segments longer than 32 edges.  Geom<32,8> (the 32-wide convs) only.
// ------------------------------------------------------------------------------------------
#ifndef GASFM_GLDS_BWD_MINWAVES
#define GASFM_GLDS_BWD_MINWAVES 1
#endif
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef const __attribute__((address_space(1))) void* glb_vptr;

template <class G>
__global__ __launch_bounds__(kBlock) void attn_fwd_glds_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const gasfm_work_item* __restrict__ items,
    int n_items, float slope, int finalize, float* __restrict__ out, int64_t ldOut, float* __restrict__ seg_max,
    float* __restrict__ seg_sum, int64_t ldStat, float* __restrict__ part) {
  static_assert(G::VEC == 4 && G::LPE == 8 && G::EPR == 8 && G::U == 4 && G::HPL == 1, "Geom<32,8> only");
  constexpr int LDP = G::HC + 2 * G::H;
  __shared__ float4 lbuf[kBlock / kWave][5 * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int row = lane / G::LPE;
  const int li = lane % G::LPE;
  const int f0 = li * G::VEC;
  const int nwaves = gridDim.x * (blockDim.x / kWave);
  float4* B = lbuf[threadIdx.x / kWave];
  float attv[G::VEC], bv[G::VEC];  // in registers: no vector load inside the prefetch span
  load_vec<G::VEC>(attv, att + f0);
  if (finalize) load_vec<G::VEC>(bv, bias + f0);
  auto issue = [&](const gasfm_work_item& w) {  // empty items issue nothing (their loop never runs)
    if (w.begin >= w.end) return;
    const int64_t safe = w.begin;
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const int64_t e = w.begin + u * G::EPR + row;
      const float* src = XL + (e < w.end ? e : safe) * ldXL + f0;
      __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(B + u * kWave), 16, 0, 0);
    }
    __builtin_amdgcn_global_load_lds((glb_vptr)(XR + int64_t(w.seg) * ldXR + f0), (lds_vptr)(B + 4 * kWave), 16,
                                     0, 0);
  };
  int it = wave_id_uniform();
  gasfm_work_item wn{0, 0, 0, -1};
  if (it < n_items) {
    wn = items[it];
    issue(wn);
  }
  for (; it < n_items; it += nwaves) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float xl[G::U][G::VEC], xr[G::VEC];
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const float4 v = B[u * kWave + lane];
      xl[u][0] = v.x;
      xl[u][1] = v.y;
      xl[u][2] = v.z;
      xl[u][3] = v.w;
    }
    {
      const float4 v = B[4 * kWave + lane];
      xr[0] = v.x;
      xr[1] = v.y;
      xr[2] = v.z;
      xr[3] = v.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const gasfm_work_item w = wn;
    if (it + nwaves < n_items) {
      wn = items[it + nwaves];
      issue(wn);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issue ahead of this item's compute
    float m = -INFINITY, ssum = 0.f, acc[G::VEC] = {0.f, 0.f, 0.f, 0.f};
    auto chunk = [&](int e0) {
      bool valid[G::U];
#pragma unroll
      for (int u = 0; u < G::U; ++u) valid[u] = e0 + u * G::EPR + row < w.end;
      float lg[G::U];
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        float p = 0.f;
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) p = fmaf(leaky(xl[u][v] + xr[v], slope), attv[v], p);
        p = head_sum<G::LPH>(p);
        lg[u] = valid[u] ? p : -INFINITY;
      }
      float cm = lg[0];
#pragma unroll
      for (int u = 1; u < G::U; ++u) cm = fmaxf(cm, lg[u]);
      const float mn = fmaxf(m, cm);
      const float f = safe_scale(m, mn);
      ssum *= f;
#pragma unroll
      for (int v = 0; v < G::VEC; ++v) acc[v] *= f;
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        const float pe = (lg[u] == -INFINITY) ? 0.f : __expf(lg[u] - mn);
        ssum += pe;
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) acc[v] = fmaf(pe, xl[u][v], acc[v]);
      }
      m = mn;
    };
    // first chunk straight from the prefetched registers: no vector-memory wait on this path
    if (w.begin < w.end) chunk(w.begin);
    // segments longer than 32 edges: further chunks with plain loads (these drain the prefetch)
    for (int e0 = w.begin + G::EPR * G::U; e0 < w.end; e0 += G::EPR * G::U) {
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        const int e = e0 + u * G::EPR + row;
        load_vec<G::VEC>(xl[u], XL + int64_t(e < w.end ? e : e0) * ldXL + f0);
      }
      chunk(e0);
    }
    float mm[1] = {m}, ss[1] = {ssum};
    reduce_rows<G>(mm, ss, acc);
    if (row == 0) {
      const bool head_leader = (li % G::LPH) == 0;
      const int h0 = f0 / G::C;
      if (w.slot < 0) {
        float o[G::VEC];
        const float inv = 1.f / (ss[0] + 1e-16f);
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) o[v] = finalize ? fmaf(acc[v], inv, bv[v]) : acc[v];
        store_vec<G::VEC>(out + int64_t(w.seg) * ldOut + f0, o);
        if (head_leader) {
          seg_max[int64_t(w.seg) * ldStat + h0] = mm[0];
          seg_sum[int64_t(w.seg) * ldStat + h0] = ss[0];
        }
      } else {
        float* pr = part + int64_t(w.slot) * LDP;
        store_vec<G::VEC>(pr + f0, acc);
        if (head_leader) {
          pr[G::HC + h0] = mm[0];
          pr[G::HC + G::H + h0] = ss[0];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// forward, grouped items (Geom<32,8>, XL streamed in segment order, perm == NULL).
// A wave task is 8 consecutive work items; lane group g (8 lanes = one 128-B edge row) owns
// item g of the task and walks its edges U rows per iteration, keeping the segment's online
// softmax state in its own lanes: no cross-row merge per item (the row-parallel kernels above
// spend ~a chunk's worth of shuffles and exps merging 8 row states per item), and the 8 output
// rows of a task are stored side by side.  Short point segments (~20 edges) then run at
// ~(mean / padded max) lane occupancy instead of 20/32, with no per-item tail.
// Pipelining: every iteration waits for its rows, issues the NEXT iteration's U rows (or, at
// the last iteration of a task, the next task's first rows and XR rows), then computes.
// S > 1 (round 6, small shards): S lane groups share an item -- group s of the item takes rows
// k + s U .. k + s U + U - 1 of each S U-row step -- so a task holds 8 / S items, the grid S times
// the waves, and a wave's dependent chain of row round trips is S times shorter; the S online
// softmax states merge by an xor butterfly over the groups at the item's end (group 0 stores).
// A rank-of-8 point shard (25k points) is ~3k tasks at S = 1: 12 waves per CU, each walking ~8
// round trips, i.e. latency-bound.
// ------------------------------------------------------------------------------------------
template <int U, int MINW, int S>
__global__ __launch_bounds__(kBlock, MINW) void attn_fwd_grp_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const gasfm_work_item* __restrict__ items,
    int n_items, float slope, int finalize, float* __restrict__ out, int64_t ldOut, float* __restrict__ seg_max,
    float* __restrict__ seg_sum, int64_t ldStat, float* __restrict__ part) {
  static_assert(S == 1 || S == 2 || S == 4, "lane groups per item");
  constexpr int HC = 32, H = 4, C = 8, LDP = HC + 2 * H, GR = 8 / S, STEP = U * S;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = (lane >> 3) / S, sub = (lane >> 3) % S, li = lane & 7, f0 = li * 4, h = f0 / C;
  const int nwaves = gridDim.x * (blockDim.x / kWave);
  const int ntasks = (n_items + GR - 1) / GR;
  float attv[4], bv[4] = {0.f, 0.f, 0.f, 0.f};
  load_vec<4>(attv, att + f0);
  if (finalize) load_vec<4>(bv, bias + f0);

  auto item_of = [&](int t) {
    const int i = t * GR + g;
    gasfm_work_item w{-1, 0, 0, -1};
    if (t < ntasks && i < n_items) w = items[i];
    return w;
  };
  auto wave_max_len = [&](const gasfm_work_item& w) {
    int l = w.end - w.begin;
    l = max(l, __shfl_xor(l, 8));
    l = max(l, __shfl_xor(l, 16));
    l = max(l, __shfl_xor(l, 32));
    return __builtin_amdgcn_readfirstlane(l);
  };
  auto issue = [&](const gasfm_work_item& w, int k, float (&x)[U][4]) {
    const int64_t base = w.begin < w.end ? w.begin : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = int64_t(w.begin) + k + sub * U + u;
      load_vec<4>(x[u], XL + (r < w.end ? r : base) * ldXL + f0);
    }
  };

  int t = wave_id_uniform();
  if (t >= ntasks) return;
  gasfm_work_item w = item_of(t);
  int L = wave_max_len(w);
  float xr[4] = {0.f, 0.f, 0.f, 0.f}, nx[U][4];
  if (w.seg >= 0) load_vec<4>(xr, XR + int64_t(w.seg) * ldXR + f0);
  if (L > 0) issue(w, 0, nx);
  for (; t < ntasks; t += nwaves) {
    const gasfm_work_item wn = item_of(t + nwaves);  // consumed at this task's last iteration
    int Ln = 0;
    float xrn[4] = {0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, ssum = 0.f, acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int len = w.end - w.begin;
    for (int k = 0; k < L; k += STEP) {
      float xl[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) xl[u][v] = nx[u][v];
      if (k + STEP < L) {
        issue(w, k + STEP, nx);
      } else {  // last iteration of this task: start the next one
        Ln = wave_max_len(wn);
        if (wn.seg >= 0) load_vec<4>(xrn, XR + int64_t(wn.seg) * ldXR + f0);
        if (Ln > 0) issue(wn, 0, nx);
      }
      float lg[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float p = 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) p = fmaf(leaky(xl[u][v] + xr[v], slope), attv[v], p);
        p += xor_lane<1>(p);  // the 2 lanes of a head
        lg[u] = (k + sub * U + u < len) ? p : -INFINITY;
      }
      float cm = lg[0];
#pragma unroll
      for (int u = 1; u < U; ++u) cm = fmaxf(cm, lg[u]);
      const float mn = fmaxf(m, cm);
      const float f = safe_scale(m, mn);
      ssum *= f;
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[v] *= f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float pe = (lg[u] == -INFINITY) ? 0.f : __expf(lg[u] - mn);
        ssum += pe;
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[v] = fmaf(pe, xl[u][v], acc[v]);
      }
      m = mn;
    }
    if (L == 0) {  // every item of the task empty: the next task was not started above
      Ln = wave_max_len(wn);
      if (wn.seg >= 0) load_vec<4>(xrn, XR + int64_t(wn.seg) * ldXR + f0);
      if (Ln > 0) issue(wn, 0, nx);
    }
    if constexpr (S > 1) {  // the item's S group states, butterfly over the group bits of the lane id
#pragma unroll
      for (int o = 8; o < 8 * S; o *= 2) {
        const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(ssum, o);
        float a2[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) a2[v] = __shfl_xor(acc[v], o);
        const float mn = fmaxf(m, m2);
        const float f1 = safe_scale(m, mn), f2 = safe_scale(m2, mn);
        ssum = ssum * f1 + s2 * f2;
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[v] = acc[v] * f1 + a2[v] * f2;
        m = mn;
      }
    }
    if (w.seg >= 0 && sub == 0) {
      const bool head_leader = (li & 1) == 0;
      if (w.slot < 0) {
        float o[4];
        const float inv = 1.f / (ssum + 1e-16f);
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v] = finalize ? fmaf(acc[v], inv, bv[v]) : acc[v];
        store_vec<4>(out + int64_t(w.seg) * ldOut + f0, o);
        if (head_leader) {
          seg_max[int64_t(w.seg) * ldStat + h] = m;
          seg_sum[int64_t(w.seg) * ldStat + h] = ssum;
        }
      } else {
        float* pr = part + int64_t(w.slot) * LDP;
        store_vec<4>(pr + f0, acc);
        if (head_leader) {
          pr[HC + h] = m;
          pr[HC + H + h] = ssum;
        }
      }
    }
    w = wn;
    L = Ln;
#pragma unroll
    for (int v = 0; v < 4; ++v) xr[v] = xrn[v];
  }
}

// Ordered merge of partial states.  One workgroup per combine entry; rows of
// the workgroup take slots k = row, row + R, ... in order and the row states
// are merged in row order (first within a wave, then across waves via LDS),
// so the summation order is fixed for a given launch geometry.
template <class G>
__global__ __launch_bounds__(1024) void attn_combine_kernel(
    const gasfm_combine_item* __restrict__ comb, const float* __restrict__ part,
    const float* __restrict__ bias, int finalize, float* __restrict__ out, int64_t ldOut,
    float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int LDP = G::HC + 2 * G::H;
  const gasfm_combine_item ci = comb[blockIdx.x];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  const int li = lane % G::LPE;
  const int f0 = li * G::VEC;
  const int grow = threadIdx.x / G::LPE;  // global row id in the workgroup
  const int R = blockDim.x / G::LPE;
  const int h0 = f0 / G::C;

  float m[G::HPL], s[G::HPL], a[G::VEC];
#pragma unroll
  for (int hh = 0; hh < G::HPL; ++hh) {
    m[hh] = -INFINITY;
    s[hh] = 0.f;
  }
#pragma unroll
  for (int v = 0; v < G::VEC; ++v) a[v] = 0.f;

  for (int k = grow; k < ci.slot_count; k += R) {
    const int64_t slot = int64_t(ci.slot_begin) + int64_t(k) * ci.slot_stride;
    float m2[G::HPL], s2[G::HPL], a2[G::VEC];
#pragma unroll
    for (int hh = 0; hh < G::HPL; ++hh) {
      m2[hh] = part[slot * LDP + G::HC + h0 + hh];
      s2[hh] = part[slot * LDP + G::HC + G::H + h0 + hh];
    }
    load_vec<G::VEC>(a2, part + slot * LDP + f0);
    merge_state<G>(m, s, a, m2, s2, a2);
  }
  reduce_rows<G>(m, s, a);
  // cross-wave merge through LDS: wave w's row-0 lanes publish their state
  constexpr int ST = G::VEC + 2 * G::HPL;
  const int row_in_wave = lane / G::LPE;
  if (row_in_wave == 0) {
    float* p = lds + (wv * G::LPE + li) * ST;
#pragma unroll
    for (int v = 0; v < G::VEC; ++v) p[v] = a[v];
#pragma unroll
    for (int hh = 0; hh < G::HPL; ++hh) {
      p[G::VEC + hh] = m[hh];
      p[G::VEC + G::HPL + hh] = s[hh];
    }
  }
  __syncthreads();
  if (wv == 0 && row_in_wave == 0) {
    for (int w2 = 1; w2 < nw; ++w2) {
      const float* p = lds + (w2 * G::LPE + li) * ST;
      float m2[G::HPL], s2[G::HPL], a2[G::VEC];
#pragma unroll
      for (int v = 0; v < G::VEC; ++v) a2[v] = p[v];
#pragma unroll
      for (int hh = 0; hh < G::HPL; ++hh) {
        m2[hh] = p[G::VEC + hh];
        s2[hh] = p[G::VEC + G::HPL + hh];
      }
      merge_state<G>(m, s, a, m2, s2, a2);
    }
    float o[G::VEC];
#pragma unroll
    for (int hh = 0; hh < G::HPL; ++hh) {
      const float inv = 1.f / (s[hh] + 1e-16f);
#pragma unroll
      for (int c = 0; c < G::CPH; ++c) {
        const int v = hh * G::CPH + c;
        o[v] = finalize ? fmaf(a[v], inv, bias[f0 + v]) : a[v];
      }
    }
    store_vec<G::VEC>(out + int64_t(ci.seg) * ldOut + f0, o);
    if ((li % G::LPH) == 0) {
#pragma unroll
      for (int hh = 0; hh < G::HPL; ++hh) {
        seg_max[int64_t(ci.seg) * ldStat + h0 + hh] = m[hh];
        seg_sum[int64_t(ci.seg) * ldStat + h0 + hh] = s[hh];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward
//   alpha_j = exp(e_j - M) / (S + 1e-16)          (M, S: the forward's final stats)
//   delta   = sum_c g_c (out - bias)_c             (= sum_j alpha_j * dalpha_j)
//   dalpha_j = sum_c g_c XL_jc ;  de_j = alpha_j (dalpha_j - delta)
//   dz_j = de_j * att * leaky'(z_j) ;  dXL_j = alpha_j g + dz_j ;  dXR = sum_j dz_j
//   datt += de_j * leaky(z_j)
// ------------------------------------------------------------------------------------------
template <class G>
__global__ __launch_bounds__(kBlock) void attn_bwd_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum,
    const float* __restrict__ gout, int64_t ldG, float* __restrict__ dXL, int64_t ldDXL,
    float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr, float* __restrict__ datt_part,
    int xl_pos) {
  const int lane = threadIdx.x & (kWave - 1);
  const int row = lane / G::LPE;
  const int li = lane % G::LPE;
  const int f0 = li * G::VEC;
  const int h0 = f0 / G::C;
  const int wave = wave_id_uniform();
  const int nwaves = gridDim.x * (blockDim.x / kWave);

  float attv[G::VEC], bv[G::VEC], datt[G::VEC], dbias[G::VEC];
  load_vec<G::VEC>(attv, att + f0);
  load_vec<G::VEC>(bv, bias + f0);
#pragma unroll
  for (int v = 0; v < G::VEC; ++v) datt[v] = dbias[v] = 0.f;

  for (int it = wave; it < n_items; it += nwaves) {
    const gasfm_work_item w = items[it];
    const int64_t sg = w.seg;
    float xr[G::VEC], g[G::VEC], o[G::VEC];
    load_vec<G::VEC>(xr, XR + sg * ldXR + f0);
    load_vec<G::VEC>(g, gout + sg * ldG + f0);
    load_vec<G::VEC>(o, out + sg * ldOut + f0);
    // d bias = sum of gout over segments: count each segment once (its first item) on row 0
    if (row == 0 && (it == 0 || items[it - 1].seg != w.seg)) {
#pragma unroll
      for (int v = 0; v < G::VEC; ++v) dbias[v] += g[v];
    }
    float M[G::HPL], inv[G::HPL], delta[G::HPL];
#pragma unroll
    for (int hh = 0; hh < G::HPL; ++hh) {
      M[hh] = seg_max[sg * G::H + h0 + hh];
      inv[hh] = 1.f / (seg_sum[sg * G::H + h0 + hh] + 1e-16f);
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < G::CPH; ++c) {
        const int v = hh * G::CPH + c;
        d = fmaf(g[v], o[v] - bv[v], d);
      }
      delta[hh] = head_sum<G::LPH>(d);
    }
    float dxr[G::VEC];
#pragma unroll
    for (int v = 0; v < G::VEC; ++v) dxr[v] = 0.f;

    for (int e0 = w.begin; e0 < w.end; e0 += G::EPR * G::U) {
      float xl[G::U][G::VEC];
      int64_t src[G::U];
      bool valid[G::U];
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        const int e = e0 + u * G::EPR + row;
        valid[u] = e < w.end;
        src[u] = 0;
        if (valid[u]) {
          src[u] = perm ? int64_t(perm[e]) : int64_t(e);
          load_vec<G::VEC>(xl[u], XL + (xl_pos ? int64_t(e) : src[u]) * ldXL + f0);
        } else {
#pragma unroll
          for (int v = 0; v < G::VEC; ++v) xl[u][v] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        float z[G::VEC];
        float dx[G::VEC];
#pragma unroll
        for (int hh = 0; hh < G::HPL; ++hh) {
          float p = 0.f, da = 0.f;
#pragma unroll
          for (int c = 0; c < G::CPH; ++c) {
            const int v = hh * G::CPH + c;
            z[v] = xl[u][v] + xr[v];
            p = fmaf(leaky(z[v], slope), attv[v], p);
            da = fmaf(g[v], xl[u][v], da);
          }
          p = head_sum<G::LPH>(p);
          da = head_sum<G::LPH>(da);
          const float alpha = valid[u] ? __expf(p - M[hh]) * inv[hh] : 0.f;
          const float de = alpha * (da - delta[hh]);
#pragma unroll
          for (int c = 0; c < G::CPH; ++c) {
            const int v = hh * G::CPH + c;
            const float dz = de * attv[v] * (z[v] > 0.f ? 1.f : slope);
            dx[v] = fmaf(alpha, g[v], dz);
            dxr[v] += dz;
            datt[v] = fmaf(de, leaky(z[v], slope), datt[v]);
          }
        }
        if (valid[u]) store_vec<G::VEC>(dXL + src[u] * ldDXL + f0, dx);
      }
    }
#pragma unroll
    for (int v = 0; v < G::VEC; ++v) dxr[v] = xor_sum_from<G::LPE>(dxr[v]);
    if (row == 0) {
      if (w.slot < 0)
        store_vec<G::VEC>(dXR + sg * ldDXR + f0, dxr);
      else
        store_vec<G::VEC>(part_dxr + int64_t(w.slot) * G::HC + f0, dxr);
    }
  }
#pragma unroll
  for (int v = 0; v < G::VEC; ++v) datt[v] = xor_sum_from<G::LPE>(datt[v]);
  if (row == 0) {
    store_vec<G::VEC>(datt_part + int64_t(wave) * 2 * G::HC + f0, datt);
    store_vec<G::VEC>(datt_part + int64_t(wave) * 2 * G::HC + G::HC + f0, dbias);
  }
}

// ------------------------------------------------------------------------------------------
// backward with direct-to-LDS prefetch (Geom<32,8>; XL read at segment position e, i.e.
// perm == NULL or xl_by_position).  Per item, six global_load_lds into a wave-private buffer:
// the 32 rows of the first chunk, one instruction whose lane groups fetch XR / gout / out /
// seg_max / seg_sum of the segment, and perm of the 32 rows (the dXL destinations).  Empty
// items still fetch their segment data (d bias sums gout over every segment).
// ------------------------------------------------------------------------------------------
template <class G>
__global__ __launch_bounds__(kBlock, GASFM_GLDS_BWD_MINWAVES) void attn_bwd_glds_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum,
    const float* __restrict__ gout, int64_t ldG, float* __restrict__ dXL, int64_t ldDXL,
    float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr, float* __restrict__ datt_part) {
  static_assert(G::VEC == 4 && G::LPE == 8 && G::EPR == 8 && G::U == 4 && G::HPL == 1 && G::LPH == 2,
                "Geom<32,8> only");
  constexpr int RB = G::U * kWave;  // float4 slots of the 32 rows
  __shared__ float4 lbuf[kBlock / kWave][RB + kWave + kWave / 4];
  const int lane = threadIdx.x & (kWave - 1);
  const int row = lane / G::LPE;
  const int li = lane % G::LPE;
  const int f0 = li * G::VEC;
  const int h0 = f0 / G::C;
  const int wave = wave_id_uniform();
  const int nwaves = gridDim.x * (blockDim.x / kWave);
  float4* B = lbuf[threadIdx.x / kWave];
  int32_t* Bp = reinterpret_cast<int32_t*>(B + RB + kWave);
  float attv[G::VEC], bv[G::VEC], datt[G::VEC], dbias[G::VEC];
  load_vec<G::VEC>(attv, att + f0);
  load_vec<G::VEC>(bv, bias + f0);
#pragma unroll
  for (int v = 0; v < G::VEC; ++v) datt[v] = dbias[v] = 0.f;
  // segment-data lane groups: 0 XR, 1 gout, 2 out, 3 stats (lane 24 seg_max, 25 seg_sum)
  const int grp = lane >> 3;
  auto issue = [&](const gasfm_work_item& w) {
    const int64_t sg = w.seg;
    const float* src = XR + sg * ldXR + f0;
    if (grp == 1) src = gout + sg * ldG + f0;
    if (grp == 2) src = out + sg * ldOut + f0;
    if (grp == 3 && li == 0) src = seg_max + sg * G::H;
    if (grp == 3 && li == 1) src = seg_sum + sg * G::H;
    __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(B + RB), 16, 0, 0);
    if (w.begin >= w.end) return;
    const int64_t safe = w.begin;
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const int64_t e = w.begin + u * G::EPR + row;
      __builtin_amdgcn_global_load_lds((glb_vptr)(XL + (e < w.end ? e : safe) * ldXL + f0),
                                       (lds_vptr)(B + u * kWave), 16, 0, 0);
    }
    if (perm) {
      const int64_t e = w.begin + lane;
      __builtin_amdgcn_global_load_lds((glb_vptr)(perm + (e < w.end ? e : safe)), (lds_vptr)Bp, 4, 0, 0);
    }
  };
  int it = wave;
  gasfm_work_item wn{0, 0, 0, -1};
  if (it < n_items) {
    wn = items[it];
    issue(wn);
  }
  for (; it < n_items; it += nwaves) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const gasfm_work_item w = wn;
    float xl[G::U][G::VEC], xr[G::VEC], g[G::VEC], o[G::VEC];
    int64_t dst[G::U];
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const float4 v = B[u * kWave + lane];
      xl[u][0] = v.x;
      xl[u][1] = v.y;
      xl[u][2] = v.z;
      xl[u][3] = v.w;
      const int64_t e = w.begin + u * G::EPR + row;
      dst[u] = perm ? int64_t(Bp[u * G::EPR + row]) : e;
    }
    {
      const float4 a = B[RB + li], b = B[RB + 8 + li], c = B[RB + 16 + li];
      xr[0] = a.x, xr[1] = a.y, xr[2] = a.z, xr[3] = a.w;
      g[0] = b.x, g[1] = b.y, g[2] = b.z, g[3] = b.w;
      o[0] = c.x, o[1] = c.y, o[2] = c.z, o[3] = c.w;
    }
    const float4 smx = B[RB + 24], ssm = B[RB + 25];
    const float smxv[4] = {smx.x, smx.y, smx.z, smx.w}, ssmv[4] = {ssm.x, ssm.y, ssm.z, ssm.w};
    const float M = smxv[h0], inv = 1.f / (ssmv[h0] + 1e-16f);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool first = it == 0 || items[it - 1].seg != w.seg;
    if (it + nwaves < n_items) {
      wn = items[it + nwaves];
      issue(wn);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issue ahead of this item's compute
    // d bias = sum of gout over segments: each segment once (its first item) on row 0
    if (row == 0 && first) {
#pragma unroll
      for (int v = 0; v < G::VEC; ++v) dbias[v] += g[v];
    }
    float d = 0.f;
#pragma unroll
    for (int v = 0; v < G::VEC; ++v) d = fmaf(g[v], o[v] - bv[v], d);
    const float delta = head_sum<G::LPH>(d);
    float dxr[G::VEC] = {0.f, 0.f, 0.f, 0.f};
    auto chunk = [&](int e0) {
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        const bool valid = e0 + u * G::EPR + row < w.end;
        float z[G::VEC], dx[G::VEC];
        float p = 0.f, da = 0.f;
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) {
          z[v] = xl[u][v] + xr[v];
          p = fmaf(leaky(z[v], slope), attv[v], p);
          da = fmaf(g[v], xl[u][v], da);
        }
        p = head_sum<G::LPH>(p);
        da = head_sum<G::LPH>(da);
        const float alpha = valid ? __expf(p - M) * inv : 0.f;
        const float de = alpha * (da - delta);
#pragma unroll
        for (int v = 0; v < G::VEC; ++v) {
          const float dz = de * attv[v] * (z[v] > 0.f ? 1.f : slope);
          dx[v] = fmaf(alpha, g[v], dz);
          dxr[v] += dz;
          datt[v] = fmaf(de, leaky(z[v], slope), datt[v]);
        }
        if (valid) store_vec<G::VEC>(dXL + dst[u] * ldDXL + f0, dx);
      }
    };
    if (w.begin < w.end) chunk(w.begin);
    for (int e0 = w.begin + G::EPR * G::U; e0 < w.end; e0 += G::EPR * G::U) {  // long segments
#pragma unroll
      for (int u = 0; u < G::U; ++u) {
        const int e = e0 + u * G::EPR + row;
        const int ec = e < w.end ? e : e0;
        load_vec<G::VEC>(xl[u], XL + int64_t(ec) * ldXL + f0);
        dst[u] = perm ? int64_t(perm[ec]) : int64_t(e);
      }
      chunk(e0);
    }
#pragma unroll
    for (int v = 0; v < G::VEC; ++v) dxr[v] = xor_sum_from<G::LPE>(dxr[v]);
    if (row == 0) {
      if (w.slot < 0)
        store_vec<G::VEC>(dXR + int64_t(w.seg) * ldDXR + f0, dxr);
      else
        store_vec<G::VEC>(part_dxr + int64_t(w.slot) * G::HC + f0, dxr);
    }
  }
#pragma unroll
  for (int v = 0; v < G::VEC; ++v) datt[v] = xor_sum_from<G::LPE>(datt[v]);
  if (row == 0) {
    store_vec<G::VEC>(datt_part + int64_t(wave) * 2 * G::HC + f0, datt);
    store_vec<G::VEC>(datt_part + int64_t(wave) * 2 * G::HC + G::HC + f0, dbias);
  }
}

// dXR[seg] = ordered sum of its partial slots.
// grid = (combine entries, column blocks of CB = min(HC, 64)): R = kBlock / CB row groups take
// slots k = grp, grp + R, ... and are added in group order (deterministic for a given HC).
// One or two (part, out) pairs over the same combine entries (blockIdx.z selects the pair): the
// camera plan's dXR and the folded epilogue's dSv partial rows share their slots (round 5: one
// launch for both).
struct CombPair {
  const float* part[2];
  float* out[2];
  int64_t ld[2];
};
__global__ __launch_bounds__(kBlock) void attn_bwd_combine_kernel(const gasfm_combine_item* __restrict__ comb,
                                                             int n_comb, int HC, CombPair pr) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const float* __restrict__ part = pr.part[blockIdx.z];
  float* __restrict__ dXR = pr.out[blockIdx.z];
  const int64_t ld = pr.ld[blockIdx.z];
  const gasfm_combine_item ci = comb[blockIdx.x];
  const int CB = HC < 64 ? HC : 64;
  const int R = kBlock / CB;
  const int grp = threadIdx.x / CB;
  const int f = blockIdx.y * CB + int(threadIdx.x % CB);
  float a0 = 0.f, a1 = 0.f;
  if (grp < R && f < HC) {
    int k = grp;
    for (; k + R < ci.slot_count; k += 2 * R) {
      a0 += part[(int64_t(ci.slot_begin) + int64_t(k) * ci.slot_stride) * HC + f];
      a1 += part[(int64_t(ci.slot_begin) + int64_t(k + R) * ci.slot_stride) * HC + f];
    }
    if (k < ci.slot_count) a0 += part[(int64_t(ci.slot_begin) + int64_t(k) * ci.slot_stride) * HC + f];
  }
  sh[threadIdx.x] = a0 + a1;
  __syncthreads();
  if (grp == 0 && f < HC) {
    float t = 0.f;
    for (int g = 0; g < R; ++g) t += sh[g * CB + threadIdx.x];
    dXR[int64_t(ci.seg) * ld + f] = t;
  }
}

// ------------------------------------------------------------------------------------------
// generic (any H, C) fallback: one wave per item, lanes over the HC features, edges serial.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void attn_fwd_generic(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, int H, int C, float slope, int finalize,
    float* __restrict__ out, int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int LDP = H * C + 2 * H;
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = threadIdx.x / kWave;
  float* lg = lds + wib * 2 * H;  // [H] logits scratch + [H] running max
  const int HC = H * C;
  const int nwaves = gridDim.x * (blockDim.x / kWave);
  for (int it = wave_id_uniform(); it < n_items; it += nwaves) {
    const gasfm_work_item w = items[it];
    // Two passes per item: max, then exp/sum/acc (simple and exact).
    for (int h = lane; h < H; h += kWave) lg[H + h] = -INFINITY;
    __builtin_amdgcn_wave_barrier();
    for (int e = w.begin; e < w.end; ++e) {
      const int64_t src = perm ? perm[e] : e;
      for (int h = lane; h < H; h += kWave) {
        float p = 0.f;
        for (int c = 0; c < C; ++c) {
          const int f = h * C + c;
          p = fmaf(leaky(XL[src * ldXL + f] + XR[int64_t(w.seg) * ldXR + f], slope), att[f], p);
        }
        lg[H + h] = fmaxf(lg[H + h], p);
      }
    }
    __builtin_amdgcn_wave_barrier();
    for (int f = lane; f < HC; f += kWave) {
      const int h = f / C;
      const float M = lg[H + h];
      float s = 0.f, a = 0.f;
      for (int e = w.begin; e < w.end; ++e) {
        const int64_t src = perm ? perm[e] : e;
        float p = 0.f;
        for (int c = 0; c < C; ++c) {
          const int ff = h * C + c;
          p = fmaf(leaky(XL[src * ldXL + ff] + XR[int64_t(w.seg) * ldXR + ff], slope), att[ff], p);
        }
        const float ex = __expf(p - M);
        s += ex;
        a = fmaf(ex, XL[src * ldXL + f], a);
      }
      if (w.slot < 0) {
        out[int64_t(w.seg) * ldOut + f] = finalize ? a / (s + 1e-16f) + bias[f] : a;
        if (f % C == 0) {
          seg_max[int64_t(w.seg) * ldStat + h] = M;
          seg_sum[int64_t(w.seg) * ldStat + h] = s;
        }
      } else {
        part[int64_t(w.slot) * LDP + f] = a;
        if (f % C == 0) {
          part[int64_t(w.slot) * LDP + HC + h] = M;
          part[int64_t(w.slot) * LDP + HC + H + h] = s;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ __launch_bounds__(kBlock) void attn_combine_generic(
    const gasfm_combine_item* __restrict__ comb, int n_comb, int H, int C, const float* __restrict__ part,
    const float* __restrict__ bias, int finalize, float* __restrict__ out, int64_t ldOut, float* __restrict__ seg_max,
    float* __restrict__ seg_sum, int64_t ldStat) {
  const int wave = wave_id_uniform();
  const int lane = threadIdx.x & (kWave - 1);
  if (wave >= n_comb) return;
  const gasfm_combine_item ci = comb[wave];
  const int HC = H * C;
  for (int f = lane; f < HC; f += kWave) {
    const int h = f / C;
    float m = -INFINITY, s = 0.f, a = 0.f;
    for (int k = 0; k < ci.slot_count; ++k) {
      const int64_t slot = int64_t(ci.slot_begin) + int64_t(k) * ci.slot_stride;
      const int64_t LDP = HC + 2 * H;
      const float m2 = part[slot * LDP + HC + h], s2 = part[slot * LDP + HC + H + h], a2 = part[slot * LDP + f];
      const float mn = fmaxf(m, m2);
      const float f1 = safe_scale(m, mn), f2 = safe_scale(m2, mn);
      s = s * f1 + s2 * f2;
      a = a * f1 + a2 * f2;
      m = mn;
    }
    out[int64_t(ci.seg) * ldOut + f] = finalize ? a / (s + 1e-16f) + bias[f] : a;
    if (f % C == 0) {
      seg_max[int64_t(ci.seg) * ldStat + h] = m;
      seg_sum[int64_t(ci.seg) * ldStat + h] = s;
    }
  }
}

__global__ __launch_bounds__(kBlock) void attn_bwd_generic(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, int H, int C, float slope,
    const float* __restrict__ out, int64_t ldOut, const float* __restrict__ seg_max,
    const float* __restrict__ seg_sum, const float* __restrict__ gout, int64_t ldG, float* __restrict__ dXL,
    int64_t ldDXL, float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr,
    float* __restrict__ datt_part, int xl_pos) {
  // one lane per feature f; per-head scalars recomputed per lane (serial over C) — slow but general.
  const int wave = wave_id_uniform();
  const int lane = threadIdx.x & (kWave - 1);
  const int nwaves = gridDim.x * (blockDim.x / kWave);
  const int HC = H * C;
  for (int f = lane; f < 2 * HC; f += kWave) datt_part[int64_t(wave) * 2 * HC + f] = 0.f;
  for (int it = wave; it < n_items; it += nwaves) {
    const gasfm_work_item w = items[it];
    const int64_t sg = w.seg;
    const bool first = it == 0 || items[it - 1].seg != w.seg;
    for (int f = lane; f < HC; f += kWave) {
      if (first) datt_part[int64_t(wave) * 2 * HC + HC + f] += gout[sg * ldG + f];
      const int h = f / C;
      const float M = seg_max[sg * H + h];
      const float inv = 1.f / (seg_sum[sg * H + h] + 1e-16f);
      float delta = 0.f;
      for (int c = 0; c < C; ++c) {
        const int ff = h * C + c;
        delta = fmaf(gout[sg * ldG + ff], out[sg * ldOut + ff] - bias[ff], delta);
      }
      float dxr = 0.f, dat = 0.f;
      for (int e = w.begin; e < w.end; ++e) {
        const int64_t src = perm ? perm[e] : e;
        const int64_t xs = xl_pos ? int64_t(e) : src;
        float p = 0.f, da = 0.f;
        for (int c = 0; c < C; ++c) {
          const int ff = h * C + c;
          const float x = XL[xs * ldXL + ff];
          p = fmaf(leaky(x + XR[sg * ldXR + ff], slope), att[ff], p);
          da = fmaf(gout[sg * ldG + ff], x, da);
        }
        const float alpha = __expf(p - M) * inv;
        const float de = alpha * (da - delta);
        const float z = XL[xs * ldXL + f] + XR[sg * ldXR + f];
        const float dz = de * att[f] * (z > 0.f ? 1.f : slope);
        dXL[src * ldDXL + f] = fmaf(alpha, gout[sg * ldG + f], dz);
        dxr += dz;
        dat = fmaf(de, leaky(z, slope), dat);
      }
      if (w.slot < 0)
        dXR[sg * ldDXR + f] = dxr;
      else
        part_dxr[int64_t(w.slot) * HC + f] = dxr;
      datt_part[int64_t(wave) * 2 * HC + f] += dat;
    }
  }
}

// ------------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------------
// Item-loop kernels run one resident wave per SIMD slot: a grid larger than what fits on
// the chip leaves a second round of waves that each carry a full share of items (measured:
// point-direction forward 278 us at 8192 waves vs 193 us at the 7168 that fit).  The grid is
// the occupancy limit of the kernel x CU count; GASFM_ATTN_WAVES caps it (tuning sweeps).
static int env_wave_cap() {
  const int v = int(tune(GASFM_TUNE_ATTN_WAVE_CAP));
  return v > 0 ? v : 0;
}

// Direct-to-LDS forward for streamed (perm-free) 32-wide convs: default on (point direction
// 165 -> 140 us, camera 109 -> 106 us on config 4); GASFM_ATTN_GLDS=0 selects the register path.
static bool glds_enabled() { return tune(GASFM_TUNE_ATTN_GLDS) != 0.0; }

// Grouped-item forward (attn_fwd_grp_kernel<U, MINW>) for streamed 32-wide convs: GASFM_ATTN_GRP
// = 4 / 8 (U rows per lane per iteration), 46 / 48 (U = 4 at >= 6 / 8 waves per SIMD), 0 = off
// (direct-to-LDS kernel).
static int grp_rows() {
  const int v = int(tune(GASFM_TUNE_ATTN_GRP_ROWS));
  return (v == 8 || v == 4 || v == 46 || v == 48) ? v : 0;
}

// Lane groups per item of the U = 4 grouped forward (GASFM_ATTN_SPLIT: 1 / 2 / 4 forced; 0 = by
// size: S = 2 when the S = 1 tasks fit in one round of the resident waves, i.e. every wave would
// walk a single task's chain of row round trips; else S = 1).  Measured (profiles/r6_ab_attn_split.txt,
// events): a rank-of-8 shard's 25k points 23.6-24.2 -> 21.7-21.9 us at S = 2 (22.4-22.5 at S = 4);
// config 4's 200k points (25k tasks, 6x the resident waves) 114.0 at S = 1 vs 114.7 / 120.1.
static int grp_split(int n_items, int resident_waves) {
  const int v = int(tune(GASFM_TUNE_ATTN_GRP_SPLIT));
  if (v == 1 || v == 2 || v == 4) return v;
  return int64_t(n_items) <= int64_t(8) * resident_waves ? 2 : 1;
}

// Minimum fill (wave tasks / resident waves) for the grouped-item forward (A/B knob
// GASFM_ATTN_GRP_MIN_FILL; 0 = always grouped when enabled).
static double grp_min_fill() { return tune(GASFM_TUNE_ATTN_GRP_MIN_FILL); }

static int grid_for(int n_items, int resident) {
  int waves = n_items > 0 ? n_items : 1;
  const int cap = env_wave_cap() ? env_wave_cap() : resident * (kBlock / kWave);
  if (waves > cap) waves = cap;
  return (waves + (kBlock / kWave) - 1) / (kBlock / kWave);
}

template <class F>
static bool dispatch_shape(int H, int C, F&& f) {
  const int HC = H * C;
  if (HC == 32 && C == 8) return f(Geom<32, 8>{}), true;
  if (HC == 4 && C == 1) return f(Geom<4, 1>{}), true;
  if (HC == 64 && C == 16) return f(Geom<64, 16>{}), true;
  if (HC == 1024 && C == 256) return f(Geom<1024, 256>{}), true;
  if (HC == 32 && C == 32) return f(Geom<32, 32>{}), true;
  if (HC == 64 && C == 64) return f(Geom<64, 64>{}), true;
  if (HC == 128 && C == 32) return f(Geom<128, 32>{}), true;
  if (HC == 256 && C == 64) return f(Geom<256, 64>{}), true;
  return false;
}

}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_gat_attn_fwd(const float* XL, int64_t ldXL, const float* XR, int64_t ldXR,
                                  const float* att, const float* bias, const int32_t* perm,
                                  const gasfm_work_item* items, int32_t n_items, int32_t H, int32_t C,
                                  float slope, int32_t finalize, float* out, int64_t ldOut,
                                  float* seg_max, float* seg_sum, int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(H > 0 && C > 0 && n_items >= 0, "gasfm_gat_attn_fwd: H=%d C=%d n_items=%d", H, C, n_items);
  if (n_items == 0) return GASFM_OK;
  GASFM_REQUIRE(XL && XR && att && items && ((out && seg_max && seg_sum && bias) || part),
                "gasfm_gat_attn_fwd: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec_ok = (H * C) % 4 == 0 && ldXL % 4 == 0 && ldXR % 4 == 0 && ldOut % 4 == 0 &&
                      aligned16(XL) && aligned16(XR) && aligned16(out) && aligned16(att) &&
                      aligned16(bias) && (!part || aligned16(part)) && ((H * C + 2 * H) % 4 == 0);
  bool done = false;
  const int grp = grp_rows();
  // The grouped kernel packs 8 items into one wave task: right for many short segments (points,
  // ~20 edges each), wrong when that leaves the chip underfilled -- the camera direction of a
  // 1/8-points shard has ~2k items of up to 256 edges, i.e. 250 tasks = 72 workgroups (46 us vs
  // 20 us for the point direction).  Below grp_min_fill() of the resident waves, one item per
  // wave (the direct-to-LDS kernel) instead.
  const bool grp_fills = [&] {
    if (grp <= 0) return false;
    const int tasks = (n_items + 7) / 8;
    const int res = resident_blocks(reinterpret_cast<const void*>(&attn_fwd_grp_kernel<4, 1, 1>), kBlock, 0) *
                    (kBlock / kWave);
    return double(tasks) >= grp_min_fill() * double(res);
  }();
  if (vec_ok && perm == nullptr && H * C == 32 && C == 8 && grp_fills) {
    auto launch = [&](auto kern, int S) {
      const int per = 8 / S;
      const int tasks = (n_items + per - 1) / per;
      const int grid = grid_for(tasks, resident_blocks(reinterpret_cast<const void*>(kern), kBlock, 0));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, XL, ldXL, XR, ldXR, att, bias, items, n_items,
                         slope, finalize, out, ldOut, seg_max, seg_sum, ldStat, part);
    };
    note_dispatch(GASFM_K_ATTN_FWD_GRP);
    if (grp == 8) {
      launch(&attn_fwd_grp_kernel<8, 1, 1>, 1);
    } else if (grp == 46) {
      launch(&attn_fwd_grp_kernel<4, 6, 1>, 1);
    } else if (grp == 48) {
      launch(&attn_fwd_grp_kernel<4, 8, 1>, 1);
    } else {
      const int res =
          resident_blocks(reinterpret_cast<const void*>(&attn_fwd_grp_kernel<4, 1, 2>), kBlock, 0) * (kBlock / kWave);
      const int S = grp_split(n_items, env_wave_cap() ? env_wave_cap() : res);
      if (S == 4) {
        note_dispatch(GASFM_K_ATTN_FWD_GRP_S4);
        launch(&attn_fwd_grp_kernel<4, 1, 4>, 4);
      } else if (S == 2) {
        note_dispatch(GASFM_K_ATTN_FWD_GRP_S2);
        launch(&attn_fwd_grp_kernel<4, 1, 2>, 2);
      } else {
        launch(&attn_fwd_grp_kernel<4, 1, 1>, 1);
      }
    }
    done = true;
  }
  if (!done && vec_ok && perm == nullptr && H * C == 32 && C == 8 && glds_enabled()) {
    using G = Geom<32, 8>;
    const int grid =
        grid_for(n_items, resident_blocks(reinterpret_cast<const void*>(&attn_fwd_glds_kernel<G>), kBlock, 0));
    note_dispatch(GASFM_K_ATTN_FWD_GLDS);
    hipLaunchKernelGGL((attn_fwd_glds_kernel<G>), dim3(grid), dim3(kBlock), 0, st, XL, ldXL, XR, ldXR, att, bias,
                       items, n_items, slope, finalize, out, ldOut, seg_max, seg_sum, ldStat, part);
    done = true;
  }
  if (vec_ok && !done) {
    done = dispatch_shape(H, C, [&](auto g) {
      using G = decltype(g);
      const int grid = grid_for(n_items, resident_blocks(reinterpret_cast<const void*>(&attn_fwd_kernel<G>), kBlock, 0));
      note_dispatch(GASFM_K_ATTN_FWD_VEC);
      hipLaunchKernelGGL((attn_fwd_kernel<G>), dim3(grid), dim3(kBlock), 0, st, XL, ldXL, XR, ldXR, att,
                         bias, perm, items, n_items, slope, finalize, out, ldOut, seg_max, seg_sum, ldStat, part);
    });
  }
  if (!done) {
    const size_t lds = (kBlock / kWave) * 2 * H * sizeof(float);
    const int grid = grid_for(n_items, resident_blocks(reinterpret_cast<const void*>(&attn_fwd_generic), kBlock, lds));
    note_dispatch(GASFM_K_ATTN_FWD_GENERIC);
    hipLaunchKernelGGL(attn_fwd_generic, dim3(grid), dim3(kBlock), lds, st,
                       XL, ldXL, XR, ldXR, att, bias, perm, items, n_items, H, C, slope, finalize, out, ldOut,
                       seg_max, seg_sum, ldStat, part);
  }
  return launch_status("gasfm_gat_attn_fwd");
}

// 1 (default since round 4): rank-0-of-8 proxy 8.00-8.02 -> 7.88 ms, config 4 unchanged (29.56-29.75
// vs 29.60-29.71), profiles/r4_ab5.txt
#ifndef GASFM_COMBINE_SMALL
#define GASFM_COMBINE_SMALL 1
#endif
extern "C" int gasfm_gat_attn_combine(const gasfm_combine_item* combine, int32_t n_combine, int32_t H,
                                      int32_t C, const float* part, const float* bias, int32_t finalize, float* out,
                                      int64_t ldOut, float* seg_max, float* seg_sum, int64_t ldStat, void* stream) {
  GASFM_REQUIRE(H > 0 && C > 0 && n_combine >= 0, "gasfm_gat_attn_combine: bad args");
  if (n_combine == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec_ok = (H * C) % 4 == 0 && ldOut % 4 == 0 && aligned16(out) && aligned16(part) &&
                      aligned16(bias) && ((H * C + 2 * H) % 4 == 0);
  bool done = false;
  if (vec_ok) {
    done = dispatch_shape(H, C, [&](auto g) {
      using G = decltype(g);
      // GASFM_COMBINE_SMALL (round 4): 256 threads for the narrow rows (HC <= 64: 32 to 256 slot
      // rows per pass, while a combine entry holds <= ~64 slots after the two-level split) instead
      // of 1024 threads whose 16-wave LDS merge and launch cost dominate a few-slot merge
      const int threads = (GASFM_COMBINE_SMALL && G::HC <= 64) ? 256 : 1024;
      const size_t lds = size_t(threads / kWave) * G::LPE * (G::VEC + 2 * G::HPL) * sizeof(float);
      note_dispatch(GASFM_K_ATTN_COMBINE_VEC);
      hipLaunchKernelGGL((attn_combine_kernel<G>), dim3(n_combine), dim3(threads), lds, st, combine, part, bias,
                         finalize, out, ldOut, seg_max, seg_sum, ldStat);
    });
  }
  if (!done) {
    const int grid = (n_combine + (kBlock / kWave) - 1) / (kBlock / kWave);
    note_dispatch(GASFM_K_ATTN_COMBINE_GENERIC);
    hipLaunchKernelGGL(attn_combine_generic, dim3(grid), dim3(kBlock), 0, st, combine, n_combine, H, C, part, bias,
                       finalize, out, ldOut, seg_max, seg_sum, ldStat);
  }
  return launch_status("gasfm_gat_attn_combine");
}

// Backward grid: the same for the vectorised and the generic kernel of a shape, since the
// caller sizes the per-wave datt/dbias partials (gasfm_gat_attn_bwd_waves) before the launch.
static int bwd_grid(int n_items, int H, int C) {
  int res = resident_blocks(reinterpret_cast<const void*>(&attn_bwd_generic), kBlock, 0);
  dispatch_shape(H, C, [&](auto g) {
    using G = decltype(g);
    const int r = resident_blocks(reinterpret_cast<const void*>(&attn_bwd_kernel<G>), kBlock, 0);
    res = r < res ? r : res;
  });
  if (H * C == 32 && C == 8) {
    const int r = resident_blocks(reinterpret_cast<const void*>(&attn_bwd_glds_kernel<Geom<32, 8>>), kBlock, 0);
    res = r < res ? r : res;
  }
  return grid_for(n_items, res);
}

extern "C" int gasfm_gat_attn_bwd_waves(int32_t n_items, int32_t H, int32_t C) {
  if (n_items <= 0 || H <= 0 || C <= 0) return 0;
  return bwd_grid(n_items, H, C) * (kBlock / kWave);
}

extern "C" int gasfm_gat_attn_bwd(const float* XL, int64_t ldXL, const float* XR, int64_t ldXR,
                                  const float* att, const float* bias, const int32_t* perm,
                                  const gasfm_work_item* items, int32_t n_items, int32_t H, int32_t C,
                                  float slope, const float* out, int64_t ldOut, const float* seg_max,
                                  const float* seg_sum, const float* gout, int64_t ldG, float* dXL,
                                  int64_t ldDXL, float* dXR, int64_t ldDXR, float* part_dxr,
                                  float* datt_part, int32_t xl_by_position, void* stream) {
  GASFM_REQUIRE(H > 0 && C > 0 && n_items >= 0, "gasfm_gat_attn_bwd: bad args");
  if (n_items == 0) return GASFM_OK;
  GASFM_REQUIRE(XL && XR && att && bias && items && out && seg_max && seg_sum && gout && dXL && dXR && datt_part,
                "gasfm_gat_attn_bwd: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = bwd_grid(n_items, H, C);
  const bool vec_ok = (H * C) % 4 == 0 && ldXL % 4 == 0 && ldXR % 4 == 0 && ldOut % 4 == 0 && ldG % 4 == 0 &&
                      ldDXL % 4 == 0 && ldDXR % 4 == 0 && aligned16(XL) && aligned16(XR) && aligned16(out) &&
                      aligned16(gout) && aligned16(dXL) && aligned16(dXR) && aligned16(att) &&
                      aligned16(bias) && aligned16(datt_part) && (!part_dxr || aligned16(part_dxr));
  bool done = false;
  if (!done && vec_ok && H * C == 32 && C == 8 && (perm == nullptr || xl_by_position) && glds_enabled() &&
      aligned16(seg_max) && aligned16(seg_sum)) {
    note_dispatch(GASFM_K_ATTN_BWD_GLDS);
    hipLaunchKernelGGL((attn_bwd_glds_kernel<Geom<32, 8>>), dim3(grid), dim3(kBlock), 0, st, XL, ldXL, XR, ldXR,
                       att, bias, perm, items, n_items, slope, out, ldOut, seg_max, seg_sum, gout, ldG, dXL, ldDXL,
                       dXR, ldDXR, part_dxr, datt_part);
    done = true;
  }
  if (vec_ok && !done) {
    done = dispatch_shape(H, C, [&](auto g) {
      using G = decltype(g);
      note_dispatch(GASFM_K_ATTN_BWD_VEC);
      hipLaunchKernelGGL((attn_bwd_kernel<G>), dim3(grid), dim3(kBlock), 0, st, XL, ldXL, XR, ldXR, att, bias,
                         perm, items, n_items, slope, out, ldOut, seg_max, seg_sum, gout, ldG, dXL, ldDXL, dXR,
                         ldDXR, part_dxr, datt_part, int(xl_by_position != 0));
    });
  }
  if (!done) {
    note_dispatch(GASFM_K_ATTN_BWD_GENERIC);
    hipLaunchKernelGGL(attn_bwd_generic, dim3(grid), dim3(kBlock), 0, st, XL, ldXL, XR, ldXR, att, bias, perm,
                       items, n_items, H, C, slope, out, ldOut, seg_max, seg_sum, gout, ldG, dXL, ldDXL, dXR,
                       ldDXR, part_dxr, datt_part, int(xl_by_position != 0));
  }
  return launch_status("gasfm_gat_attn_bwd");
}

extern "C" int gasfm_gat_attn_bwd_combine(const gasfm_combine_item* combine, int32_t n_combine, int32_t HC,
                                          const float* part_dxr, float* dXR, int64_t ldDXR, void* stream) {
  GASFM_REQUIRE(HC > 0 && n_combine >= 0, "gasfm_gat_attn_bwd_combine: bad args");
  if (n_combine == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int cb = HC < 64 ? HC : 64;
  const CombPair pr{{part_dxr, part_dxr}, {dXR, dXR}, {ldDXR, ldDXR}};
  hipLaunchKernelGGL(attn_bwd_combine_kernel, dim3(n_combine, (HC + cb - 1) / cb, 1), dim3(kBlock),
                     kBlock * sizeof(float), st, combine, n_combine, HC, pr);
  return launch_status("gasfm_gat_attn_bwd_combine");
}

extern "C" int gasfm_gat_attn_bwd_combine2(const gasfm_combine_item* combine, int32_t n_combine, int32_t HC,
                                           const float* part_a, float* out_a, int64_t ld_a, const float* part_b,
                                           float* out_b, int64_t ld_b, void* stream) {
  GASFM_REQUIRE(HC > 0 && n_combine >= 0 && part_a && out_a && part_b && out_b,
                "gasfm_gat_attn_bwd_combine2: bad args");
  if (n_combine == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int cb = HC < 64 ? HC : 64;
  const CombPair pr{{part_a, part_b}, {out_a, out_b}, {ld_a, ld_b}};
  hipLaunchKernelGGL(attn_bwd_combine_kernel, dim3(n_combine, (HC + cb - 1) / cb, 2), dim3(kBlock),
                     kBlock * sizeof(float), st, combine, n_combine, HC, pr);
  return launch_status("gasfm_gat_attn_bwd_combine2");
}
