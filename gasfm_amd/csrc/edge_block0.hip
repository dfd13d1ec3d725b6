// Per-edge body of GASFM block 0 (2-wide embedded projections -> 32-wide features), gfx950.
//
// Block 0 (code/models/layers.py:148-263 with n_feat_proj_in = 2, graph_attn_sfm.py:61-84)
// differs from the 32-wide blocks: LayerNorm over 2 features, GATv2 lin_l 2 -> 4 per
// direction (H=4, C=1), no init-feature concat, and a projected residual
//   P' = Wsk relu(LN_b(P)) + bsk + (Wp relu(LN_a(P)) + bp + Sp[pt] + Sv[cam] + Sg) / 4
// (residual_skipconn_proj_norm_layer + skip_projection, layers.py:214-220, 256-261).
// torch runs its 2-wide LayerNorm through a row-moments kernel at ~11 ms per call on
// 4M rows; here every op is one thread (or one 8-lane group) per edge.
//
//   edge0_prologue_fwd  XL0[e] = W0 relu(LN_a(P[e])) + b0          (W0 [8 x 2])
//   edge0_epilogue_fwd  the P' above, 8 lanes x float4 per edge
//   edge0_epilogue_bwd  camera work items: dSv, dWp, dWsk, dbsk, dgamma_b, dbeta_b partials,
//                       aux[e] = (dP_hat_a from Wp, dP from the LN_b branch)
//   edge0_prologue_bwd  dP = LN_a_bwd(mask (W0^T dXL0 + aux.xy)) + aux.zw; dW0, db0,
//                       dgamma_a, dbeta_a partials
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "lanes.hpp"

#ifndef GASFM_E0_EPI_U
#define GASFM_E0_EPI_U 4  // edge0_epilogue_bwd: 8-edge row groups whose loads are in flight together
#endif

namespace gasfm {
namespace {

constexpr int kW = 64;
constexpr int kT = 256;
constexpr int kMaxGrid = 1024;

struct LN2 {
  float xh0, xh1, rstd;
};

__device__ __forceinline__ LN2 ln2(float a, float b, float eps) {
  const float mean = 0.5f * (a + b);
  const float d0 = a - mean, d1 = b - mean;
  const float rstd = rsq_normal(0.5f * (d0 * d0 + d1 * d1) + eps);
  return {d0 * rstd, d1 * rstd, rstd};
}

// LN backward for 2 features given g_k = dy_k * gamma_k.
__device__ __forceinline__ void ln2_bwd(const LN2& l, float g0, float g1, float& dx0, float& dx1) {
  const float mg = 0.5f * (g0 + g1);
  const float mgx = 0.5f * (g0 * l.xh0 + g1 * l.xh1);
  dx0 = l.rstd * (g0 - mg - l.xh0 * mgx);
  dx1 = l.rstd * (g1 - mg - l.xh1 * mgx);
}

template <int N>
__device__ __forceinline__ void block_reduce_store(float (&v)[N], float* out, float* sh) {
  // wave reduce (xor over all 64 lanes), then waves in order through LDS
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = group_sum<kW>(v[k]);
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < N; ++k) sh[wave * N + k] = v[k];
  __syncthreads();
  if (threadIdx.x < N) {
    float s = 0.f;
    for (int w = 0; w < kT / kW; ++w) s += sh[w * N + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kT) void edge0_prologue_fwd_kernel(const float2* __restrict__ P, int64_t E,
                                                               const float* __restrict__ ga,
                                                               const float* __restrict__ ba, float eps,
                                                               const float* __restrict__ W0,
                                                               const float* __restrict__ b0,
                                                               float4* __restrict__ XL,
                                                               const int32_t* __restrict__ pos) {
  float w[8][2], bb[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    w[o][0] = W0[2 * o];
    w[o][1] = W0[2 * o + 1];
    bb[o] = b0[o];
  }
  const float g0 = ga[0], g1 = ga[1], e0 = ba[0], e1 = ba[1];
  for (int64_t e = blockIdx.x * int64_t(kT) + threadIdx.x; e < E; e += int64_t(gridDim.x) * kT) {
    const float2 p = P[e];
    const LN2 l = ln2(p.x, p.y, eps);
    const float h0 = fmaxf(fmaf(l.xh0, g0, e0), 0.f), h1 = fmaxf(fmaf(l.xh1, g1, e1), 0.f);
    float y[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) y[o] = fmaf(w[o][0], h0, fmaf(w[o][1], h1, bb[o]));
    // point half at the edge's position in point order (pos), camera half at e
    XL[2 * (pos ? int64_t(pos[e]) : e)] = make_float4(y[0], y[1], y[2], y[3]);
    XL[2 * e + 1] = make_float4(y[4], y[5], y[6], y[7]);
  }
}

// The same XL0 written row by row: row r holds the point half of edge perm[r] (perm = the point
// plan's permutation, the inverse of pos) and the camera half of edge r, so each thread stores one
// whole 32-B row and the rows of a wave are one contiguous 2 KB run.  The scattered variant above
// stores the point halves as 16-B pieces at random rows (partial-line writes); here the only random
// access is the 8-B read of P[perm[r]] (32 B per edge of P in total: the array sits in L2 / MALL).
// Both halves are the same float operations on the same P row as above: bitwise the same XL0.
__global__ __launch_bounds__(kT) void edge0_prologue_fwd_rows_kernel(const float2* __restrict__ P, int64_t E,
                                                                    const float* __restrict__ ga,
                                                                    const float* __restrict__ ba, float eps,
                                                                    const float* __restrict__ W0,
                                                                    const float* __restrict__ b0,
                                                                    float4* __restrict__ XL,
                                                                    const int32_t* __restrict__ perm) {
  float w[8][2], bb[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    w[o][0] = W0[2 * o];
    w[o][1] = W0[2 * o + 1];
    bb[o] = b0[o];
  }
  const float g0 = ga[0], g1 = ga[1], e0 = ba[0], e1 = ba[1];
  for (int64_t r = blockIdx.x * int64_t(kT) + threadIdx.x; r < E; r += int64_t(gridDim.x) * kT) {
    const float2 pc = P[r];
    const float2 pp = P[perm[r]];
    const LN2 lp = ln2(pp.x, pp.y, eps), lc = ln2(pc.x, pc.y, eps);
    const float hp0 = fmaxf(fmaf(lp.xh0, g0, e0), 0.f), hp1 = fmaxf(fmaf(lp.xh1, g1, e1), 0.f);
    const float hc0 = fmaxf(fmaf(lc.xh0, g0, e0), 0.f), hc1 = fmaxf(fmaf(lc.xh1, g1, e1), 0.f);
    float y[8];
#pragma unroll
    for (int o = 0; o < 4; ++o) y[o] = fmaf(w[o][0], hp0, fmaf(w[o][1], hp1, bb[o]));
#pragma unroll
    for (int o = 4; o < 8; ++o) y[o] = fmaf(w[o][0], hc0, fmaf(w[o][1], hc1, bb[o]));
    XL[2 * r] = make_float4(y[0], y[1], y[2], y[3]);
    XL[2 * r + 1] = make_float4(y[4], y[5], y[6], y[7]);
  }
}

// 8 lanes per edge (lane owns output columns c = 4*(lane&7) .. +3), 8 edges per wave step.
__global__ __launch_bounds__(kT) void edge0_epilogue_fwd_kernel(
    const float2* __restrict__ P, const int32_t* __restrict__ cam, const int32_t* __restrict__ pt, int64_t E,
    const float* __restrict__ ga, const float* __restrict__ ba, const float* __restrict__ gb,
    const float* __restrict__ bbt, float eps, const float* __restrict__ Wp, const float* __restrict__ bp,
    const float* __restrict__ Wsk, const float* __restrict__ bsk, const float* __restrict__ Sp,
    const float* __restrict__ Sv, int64_t ldSv, const float* __restrict__ Sg, float scale,
    float* __restrict__ Pout) {
  const int lane = threadIdx.x & (kW - 1);
  const int c0 = 4 * (lane & 7);
  float wp[4][2], wsk[4][2], cst[4], bs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    wp[k][0] = Wp[2 * (c0 + k)];
    wp[k][1] = Wp[2 * (c0 + k) + 1];
    wsk[k][0] = Wsk[2 * (c0 + k)];
    wsk[k][1] = Wsk[2 * (c0 + k) + 1];
    cst[k] = bp[c0 + k] + Sg[c0 + k];
    bs[k] = bsk[c0 + k];
  }
  const float ga0 = ga[0], ga1 = ga[1], ba0 = ba[0], ba1 = ba[1];
  const float gb0 = gb[0], gb1 = gb[1], bb0 = bbt[0], bb1 = bbt[1];
  const int64_t stride = int64_t(gridDim.x) * (kT / 8);
  for (int64_t e = blockIdx.x * int64_t(kT / 8) + threadIdx.x / 8; e < E; e += stride) {
    const float2 p = P[e];
    const LN2 l = ln2(p.x, p.y, eps);
    const float ha0 = fmaxf(fmaf(l.xh0, ga0, ba0), 0.f), ha1 = fmaxf(fmaf(l.xh1, ga1, ba1), 0.f);
    const float hb0 = fmaxf(fmaf(l.xh0, gb0, bb0), 0.f), hb1 = fmaxf(fmaf(l.xh1, gb1, bb1), 0.f);
    const float4 sp = *reinterpret_cast<const float4*>(Sp + int64_t(pt[e]) * 32 + c0);
    const float4 sv = *reinterpret_cast<const float4*>(Sv + int64_t(cam[e]) * ldSv + c0);
    const float spv[4] = {sp.x, sp.y, sp.z, sp.w}, svv[4] = {sv.x, sv.y, sv.z, sv.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = fmaf(wp[k][0], ha0, fmaf(wp[k][1], ha1, cst[k])) + spv[k] + svv[k];
      o[k] = fmaf(d, scale, fmaf(wsk[k][0], hb0, fmaf(wsk[k][1], hb1, bs[k])));
    }
    *reinterpret_cast<float4*>(Pout + e * 32 + c0) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// One wave per camera work item; 8 lanes per edge (4 columns each), 8 edges per step.
// part row per workgroup: [dWp 64 | dWsk 64 | dbsk 32 | dgamma_b 2 | dbeta_b 2]
constexpr int kPart0E = 64 + 64 + 32 + 4;
constexpr int kU = GASFM_E0_EPI_U;
__global__ __launch_bounds__(kT) void edge0_epilogue_bwd_kernel(
    const gasfm_work_item* __restrict__ items, int n_items, const float* __restrict__ dPo,
    const float2* __restrict__ P, const float* __restrict__ ga, const float* __restrict__ ba,
    const float* __restrict__ gb, const float* __restrict__ bbt, float eps, const float* __restrict__ Wp,
    const float* __restrict__ Wsk, float scale, float* __restrict__ dSv, float* __restrict__ part_dsv,
    float4* __restrict__ aux, float* __restrict__ part) {
  __shared__ float sh[(kT / kW) * kPart0E];
  const int lane = threadIdx.x & (kW - 1);
  const int row = lane >> 3, c0 = 4 * (lane & 7);
  float wp[4][2], wsk[4][2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    wp[k][0] = Wp[2 * (c0 + k)] * scale;
    wp[k][1] = Wp[2 * (c0 + k) + 1] * scale;
    wsk[k][0] = Wsk[2 * (c0 + k)];
    wsk[k][1] = Wsk[2 * (c0 + k) + 1];
  }
  const float ga0 = ga[0], ga1 = ga[1], ba0 = ba[0], ba1 = ba[1];
  const float gb0 = gb[0], gb1 = gb[1], bb0 = bbt[0], bb1 = bbt[1];
  float dwp[4][2] = {}, dwsk[4][2] = {}, dbsk[4] = {}, dgb[2] = {}, dbb[2] = {};
  const int nw = gridDim.x * (kT / kW);
  for (int it = __builtin_amdgcn_readfirstlane(blockIdx.x * (kT / kW) + threadIdx.x / kW); it < n_items; it += nw) {
    const gasfm_work_item w = items[it];
    float dsv[4] = {};
    // kU row groups of 8 edges per step: their loads are issued together (kU x 1 KB of dP' per wave
    // in flight instead of one), then consumed in edge order (the sums' order is unchanged)
    for (int e0 = w.begin; e0 < w.end; e0 += 8 * kU) {
      float4 d4[kU];
      float2 pv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {  // unconditional loads (rows past the item re-read its last edge)
        const int ec = min(e0 + 8 * u + row, w.end - 1);
        d4[u] = *reinterpret_cast<const float4*>(dPo + int64_t(ec) * 32 + c0);
        pv[u] = P[ec];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + 8 * u + row;
        const bool valid = e < w.end;  // dead rows masked at the consumers
        const float2 p = valid ? pv[u] : make_float2(0.f, 1.f);
        const float4 dv = valid ? d4[u] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float d[4] = {dv.x, dv.y, dv.z, dv.w};
        const LN2 l = ln2(p.x, p.y, eps);
        const float ya0 = fmaf(l.xh0, ga0, ba0), ya1 = fmaf(l.xh1, ga1, ba1);
        const float yb0 = fmaf(l.xh0, gb0, bb0), yb1 = fmaf(l.xh1, gb1, bb1);
        const float ha0 = fmaxf(ya0, 0.f), ha1 = fmaxf(ya1, 0.f), hb0 = fmaxf(yb0, 0.f), hb1 = fmaxf(yb1, 0.f);
        float qa0 = 0.f, qa1 = 0.f, qb0 = 0.f, qb1 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dsv[k] += d[k];
          dwp[k][0] = fmaf(d[k], ha0, dwp[k][0]);
          dwp[k][1] = fmaf(d[k], ha1, dwp[k][1]);
          dwsk[k][0] = fmaf(d[k], hb0, dwsk[k][0]);
          dwsk[k][1] = fmaf(d[k], hb1, dwsk[k][1]);
          dbsk[k] += d[k];
          qa0 = fmaf(d[k], wp[k][0], qa0);
          qa1 = fmaf(d[k], wp[k][1], qa1);
          qb0 = fmaf(d[k], wsk[k][0], qb0);
          qb1 = fmaf(d[k], wsk[k][1], qb1);
        }
        qa0 = group_sum<8>(qa0);
        qa1 = group_sum<8>(qa1);
        qb0 = group_sum<8>(qb0);
        qb1 = group_sum<8>(qb1);
        // LN_b / ReLU backward of the skip branch (every lane of the row holds the same values)
        const float db0 = yb0 > 0.f ? qb0 : 0.f, db1 = yb1 > 0.f ? qb1 : 0.f;
        float dx0, dx1;
        ln2_bwd(l, db0 * gb0, db1 * gb1, dx0, dx1);
        if ((lane & 7) == 0 && valid) {
          dgb[0] = fmaf(db0, l.xh0, dgb[0]);
          dgb[1] = fmaf(db1, l.xh1, dgb[1]);
          dbb[0] += db0;
          dbb[1] += db1;
          aux[e] = make_float4(qa0, qa1, dx0, dx1);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      dsv[k] = xor_sum_from<8>(dsv[k]);
    if (row == 0) {
      const float4 r = make_float4(dsv[0] * scale, dsv[1] * scale, dsv[2] * scale, dsv[3] * scale);
      float* dst = (w.slot < 0) ? dSv + int64_t(w.seg) * 32 : part_dsv + int64_t(w.slot) * 32;
      *reinterpret_cast<float4*>(dst + c0) = r;
    }
  }
  // reduce over the 8 edge rows (xor 8/16/32 keeps the column group), then waves through LDS
  float r[20];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    r[2 * k] = dwp[k][0] * scale;
    r[2 * k + 1] = dwp[k][1] * scale;
    r[8 + 2 * k] = dwsk[k][0];
    r[8 + 2 * k + 1] = dwsk[k][1];
    r[16 + k] = dbsk[k];
  }
  float t[4] = {dgb[0], dgb[1], dbb[0], dbb[1]};
#pragma unroll
  for (int k = 0; k < 20; ++k) r[k] = xor_sum_from<8>(r[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = xor_sum_from<8>(t[k]);
  const int wave = threadIdx.x / kW;
  float* sw = sh + wave * kPart0E;
  if (row == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sw[2 * (c0 + k)] = r[2 * k];
      sw[2 * (c0 + k) + 1] = r[2 * k + 1];
      sw[64 + 2 * (c0 + k)] = r[8 + 2 * k];
      sw[64 + 2 * (c0 + k) + 1] = r[8 + 2 * k + 1];
      sw[128 + c0 + k] = r[16 + k];
    }
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) sw[160 + k] = t[k];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kPart0E; k += kT) {
    float s2 = 0.f;
    for (int w2 = 0; w2 < kT / kW; ++w2) s2 += sh[w2 * kPart0E + k];
    part[int64_t(blockIdx.x) * kPart0E + k] = s2;
  }
}

// thread per edge; part row per workgroup: [dW0 16 | db0 8 | dgamma_a 2 | dbeta_a 2]
constexpr int kPart0P = 16 + 8 + 4;
__global__ __launch_bounds__(kT) void edge0_prologue_bwd_kernel(const float4* __restrict__ dXL, const float2* __restrict__ P,
                                                               const float4* __restrict__ aux, int64_t E,
                                                               const float* __restrict__ ga,
                                                               const float* __restrict__ ba, float eps,
                                                               const float* __restrict__ W0, float2* __restrict__ dP,
                                                               float* __restrict__ part) {
  __shared__ float sh[(kT / kW) * kPart0P];
  float w[8][2];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    w[o][0] = W0[2 * o];
    w[o][1] = W0[2 * o + 1];
  }
  const float g0 = ga[0], g1 = ga[1], e0 = ba[0], e1 = ba[1];
  float v[kPart0P];
#pragma unroll
  for (int k = 0; k < kPart0P; ++k) v[k] = 0.f;
  for (int64_t e = blockIdx.x * int64_t(kT) + threadIdx.x; e < E; e += int64_t(gridDim.x) * kT) {
    const float4 x0 = dXL[2 * e], x1 = dXL[2 * e + 1];
    const float dx[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    const float4 a = aux ? aux[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float2 p = P[e];
    const LN2 l = ln2(p.x, p.y, eps);
    const float y0 = fmaf(l.xh0, g0, e0), y1 = fmaf(l.xh1, g1, e1);
    const float h0 = fmaxf(y0, 0.f), h1 = fmaxf(y1, 0.f);
    float dh0 = a.x, dh1 = a.y;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      dh0 = fmaf(w[o][0], dx[o], dh0);
      dh1 = fmaf(w[o][1], dx[o], dh1);
      v[2 * o] = fmaf(dx[o], h0, v[2 * o]);
      v[2 * o + 1] = fmaf(dx[o], h1, v[2 * o + 1]);
      v[16 + o] += dx[o];
    }
    const float dy0 = y0 > 0.f ? dh0 : 0.f, dy1 = y1 > 0.f ? dh1 : 0.f;
    v[24] = fmaf(dy0, l.xh0, v[24]);
    v[25] = fmaf(dy1, l.xh1, v[25]);
    v[26] += dy0;
    v[27] += dy1;
    float q0, q1;
    ln2_bwd(l, dy0 * g0, dy1 * g1, q0, q1);
    dP[e] = make_float2(q0 + a.z, q1 + a.w);
  }
  block_reduce_store<kPart0P>(v, part + int64_t(blockIdx.x) * kPart0P, sh);
}

int grid_for(int64_t units, int per_block) {
  const int64_t g = (units + per_block - 1) / per_block;
  return int(g < 1 ? 1 : (g > kMaxGrid ? kMaxGrid : g));
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_edge0_part_rows(int32_t which, int64_t E, int32_t n_items) {
  return which == 0 ? grid_for(E, kT) : grid_for(n_items, kT / kW);
}

extern "C" int gasfm_edge0_prologue_fwd(const float* P, int64_t E, const float* ln_w, const float* ln_b, float eps,
                                        const float* W0, const float* b0, float* XL, const int32_t* pos,
                                        void* stream) {
  GASFM_REQUIRE(P && ln_w && ln_b && W0 && b0 && XL && aligned16(XL), "gasfm_edge0_prologue_fwd: bad args");
  if (E == 0) return GASFM_OK;
  hipLaunchKernelGGL(edge0_prologue_fwd_kernel, dim3(grid_for(E, kT)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float2*>(P), E, ln_w, ln_b, eps,
                     W0, b0, reinterpret_cast<float4*>(XL), pos);
  return launch_status("gasfm_edge0_prologue_fwd");
}

extern "C" int gasfm_edge0_prologue_fwd_rows(const float* P, int64_t E, const float* ln_w, const float* ln_b,
                                             float eps, const float* W0, const float* b0, float* XL,
                                             const int32_t* perm, void* stream) {
  GASFM_REQUIRE(P && ln_w && ln_b && W0 && b0 && XL && perm && aligned16(XL),
                "gasfm_edge0_prologue_fwd_rows: bad args");
  if (E == 0) return GASFM_OK;
  hipLaunchKernelGGL(edge0_prologue_fwd_rows_kernel, dim3(grid_for(E, kT)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float2*>(P), E, ln_w, ln_b, eps,
                     W0, b0, reinterpret_cast<float4*>(XL), perm);
  return launch_status("gasfm_edge0_prologue_fwd_rows");
}

extern "C" int gasfm_edge0_epilogue_fwd(const float* P, const int32_t* cam, const int32_t* pt, int64_t E,
                                        const float* ln_a_w, const float* ln_a_b, const float* ln_b_w,
                                        const float* ln_b_b, float eps, const float* Wp, const float* bp,
                                        const float* Wsk, const float* bsk, const float* Sp, const float* Sv,
                                        int64_t ldSv, const float* Sg, float scale, float* Pout, void* stream) {
  GASFM_REQUIRE(P && cam && pt && Wp && bp && Wsk && bsk && Sp && Sv && Sg && Pout && aligned16(Sp) &&
                    aligned16(Sv) && aligned16(Pout) && ldSv >= 32 && ldSv % 4 == 0,
                "gasfm_edge0_epilogue_fwd: bad args");
  if (E == 0) return GASFM_OK;
  hipLaunchKernelGGL(edge0_epilogue_fwd_kernel, dim3(grid_for(E, kT / 8)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float2*>(P), cam, pt, E, ln_a_w,
                     ln_a_b, ln_b_w, ln_b_b, eps, Wp, bp, Wsk, bsk, Sp, Sv, ldSv, Sg, scale, Pout);
  return launch_status("gasfm_edge0_epilogue_fwd");
}

extern "C" int gasfm_edge0_epilogue_bwd(const gasfm_work_item* items, int32_t n_items, const float* dPo,
                                        const float* P, const float* ln_a_w, const float* ln_a_b,
                                        const float* ln_b_w, const float* ln_b_b, float eps, const float* Wp,
                                        const float* Wsk, float scale, float* dSv, float* part_dsv, float* aux,
                                        float* part, void* stream) {
  GASFM_REQUIRE(items && dPo && P && Wp && Wsk && dSv && aux && part && aligned16(dPo) && aligned16(aux),
                "gasfm_edge0_epilogue_bwd: bad args");
  if (n_items <= 0) return GASFM_OK;
  hipLaunchKernelGGL(edge0_epilogue_bwd_kernel, dim3(grid_for(n_items, kT / kW)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), items, n_items, dPo, reinterpret_cast<const float2*>(P),
                     ln_a_w, ln_a_b, ln_b_w, ln_b_b, eps, Wp, Wsk, scale, dSv, part_dsv,
                     reinterpret_cast<float4*>(aux), part);
  return launch_status("gasfm_edge0_epilogue_bwd");
}

extern "C" int gasfm_edge0_prologue_bwd(const float* dXL, const float* P, const float* aux, int64_t E,
                                        const float* ln_w, const float* ln_b, float eps, const float* W0, float* dP,
                                        float* part, void* stream) {
  GASFM_REQUIRE(dXL && P && ln_w && ln_b && W0 && dP && part && aligned16(dXL) && (!aux || aligned16(aux)),
                "gasfm_edge0_prologue_bwd: bad args");
  if (E == 0) return GASFM_OK;
  hipLaunchKernelGGL(edge0_prologue_bwd_kernel, dim3(grid_for(E, kT)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float4*>(dXL),
                     reinterpret_cast<const float2*>(P), reinterpret_cast<const float4*>(aux), E, ln_w, ln_b, eps,
                     W0, reinterpret_cast<float2*>(dP), part);
  return launch_status("gasfm_edge0_prologue_bwd");
}
