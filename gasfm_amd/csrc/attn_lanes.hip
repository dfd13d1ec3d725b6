// Block 0's point-direction GATv2 attention (H = 4 heads of C = 1, 16-byte XL rows): one LANE
// per work item instead of one wave.
//
// Block 0 of every GASFM conf attends over 2-wide embedded projections projected to H*C = 4
// (reference code/models/layers.py:329-335, 426-432 with n_feat_proj_in = 2).  The general
// kernels (gat_attn.hip, Geom<4,1>) give each ~20-edge point segment a whole 64-lane wave: 20
// lanes load one 16-byte row each, then six cross-lane merge steps of the four (max, sum, acc)
// states run for one point -- 226 us for 64 MB of XL at config 4.  Here lane i walks item i's
// edges itself: an online softmax per head in registers, four rows requested per loop step
// (clamped addresses, masked values), no cross-lane work.  Consecutive lanes take consecutive
// points, whose rows are consecutive ranges of the point-ordered XL half, so a wave's loads stay
// within a few KB (L1/L2) and every byte of XL is read from HBM once.
//
// Same outputs and conventions as attn_fwd_kernel / attn_bwd_kernel: finalize (out, seg_max,
// seg_sum) for whole segments, packed partial rows [acc 4 | max 4 | sum 4] for split pieces,
// per-wave (datt | dbias) partial rows in the backward (dbias counted once per segment, on its
// first item).  Fixed summation order per lane: deterministic.
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.hpp"
#include "lanes.hpp"

extern "C" int gasfm_gat_attn_bwd_waves(int32_t n_items, int32_t H, int32_t C);

namespace gasfm {
namespace {

constexpr int kT = 256;
constexpr int kU = 4;  // rows in flight per lane

__device__ __forceinline__ float leaky4(float z, float slope) { return z > 0.f ? z : z * slope; }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float comp(const float4& v, int h) {
  return h == 0 ? v.x : (h == 1 ? v.y : (h == 2 ? v.z : v.w));
}

// G lanes per work item (GASFM_ATTN_FWD_LANES_G; 1 = one lane per item): lane `sub` runs the online
// softmax over the item's edges sub, sub + G, ..., then the group's (max, sum, acc) states merge by
// an xor butterfly (fixed order).
#ifndef GASFM_ATTN_FWD_LANES_G
#define GASFM_ATTN_FWD_LANES_G 8
#endif
template <int G>
__global__ __launch_bounds__(kT) void attn_fwd_lanes_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, float slope, int finalize, float* __restrict__ out,
    int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  const float4 a4 = ld4(att);
  const float a[4] = {a4.x, a4.y, a4.z, a4.w};
  const int sub = threadIdx.x & (G - 1);
  const int ngroups = gridDim.x * (kT / G);
  for (int it = (blockIdx.x * kT + threadIdx.x) / G; it < n_items; it += ngroups) {
    const gasfm_work_item w = items[it];
    const float4 xr4 = ld4(XR + int64_t(w.seg) * ldXR);
    const float xr[4] = {xr4.x, xr4.y, xr4.z, xr4.w};
    float m[4], s[4], acc[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      m[h] = -INFINITY;
      s[h] = 0.f;
      acc[h] = 0.f;
    }
    const int last = w.end - 1;
    for (int e0 = w.begin + sub; e0 < w.end; e0 += G * kU) {
      float4 x[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + G * u < last ? e0 + G * u : last;
        const int64_t src = perm ? int64_t(perm[e]) : int64_t(e);
        x[u] = ld4(XL + src * ldXL);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (e0 + G * u >= w.end) break;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const float xv = comp(x[u], h);
          const float l = a[h] * leaky4(xv + xr[h], slope);
          const float mn = fmaxf(m[h], l);
          const float f = m[h] == -INFINITY ? 0.f : __expf(m[h] - mn);
          const float p = __expf(l - mn);
          s[h] = fmaf(s[h], f, p);
          acc[h] = fmaf(acc[h], f, p * xv);
          m[h] = mn;
        }
      }
    }
    if (G > 1) {  // merge the group's states (a lane without edges has m = -inf, s = acc = 0)
#pragma unroll
      for (int o = 1; o < G; o *= 2) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const float m2 = __shfl_xor(m[h], o), s2 = __shfl_xor(s[h], o), a2 = __shfl_xor(acc[h], o);
          const float mn = fmaxf(m[h], m2);
          const float f1 = m[h] == -INFINITY ? 0.f : __expf(m[h] - mn);
          const float f2 = m2 == -INFINITY ? 0.f : __expf(m2 - mn);
          s[h] = fmaf(s[h], f1, s2 * f2);
          acc[h] = fmaf(acc[h], f1, a2 * f2);
          m[h] = mn;
        }
      }
    }
    if (sub != 0) continue;
    if (w.slot < 0) {
      float o[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) o[h] = finalize ? fmaf(acc[h], 1.f / (s[h] + 1e-16f), bias[h]) : acc[h];
      *reinterpret_cast<float4*>(out + int64_t(w.seg) * ldOut) = make_float4(o[0], o[1], o[2], o[3]);
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        seg_max[int64_t(w.seg) * ldStat + h] = m[h];
        seg_sum[int64_t(w.seg) * ldStat + h] = s[h];
      }
    } else {
      float* pr = part + int64_t(w.slot) * 12;
      *reinterpret_cast<float4*>(pr) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(pr + 4) = make_float4(m[0], m[1], m[2], m[3]);
      *reinterpret_cast<float4*>(pr + 8) = make_float4(s[0], s[1], s[2], s[3]);
    }
  }
}

//   alpha = exp(l - M) / (S + 1e-16);  delta = g . (out - bias) per head;  de = alpha (g x - delta)
//   dz = de att leaky'(z);  dXL = alpha g + dz;  dXR = sum dz;  datt += de leaky(z)
// G lanes per work item (round 3: G = 8, GASFM_ATTN_BWD_LANES_G): lane `sub` of the group takes the
// item's edges sub, sub + G, ...; a group's G rows per step are consecutive (one 128-B line of the
// point-ordered XL half, where G = 1 reads 64 lines per instruction), the per-item dXR sums over
// the group's lanes (xor butterfly, fixed order).
#ifndef GASFM_ATTN_BWD_LANES_G
#define GASFM_ATTN_BWD_LANES_G 8
#endif
template <int G>
__global__ __launch_bounds__(kT) void attn_bwd_lanes_kernel(
    const float* __restrict__ XL, int64_t ldXL, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, const int32_t* __restrict__ perm,
    const gasfm_work_item* __restrict__ items, int n_items, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum,
    const float* __restrict__ gout, int64_t ldG, float* __restrict__ dXL, int64_t ldDXL, float* __restrict__ dXR,
    int64_t ldDXR, float* __restrict__ part_dxr, float* __restrict__ datt_part, int xl_pos) {
  const float4 a4 = ld4(att), b4 = ld4(bias);
  const float a[4] = {a4.x, a4.y, a4.z, a4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
  float datt[4] = {0.f, 0.f, 0.f, 0.f}, dbias[4] = {0.f, 0.f, 0.f, 0.f};
  const int sub = threadIdx.x & (G - 1);
  const int ngroups = gridDim.x * (kT / G);
  for (int it = (blockIdx.x * kT + threadIdx.x) / G; it < n_items; it += ngroups) {
    const gasfm_work_item w = items[it];
    const int64_t sg = w.seg;
    const float4 xr4 = ld4(XR + sg * ldXR), g4 = ld4(gout + sg * ldG), o4 = ld4(out + sg * ldOut);
    const float xr[4] = {xr4.x, xr4.y, xr4.z, xr4.w}, g[4] = {g4.x, g4.y, g4.z, g4.w};
    const float o[4] = {o4.x, o4.y, o4.z, o4.w};
    float M[4], inv[4], delta[4], dxr[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      M[h] = seg_max[sg * 4 + h];
      inv[h] = 1.f / (seg_sum[sg * 4 + h] + 1e-16f);
      delta[h] = g[h] * (o[h] - bv[h]);
      dxr[h] = 0.f;
    }
    if (sub == 0 && (it == 0 || items[it - 1].seg != w.seg)) {
#pragma unroll
      for (int h = 0; h < 4; ++h) dbias[h] += g[h];
    }
    const int last = w.end - 1;
    for (int e0 = w.begin + sub; e0 < w.end; e0 += G * kU) {
      float4 x[kU];
      int64_t src[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + G * u < last ? e0 + G * u : last;
        src[u] = perm ? int64_t(perm[e]) : int64_t(e);
        x[u] = ld4(XL + (xl_pos ? int64_t(e) : src[u]) * ldXL);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (e0 + G * u >= w.end) break;
        float dx[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const float xv = comp(x[u], h);
          const float z = xv + xr[h];
          const float lz = leaky4(z, slope);
          const float alpha = __expf(a[h] * lz - M[h]) * inv[h];
          const float de = alpha * (g[h] * xv - delta[h]);
          const float dz = de * a[h] * (z > 0.f ? 1.f : slope);
          dx[h] = fmaf(alpha, g[h], dz);
          dxr[h] += dz;
          datt[h] = fmaf(de, lz, datt[h]);
        }
        *reinterpret_cast<float4*>(dXL + src[u] * ldDXL) = make_float4(dx[0], dx[1], dx[2], dx[3]);
      }
    }
    if (G > 1) {
#pragma unroll
      for (int h = 0; h < 4; ++h) dxr[h] = group_sum<G>(dxr[h]);
    }
    if (sub == 0) {
      if (w.slot < 0)
        *reinterpret_cast<float4*>(dXR + sg * ldDXR) = make_float4(dxr[0], dxr[1], dxr[2], dxr[3]);
      else
        *reinterpret_cast<float4*>(part_dxr + int64_t(w.slot) * 4) = make_float4(dxr[0], dxr[1], dxr[2], dxr[3]);
    }
  }
  // per-wave partial row [datt 4 | dbias 4] (lane sums in xor-butterfly order: deterministic)
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    datt[h] = xor_sum_from<1>(datt[h]);
    dbias[h] = xor_sum_from<1>(dbias[h]);
  }
  const int wave = (blockIdx.x * kT + threadIdx.x) / 64;
  if ((threadIdx.x & 63) == 0) {
    float* p = datt_part + int64_t(wave) * 8;
    *reinterpret_cast<float4*>(p) = make_float4(datt[0], datt[1], datt[2], datt[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(dbias[0], dbias[1], dbias[2], dbias[3]);
  }
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_gat_attn_fwd_lanes(const float* XL, int64_t ldXL, const float* XR, int64_t ldXR,
                                        const float* att, const float* bias, const int32_t* perm,
                                        const gasfm_work_item* items, int32_t n_items, int32_t H, int32_t C,
                                        float slope, int32_t finalize, float* out, int64_t ldOut, float* seg_max,
                                        float* seg_sum, int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(H == 4 && C == 1 && n_items >= 0, "gasfm_gat_attn_fwd_lanes: H=%d C=%d (4 x 1 only)", H, C);
  if (n_items == 0) return GASFM_OK;
  GASFM_REQUIRE(XL && XR && att && items && ((out && seg_max && seg_sum && bias) || part),
                "gasfm_gat_attn_fwd_lanes: null pointer");
  GASFM_REQUIRE(ldXL % 4 == 0 && ldXR % 4 == 0 && (!out || ldOut % 4 == 0) && aligned16(XL) && aligned16(XR) &&
                    aligned16(att) && (!out || aligned16(out)) && (!part || aligned16(part)) && (!bias || aligned16(bias)),
                "gasfm_gat_attn_fwd_lanes: 16-byte rows required");
  constexpr int G = GASFM_ATTN_FWD_LANES_G;
  const int grid = resident_grid(reinterpret_cast<const void*>(&attn_fwd_lanes_kernel<G>), kT, 0, n_items, kT / G);
  note_dispatch(GASFM_K_ATTN_FWD_LANES);
  hipLaunchKernelGGL(attn_fwd_lanes_kernel<G>, dim3(grid), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream), XL, ldXL,
                     XR, ldXR, att, bias, perm, items, n_items, slope, finalize, out, ldOut, seg_max, seg_sum, ldStat,
                     part);
  return launch_status("gasfm_gat_attn_fwd_lanes");
}

// The grid is the general backward's (gasfm_gat_attn_bwd_waves / 4 workgroups), so the caller's
// datt_part rows (one per wave) are all written.
extern "C" int gasfm_gat_attn_bwd_lanes(const float* XL, int64_t ldXL, const float* XR, int64_t ldXR,
                                        const float* att, const float* bias, const int32_t* perm,
                                        const gasfm_work_item* items, int32_t n_items, int32_t H, int32_t C,
                                        float slope, const float* out, int64_t ldOut, const float* seg_max,
                                        const float* seg_sum, const float* gout, int64_t ldG, float* dXL,
                                        int64_t ldDXL, float* dXR, int64_t ldDXR, float* part_dxr,
                                        float* datt_part, int32_t xl_by_position, void* stream) {
  GASFM_REQUIRE(H == 4 && C == 1 && n_items >= 0, "gasfm_gat_attn_bwd_lanes: H=%d C=%d (4 x 1 only)", H, C);
  if (n_items == 0) return GASFM_OK;
  GASFM_REQUIRE(XL && XR && att && bias && items && out && seg_max && seg_sum && gout && dXL && dXR && datt_part,
                "gasfm_gat_attn_bwd_lanes: null pointer");
  GASFM_REQUIRE(ldXL % 4 == 0 && ldXR % 4 == 0 && ldOut % 4 == 0 && ldG % 4 == 0 && ldDXL % 4 == 0 &&
                    ldDXR % 4 == 0 && aligned16(XL) && aligned16(XR) && aligned16(out) && aligned16(gout) &&
                    aligned16(dXL) && aligned16(dXR) && aligned16(att) && aligned16(bias) && aligned16(datt_part) &&
                    (!part_dxr || aligned16(part_dxr)),
                "gasfm_gat_attn_bwd_lanes: 16-byte rows required");
  const int waves = gasfm_gat_attn_bwd_waves(n_items, H, C);
  GASFM_REQUIRE(waves > 0 && waves % (kT / 64) == 0, "gasfm_gat_attn_bwd_lanes: wave count %d", waves);
  note_dispatch(GASFM_K_ATTN_BWD_LANES);
  hipLaunchKernelGGL(attn_bwd_lanes_kernel<GASFM_ATTN_BWD_LANES_G>, dim3(waves / (kT / 64)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), XL, ldXL, XR, ldXR, att, bias, perm, items, n_items, slope,
                     out, ldOut, seg_max, seg_sum, gout, ldG, dXL, ldDXL, dXR, ldDXR, part_dxr, datt_part,
                     int(xl_by_position != 0));
  return launch_status("gasfm_gat_attn_bwd_lanes");
}
