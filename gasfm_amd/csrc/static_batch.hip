// Filling a shape-stable union batch (gasfm_amd/static_batch.py), gfx950.
//
// The captured training step replays one graph per BUCKET of fixed sizes; every step writes the
// sampled batch into the bucket's static buffers.  As torch ops that is ~250 small launches per
// 4-scene batch (~2.4 ms of host time); here it is one launch per scene and one for the pad scene:
//   gasfm_union_fill_scene  scene s's edges / measurements / CSRs / point-order permutation with the
//                           union offsets, its pixel measurements gathered from its dense M, its
//                           cameras' Ns^-1 (fp64, as compute_core_errors' host inverse), the scene
//                           maps, its point items and its cameras' work items + combine entries
//                           (ceil(deg / piece) pieces per camera, every camera through partial slots)
//   gasfm_union_fill_pad    the pad scene: mp cameras / npd points / ep edges with degrees spread
//                           evenly, edge k joining the k-th entries of the two degree expansions
//                           (cam-major and point-sorted at once), zero measurements, the remaining
//                           dI camera items spread over the pad cameras
// Every output is written by exactly one thread (no atomics): deterministic.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ void put_item(int32_t* items, int64_t row, int64_t seg, int64_t b, int64_t e,
                                         int64_t slot) {
  int4 v;
  v.x = int(seg);
  v.y = int(b);
  v.z = int(e);
  v.w = int(slot);
  reinterpret_cast<int4*>(items)[row] = v;
}

// camera c's pieces: items first .. first + p - 1 tile [b0, b0 + deg) (plan_work's split)
__device__ __forceinline__ void camera_items(int32_t* items, int32_t* comb, int64_t c, int64_t first, int64_t p,
                                             int64_t b0, int64_t deg) {
  const int64_t base = deg / p, rem = deg % p;
  for (int64_t q = 0; q < p; ++q) {
    const int64_t b = b0 + q * base + (q < rem ? q : rem);
    put_item(items, first + q, c, b, b + base + (q < rem ? 1 : 0), first + q);
  }
  put_item(comb, c, c, first, p, 1);
}

__device__ __forceinline__ void inv3(const float* A, float* out) {
  const double a = A[0], b = A[1], c = A[2], d = A[3], e = A[4], f = A[5], g = A[6], h = A[7], i = A[8];
  const double X = e * i - f * h, Y = f * g - d * i, Z = d * h - e * g;
  const double r = 1.0 / (a * X + b * Y + c * Z);
  const double v[9] = {X, c * h - b * i, b * f - c * e, Y, a * i - c * g, c * d - a * f, Z, b * g - a * h, a * e - b * d};
#pragma unroll
  for (int k = 0; k < 9; ++k) out[k] = float(v[k] * r);
}

__global__ __launch_bounds__(kT) void union_fill_scene_kernel(gasfm_union_scene sc, gasfm_union_out o) {
  extern __shared__ int64_t first[];  // block 0: the scene's camera item offsets
  const int64_t nthr = int64_t(gridDim.x) * kT;
  const int64_t tid = int64_t(blockIdx.x) * kT + threadIdx.x;
  const int64_t hi = sc.E > sc.n ? sc.E : sc.n;
  for (int64_t i = tid; i < (hi > sc.m ? hi : sc.m); i += nthr) {
    if (i < sc.E) {
      const int64_t lc = sc.idx[i], lp = sc.idx[sc.ld_idx + i];
      const int64_t c = lc + sc.c0, p = lp + sc.p0, e = sc.e0 + i;
      o.indices[e] = c;
      o.indices[o.ld_indices + e] = p;
      o.cam32[e] = int32_t(c);
      o.pt32[e] = int32_t(p);
      reinterpret_cast<float2*>(o.values)[e] = reinterpret_cast<const float2*>(sc.vals)[i];
      reinterpret_cast<float2*>(o.values_loss)[e] = reinterpret_cast<const float2*>(sc.vals_loss)[i];
      o.perm[e] = int32_t((sc.perm ? int64_t(sc.perm[i]) : i) + sc.e0);
      o.pos[e] = int32_t((sc.pos ? int64_t(sc.pos[i]) : i) + sc.e0);
      float2 xy = make_float2(0.f, 0.f);
      if (sc.M) {
        xy.x = sc.M[(2 * lc) * sc.ldM + lp];
        xy.y = sc.M[(2 * lc + 1) * sc.ldM + lp];
      }
      reinterpret_cast<float2*>(o.xy)[e] = xy;
    }
    if (i < sc.n) {
      const int64_t p = sc.p0 + i, b = sc.pptr[i] + sc.e0, e = sc.pptr[i + 1] + sc.e0;
      o.pt_ptr[p] = int32_t(b);
      o.cam_per_pts[p] = sc.cam_per_pts[i];
      o.sop32[p] = sc.scene;
      put_item(o.items_p, p, p, b, e, -1);
    }
    if (i < sc.m) {
      const int64_t c = sc.c0 + i;
      o.cam_ptr[c] = int32_t(sc.cptr[i] + sc.e0);
      o.pts_per_cam[c] = sc.pts_per_cam[i];
      o.soc[c] = sc.scene;
      o.soc32[c] = sc.scene;
      inv3(sc.Ns + 9 * i, o.Ns_inv + 9 * c);
    }
  }
  if (blockIdx.x != 0) return;
  // the scene's camera items: a serial prefix of the piece counts (m <= kMaxCams), then one
  // thread per camera writes its pieces
  if (threadIdx.x == 0) {
    int64_t acc = sc.item0;
    for (int64_t i = 0; i < sc.m; ++i) {
      first[i] = acc;
      const int64_t deg = sc.cptr[i + 1] - sc.cptr[i];
      acc += deg > o.piece ? (deg + o.piece - 1) / o.piece : 1;
    }
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < sc.m; i += kT) {
    const int64_t deg = sc.cptr[i + 1] - sc.cptr[i];
    const int64_t p = deg > o.piece ? (deg + o.piece - 1) / o.piece : 1;
    camera_items(o.items_c, o.comb_c, sc.c0 + i, first[i], p, sc.cptr[i] + sc.e0, deg);
  }
}

// the k-th of ep entries spread over cnt slots as evenly as possible (the first ep % cnt get one more)
__device__ __forceinline__ int64_t spread_slot(int64_t k, int64_t ep, int64_t cnt) {
  const int64_t q = ep / cnt, r = ep % cnt;
  return k < r * (q + 1) ? k / (q + 1) : r + (k - r * (q + 1)) / q;
}
__device__ __forceinline__ int64_t spread_start(int64_t j, int64_t ep, int64_t cnt) {
  const int64_t q = ep / cnt, r = ep % cnt;
  return j * q + (j < r ? j : r);
}

__global__ __launch_bounds__(kT) void union_fill_pad_kernel(gasfm_union_pad pd, gasfm_union_out o) {
  const int64_t nthr = int64_t(gridDim.x) * kT;
  const int64_t hi = pd.ep > pd.npd ? pd.ep : pd.npd;
  for (int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x; i < (hi > pd.mp ? hi : pd.mp); i += nthr) {
    if (i < pd.ep) {
      const int64_t c = pd.M + spread_slot(i, pd.ep, pd.mp), p = pd.N + spread_slot(i, pd.ep, pd.npd);
      const int64_t e = pd.E + i;
      o.indices[e] = c;
      o.indices[o.ld_indices + e] = p;
      o.cam32[e] = int32_t(c);
      o.pt32[e] = int32_t(p);
      reinterpret_cast<float2*>(o.values)[e] = make_float2(0.f, 0.f);
      reinterpret_cast<float2*>(o.values_loss)[e] = make_float2(0.f, 0.f);
      reinterpret_cast<float2*>(o.xy)[e] = make_float2(0.f, 0.f);
      o.perm[e] = int32_t(e);
      o.pos[e] = int32_t(e);
    }
    if (i < pd.npd) {
      const int64_t p = pd.N + i, b = pd.E + spread_start(i, pd.ep, pd.npd),
                    e = pd.E + spread_start(i + 1, pd.ep, pd.npd);
      o.pt_ptr[p] = int32_t(b);
      o.cam_per_pts[p] = e - b;
      o.sop32[p] = pd.scene;
      put_item(o.items_p, p, p, b, e, -1);
    }
    if (i < pd.mp) {
      const int64_t c = pd.M + i, b = pd.E + spread_start(i, pd.ep, pd.mp),
                    e = pd.E + spread_start(i + 1, pd.ep, pd.mp);
      o.cam_ptr[c] = int32_t(b);
      o.pts_per_cam[c] = e - b;
      o.soc[c] = pd.scene;
      o.soc32[c] = pd.scene;
      float* ni = o.Ns_inv + 9 * c;
#pragma unroll
      for (int k = 0; k < 9; ++k) ni[k] = (k % 4 == 0) ? 1.f : 0.f;
      const int64_t first = pd.item0 + spread_start(i, pd.dI, pd.mp);
      const int64_t p = spread_start(i + 1, pd.dI, pd.mp) - spread_start(i, pd.dI, pd.mp);
      camera_items(o.items_c, o.comb_c, c, first, p, b, e - b);
    }
    if (i == 0) {
      o.cam_ptr[pd.M + pd.mp] = int32_t(pd.E + pd.ep);
      o.pt_ptr[pd.N + pd.npd] = int32_t(pd.E + pd.ep);
    }
  }
}

int blocks_for(int64_t n) {
  const int64_t b = (n + kT - 1) / kT;
  return int(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_union_fill_scene(const gasfm_union_scene* sc, const gasfm_union_out* out, void* stream) {
  GASFM_REQUIRE(sc && out, "gasfm_union_fill_scene: null argument");
  GASFM_REQUIRE(sc->E >= 0 && sc->m > 0 && sc->n >= 0 && sc->m <= GASFM_UNION_MAX_CAMS,
                "gasfm_union_fill_scene: E=%lld m=%lld n=%lld (m <= %d)", (long long)sc->E, (long long)sc->m,
                (long long)sc->n, GASFM_UNION_MAX_CAMS);
  GASFM_REQUIRE(sc->idx && sc->vals && sc->vals_loss && sc->cptr && sc->pptr && sc->cam_per_pts && sc->pts_per_cam &&
                    sc->Ns,
                "gasfm_union_fill_scene: null input");
  GASFM_REQUIRE(out->piece > 0 && out->indices && out->cam32 && out->pt32 && out->values && out->values_loss &&
                    out->xy && out->perm && out->pos && out->cam_ptr && out->pt_ptr && out->cam_per_pts &&
                    out->pts_per_cam && out->soc && out->soc32 && out->sop32 && out->Ns_inv && out->items_c &&
                    out->comb_c && out->items_p,
                "gasfm_union_fill_scene: null output");
  int64_t hi = sc->E > sc->n ? sc->E : sc->n;
  hi = hi > sc->m ? hi : sc->m;
  hipLaunchKernelGGL(union_fill_scene_kernel, dim3(blocks_for(hi)), dim3(kT), size_t(sc->m) * sizeof(int64_t),
                     reinterpret_cast<hipStream_t>(stream), *sc, *out);
  return launch_status("gasfm_union_fill_scene");
}

extern "C" int gasfm_union_fill_pad(const gasfm_union_pad* pd, const gasfm_union_out* out, void* stream) {
  GASFM_REQUIRE(pd && out, "gasfm_union_fill_pad: null argument");
  GASFM_REQUIRE(pd->mp > 0 && pd->npd > 0 && pd->ep >= pd->mp && pd->ep >= pd->npd && pd->dI >= pd->mp,
                "gasfm_union_fill_pad: mp=%lld npd=%lld ep=%lld dI=%lld", (long long)pd->mp, (long long)pd->npd,
                (long long)pd->ep, (long long)pd->dI);
  GASFM_REQUIRE(pd->ep / pd->mp >= (pd->dI + pd->mp - 1) / pd->mp,
                "gasfm_union_fill_pad: a pad camera would get an empty piece");
  int64_t hi = pd->ep > pd->npd ? pd->ep : pd->npd;
  hi = hi > pd->mp ? hi : pd->mp;
  hipLaunchKernelGGL(union_fill_pad_kernel, dim3(blocks_for(hi)), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream),
                     *pd, *out);
  return launch_status("gasfm_union_fill_pad");
}

// ---- the per-scene global term of a union batch folded into the per-camera term (model._fold_global):
//   forward   out[c] = sv[c] + sg[soc[c]]                       (one thread per value)
//   backward  dsg[s] = sum over the cameras c of scene s of dout[c], in camera order (one workgroup per
//             scene, one thread per column: deterministic, no atomics)
namespace gasfm {
namespace {

__global__ __launch_bounds__(kT) void fold_rows_fwd_kernel(const float* __restrict__ sv, int64_t ldsv,
                                                           const float* __restrict__ sg, int64_t ldsg,
                                                           const int64_t* __restrict__ soc, int64_t m, int width,
                                                           float* __restrict__ out, int64_t ldo) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i >= m * width) return;
  const int64_t c = i / width, j = i % width;
  out[c * ldo + j] = sv[c * ldsv + j] + sg[soc[c] * ldsg + j];
}

__global__ __launch_bounds__(kT) void fold_rows_bwd_kernel(const float* __restrict__ dout, int64_t ld,
                                                           const int64_t* __restrict__ soc, int64_t m, int width,
                                                           float* __restrict__ dsg, int64_t ldsg) {
  const int s = blockIdx.x;
  for (int j = threadIdx.x; j < width; j += kT) {
    float acc = 0.f;
    for (int64_t c = 0; c < m; ++c)
      if (soc[c] == s) acc += dout[c * ld + j];
    dsg[int64_t(s) * ldsg + j] = acc;
  }
}

}  // namespace
}  // namespace gasfm

extern "C" int gasfm_fold_scene_rows_fwd(const float* sv, int64_t ldsv, const float* sg, int64_t ldsg,
                                         const int64_t* soc, int64_t m, int32_t width, float* out, int64_t ldo,
                                         void* stream) {
  GASFM_REQUIRE(sv && sg && soc && out && m >= 0 && width > 0, "gasfm_fold_scene_rows_fwd: bad arguments");
  if (m == 0) return GASFM_OK;
  const int64_t n = m * width;
  hipLaunchKernelGGL(fold_rows_fwd_kernel, dim3(unsigned((n + kT - 1) / kT)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), sv, ldsv, sg, ldsg, soc, m, width, out, ldo);
  return launch_status("gasfm_fold_scene_rows_fwd");
}

extern "C" int gasfm_fold_scene_rows_bwd(const float* dout, int64_t ld, const int64_t* soc, int64_t m, int32_t S,
                                         int32_t width, float* dsg, int64_t ldsg, void* stream) {
  GASFM_REQUIRE(dout && soc && dsg && m >= 0 && S > 0 && width > 0, "gasfm_fold_scene_rows_bwd: bad arguments");
  hipLaunchKernelGGL(fold_rows_bwd_kernel, dim3(S), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream), dout, ld,
                     soc, m, width, dsg, ldsg);
  return launch_status("gasfm_fold_scene_rows_bwd");
}
