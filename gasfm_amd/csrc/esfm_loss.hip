// ESFMLoss (code/loss_functions.py:85-123) as sparse per-edge kernels, gfx950.
//
// The reference forms the dense projections Ps @ pts3D ([m, 3, n]: 2.4 GB at config 4), masks them
// with the dense valid-observation matrix and averages; its backward goes through a gradient hook
// on the [m, 3, n] tensor.  Here every quantity is per visibility edge e = (c, p) (the same E
// edges the network runs on, values[e] = the normalised measurement = norm_M at (c, p)):
//   y_e   = P_c [X_p; w_p]                                        (3-vector)
//   pos_e = y_z >= margin (hinge) or |y_z| >= margin (no hinge)    (geo_utils.py:721-726)
//   l_e   = pos_e ? || y_xy / y_z - m_e || : (margin - y_z) * hinge_w
//   loss  = sum_e l_e / E
// Backward with the reference's hook (pts_grad_equalization_pre_perspective_divide,
// loss_functions.py:104-113): with G_e = dloss * dl_e/dy_e / E (E = E_norm: the global edge count
// when a point-sharded rank passes its own edges),
//   valid-only:  G'_e = pos_e ? normalize(G_e) / max(1, #pos) : G_e
//   otherwise:   G'_e = normalize(G_e) / E
//   none:        G'_e = G_e
// then dP_c = sum_{e in c} G'_e [X_p; w_p]^T (one workgroup per camera, edges in order) and
// d[X_p; w_p] = sum_{e in p} P_c^T G'_e (one thread per point, through the point CSR).
// Deterministic: fixed-order sums, no atomics.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "lanes.hpp"

namespace gasfm {
namespace {

constexpr int kT = 256;

struct EsfmConf {
  float margin, hinge_w;
  int hinge, equalize, valid_only;
};

struct Proj {
  float y[3];
  bool pos;
};

__device__ __forceinline__ Proj project(const float* __restrict__ P, const float* __restrict__ X, int64_t n,
                                        int c, int p, const EsfmConf& k) {
  const float* pc = P + int64_t(c) * 12;
  const float x0 = X[p], x1 = X[n + p], x2 = X[2 * n + p], x3 = X[3 * n + p];
  Proj r;
#pragma unroll
  for (int i = 0; i < 3; ++i) r.y[i] = fmaf(pc[4 * i], x0, fmaf(pc[4 * i + 1], x1, fmaf(pc[4 * i + 2], x2, pc[4 * i + 3] * x3)));
  r.pos = k.hinge ? (r.y[2] >= k.margin) : (fabsf(r.y[2]) >= k.margin);
  return r;
}

// per-edge loss value
__device__ __forceinline__ float edge_value(const Proj& r, float mx, float my, const EsfmConf& k) {
  if (!r.pos) return (k.margin - r.y[2]) * k.hinge_w;
  const float u = r.y[0] / r.y[2] - mx, v = r.y[1] / r.y[2] - my;
  return sqrtf(u * u + v * v);
}

// G'_e (see the header); scale = dloss / E, inv_pos = 1 / max(1, #pos)
__device__ __forceinline__ void edge_grad(const Proj& r, float mx, float my, const EsfmConf& k, float scale,
                                          float inv_pos, float inv_e, float (&g)[3]) {
  float d[3];
  if (r.pos) {
    const float z = r.y[2], iz = 1.f / z;
    const float u = r.y[0] * iz - mx, v = r.y[1] * iz - my;
    const float err = sqrtf(u * u + v * v);
    const float s = err > 0.f ? scale / err : 0.f;  // d||.||/d(u,v) = (u, v)/err (0 at err = 0, as torch)
    d[0] = s * u * iz;
    d[1] = s * v * iz;
    d[2] = -s * (u * r.y[0] + v * r.y[1]) * iz * iz;
  } else {
    d[0] = d[1] = 0.f;
    d[2] = -k.hinge_w * scale;
  }
  if (k.equalize && (r.pos || !k.valid_only)) {
    const float nrm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    const float f = (k.valid_only ? inv_pos : inv_e) / fmaxf(nrm, 1e-12f);  // F.normalize eps
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] *= f;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) g[i] = d[i];
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = group_sum<64>(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < kT / 64; ++w) s += sh[w];
  return s;
}

// per-workgroup partial (sum of l_e, count of pos_e) over a grid-stride slice of the edges
__global__ __launch_bounds__(kT) void esfm_fwd_kernel(const int32_t* __restrict__ cam,
                                                      const int32_t* __restrict__ pt,
                                                      const float* __restrict__ vals, int64_t E,
                                                      const float* __restrict__ P, const float* __restrict__ X,
                                                      int64_t n, EsfmConf k, float* __restrict__ part) {
  __shared__ float sh[kT / 64];
  float s = 0.f, cnt = 0.f;
  for (int64_t e = int64_t(blockIdx.x) * kT + threadIdx.x; e < E; e += int64_t(gridDim.x) * kT) {
    const float2 m = reinterpret_cast<const float2*>(vals)[e];
    const Proj r = project(P, X, n, cam[e], pt[e], k);
    s += edge_value(r, m.x, m.y, k);
    cnt += r.pos ? 1.f : 0.f;
  }
  s = block_sum(s, sh);
  cnt = block_sum(cnt, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = cnt;
  }
}

// dP_c over camera c's contiguous edge range [cptr[c], cptr[c+1]) by the workgroup
__device__ __forceinline__ void cam_grad(const int32_t* __restrict__ cptr, const int32_t* __restrict__ pt,
                                         const float* __restrict__ vals, const float* __restrict__ P,
                                         const float* __restrict__ X, int64_t n, const EsfmConf& k, int c,
                                         float scale, float inv_pos, float inv_e, float* __restrict__ dP) {
  __shared__ float sh[kT / 64 * 12];
  float acc[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = 0.f;
  for (int e = cptr[c] + threadIdx.x; e < cptr[c + 1]; e += kT) {
    const float2 m = reinterpret_cast<const float2*>(vals)[e];
    const int p = pt[e];
    const Proj r = project(P, X, n, c, p, k);
    float g[3];
    edge_grad(r, m.x, m.y, k, scale, inv_pos, inv_e, g);
    const float xs[4] = {X[p], X[n + p], X[2 * n + p], X[3 * n + p]};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 * i + j] = fmaf(g[i], xs[j], acc[4 * i + j]);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = group_sum<64>(acc[i]);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 12; ++i) sh[wave * 12 + i] = acc[i];
  __syncthreads();
  if (threadIdx.x < 12) {
    float s = 0.f;
    for (int w = 0; w < kT / 64; ++w) s += sh[w * 12 + threadIdx.x];
    dP[int64_t(c) * 12 + threadIdx.x] = s;
  }
}

// d pts3D[:, p] over point p's edges in CSR order (perm: edge ids)
__device__ __forceinline__ void pt_grad(const int32_t* __restrict__ pptr, const int32_t* __restrict__ perm,
                                        const int32_t* __restrict__ cam, const float* __restrict__ vals,
                                        const float* __restrict__ P, const float* __restrict__ X, int64_t n,
                                        const EsfmConf& k, int64_t p, float scale, float inv_pos, float inv_e,
                                        float* __restrict__ dX) {
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (int q = pptr[p]; q < pptr[p + 1]; ++q) {
    const int e = perm ? perm[q] : q;
    const float2 m = reinterpret_cast<const float2*>(vals)[e];
    const int c = cam[e];
    const Proj r = project(P, X, n, c, int(p), k);
    float g[3];
    edge_grad(r, m.x, m.y, k, scale, inv_pos, inv_e, g);
    const float* pc = P + int64_t(c) * 12;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = fmaf(pc[j], g[0], fmaf(pc[4 + j], g[1], fmaf(pc[8 + j], g[2], a[j])));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) dX[j * n + p] = a[j];
}

// dP_c: one workgroup per camera
__global__ __launch_bounds__(kT) void esfm_bwd_cam_kernel(const int32_t* __restrict__ cptr,
                                                          const int32_t* __restrict__ pt,
                                                          const float* __restrict__ vals, int64_t E_norm,
                                                          const float* __restrict__ P, const float* __restrict__ X,
                                                          int64_t n, EsfmConf k, const float* __restrict__ dloss,
                                                          const float* __restrict__ tot, float* __restrict__ dP) {
  const float inv_e = 1.f / float(E_norm), scale = dloss[0] * inv_e, inv_pos = 1.f / fmaxf(1.f, tot[1]);
  cam_grad(cptr, pt, vals, P, X, n, k, blockIdx.x, scale, inv_pos, inv_e, dP);
}

// d pts3D[:, p]: one thread per point
__global__ __launch_bounds__(kT) void esfm_bwd_pt_kernel(const int32_t* __restrict__ pptr,
                                                         const int32_t* __restrict__ perm,
                                                         const int32_t* __restrict__ cam,
                                                         const float* __restrict__ vals, int64_t E_norm,
                                                         const float* __restrict__ P, const float* __restrict__ X,
                                                         int64_t n, EsfmConf k, const float* __restrict__ dloss,
                                                         const float* __restrict__ tot, float* __restrict__ dX) {
  const int64_t p = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (p >= n) return;
  const float inv_e = 1.f / float(E_norm), scale = dloss[0] * inv_e, inv_pos = 1.f / fmaxf(1.f, tot[1]);
  pt_grad(pptr, perm, cam, vals, P, X, n, k, p, scale, inv_pos, inv_e, dX);
}

// ---- several scenes in one edge list (a union batch): scene s owns edges [eoff[s], eoff[s+1]),
// its cameras / points are the ones scene_of_cam / scene_of_pt map to s.  The batch loss is
// sum_s weight[s] * loss_s; a scene of weight 0 (padding) contributes nothing, and its cameras'
// and points' gradients are written as zeros without reading its projections.
constexpr int kSegG = 32;  // workgroups per scene in the segmented sums

// part[(s * kSegG + g)] = (sum of l_e, count of pos_e) over scene s's edges, slice g
__global__ __launch_bounds__(kT) void esfm_fwd_seg_kernel(const int32_t* __restrict__ cam,
                                                          const int32_t* __restrict__ pt,
                                                          const float* __restrict__ vals,
                                                          const int32_t* __restrict__ eoff,
                                                          const float* __restrict__ P, const float* __restrict__ X,
                                                          int64_t n, EsfmConf k, float* __restrict__ part) {
  __shared__ float sh[kT / 64];
  const int s = blockIdx.y;
  const int64_t e1 = eoff[s + 1];
  float sum = 0.f, cnt = 0.f;
  for (int64_t e = eoff[s] + int64_t(blockIdx.x) * kT + threadIdx.x; e < e1; e += int64_t(kSegG) * kT) {
    const float2 m = reinterpret_cast<const float2*>(vals)[e];
    const Proj r = project(P, X, n, cam[e], pt[e], k);
    sum += edge_value(r, m.x, m.y, k);
    cnt += r.pos ? 1.f : 0.f;
  }
  sum = block_sum(sum, sh);
  cnt = block_sum(cnt, sh);
  if (threadIdx.x == 0) {
    const int64_t row = int64_t(s) * kSegG + blockIdx.x;
    part[2 * row] = sum;
    part[2 * row + 1] = cnt;
  }
}

// tot[s] = ordered sum of scene s's kSegG partials; loss (optional) = sum over the scenes of
// weight nonzero of weight[s] * tot[s][0] / E_s, in scene order.  One workgroup, S <= kT.
__global__ __launch_bounds__(kT) void seg_total_kernel(const float* __restrict__ part, int S,
                                                       const int32_t* __restrict__ eoff,
                                                       const float* __restrict__ weight, float* __restrict__ tot,
                                                       float* __restrict__ loss) {
  __shared__ float sh[kT];
  const int s = threadIdx.x;
  if (s < S) {
    float a = 0.f, b = 0.f;
    for (int g = 0; g < kSegG; ++g) {
      a += part[2 * (int64_t(s) * kSegG + g)];
      b += part[2 * (int64_t(s) * kSegG + g) + 1];
    }
    tot[2 * s] = a;
    tot[2 * s + 1] = b;
    sh[s] = a;
  }
  __syncthreads();
  if (loss && threadIdx.x == 0) {
    float L = 0.f;
    for (int q = 0; q < S; ++q) {
      const float w = weight[q];
      if (w != 0.f) L += w * (sh[q] / float(eoff[q + 1] - eoff[q]));
    }
    loss[0] = L;
  }
}

struct SegScale {
  bool skip;
  float scale, inv_pos, inv_e;
};

__device__ __forceinline__ SegScale seg_scale(int s, const int32_t* __restrict__ eoff,
                                              const float* __restrict__ weight, const float* __restrict__ dloss,
                                              const float* __restrict__ tot) {
  SegScale r;
  const float w = weight[s];
  r.skip = w == 0.f;
  r.inv_e = 1.f / float(eoff[s + 1] - eoff[s]);
  r.scale = dloss[0] * w * r.inv_e;
  r.inv_pos = 1.f / fmaxf(1.f, tot[2 * s + 1]);
  return r;
}

__global__ __launch_bounds__(kT) void esfm_bwd_cam_seg_kernel(
    const int32_t* __restrict__ cptr, const int32_t* __restrict__ pt, const float* __restrict__ vals,
    const int32_t* __restrict__ eoff, const int32_t* __restrict__ scene_of_cam, const float* __restrict__ weight,
    const float* __restrict__ P, const float* __restrict__ X, int64_t n, EsfmConf k,
    const float* __restrict__ dloss, const float* __restrict__ tot, float* __restrict__ dP) {
  const int c = blockIdx.x;
  const SegScale sc = seg_scale(scene_of_cam[c], eoff, weight, dloss, tot);
  if (sc.skip) {
    if (threadIdx.x < 12) dP[int64_t(c) * 12 + threadIdx.x] = 0.f;
    return;
  }
  cam_grad(cptr, pt, vals, P, X, n, k, c, sc.scale, sc.inv_pos, sc.inv_e, dP);
}

__global__ __launch_bounds__(kT) void esfm_bwd_pt_seg_kernel(
    const int32_t* __restrict__ pptr, const int32_t* __restrict__ perm, const int32_t* __restrict__ cam,
    const float* __restrict__ vals, const int32_t* __restrict__ eoff, const int32_t* __restrict__ scene_of_pt,
    const float* __restrict__ weight, const float* __restrict__ P, const float* __restrict__ X, int64_t n,
    EsfmConf k, const float* __restrict__ dloss, const float* __restrict__ tot, float* __restrict__ dX) {
  const int64_t p = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (p >= n) return;
  const SegScale sc = seg_scale(scene_of_pt[p], eoff, weight, dloss, tot);
  if (sc.skip) {
#pragma unroll
    for (int j = 0; j < 4; ++j) dX[j * n + p] = 0.f;
    return;
  }
  pt_grad(pptr, perm, cam, vals, P, X, n, k, p, sc.scale, sc.inv_pos, sc.inv_e, dX);
}

// compute_core_errors' "our_repro" (code/evaluation.py:8-31; geo_utils.py:371-391): per edge
//   X = pts3D[:, p] / pts3D[3, p]   (pflat)      y = Ps_pix[c] X      err = ||xy - y_xy / y_z||
// with Ps_pix = Ns^-1 Ps_norm (pixel-space cameras, caller-supplied) and xy the PIXEL
// measurement of the edge.  err[e] is written when err != NULL; the workgroup partial is
// (sum of the non-NaN errors, their count): np.nanmean's operands.  An inf error (y_z == 0,
// y_xy != 0) is summed like numpy does.
__device__ __forceinline__ float reproj_edge(const int32_t* __restrict__ cam, const int32_t* __restrict__ pt,
                                             const float* __restrict__ xy, const float* __restrict__ P,
                                             const float* __restrict__ X, int64_t n, int64_t e) {
  const float2 m = reinterpret_cast<const float2*>(xy)[e];
  const int c = cam[e], p = pt[e];
  const float w = X[3 * n + p];
  const float x0 = X[p] / w, x1 = X[n + p] / w, x2 = X[2 * n + p] / w;
  const float* pc = P + int64_t(c) * 12;
  float y[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) y[i] = fmaf(pc[4 * i], x0, fmaf(pc[4 * i + 1], x1, fmaf(pc[4 * i + 2], x2, pc[4 * i + 3])));
  const float u = m.x - y[0] / y[2], v = m.y - y[1] / y[2];
  return sqrtf(u * u + v * v);
}

__global__ __launch_bounds__(kT) void reproj_kernel(const int32_t* __restrict__ cam, const int32_t* __restrict__ pt,
                                                    const float* __restrict__ xy, int64_t E,
                                                    const float* __restrict__ P, const float* __restrict__ X,
                                                    int64_t n, float* __restrict__ err, float* __restrict__ part) {
  __shared__ float sh[kT / 64];
  float s = 0.f, cnt = 0.f;
  for (int64_t e = int64_t(blockIdx.x) * kT + threadIdx.x; e < E; e += int64_t(gridDim.x) * kT) {
    const float r = reproj_edge(cam, pt, xy, P, X, n, e);
    if (err) err[e] = r;
    if (!isnan(r)) {
      s += r;
      cnt += 1.f;
    }
  }
  s = block_sum(s, sh);
  cnt = block_sum(cnt, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = cnt;
  }
}

// the same per scene of a union batch: part[(s * kSegG + g)] over scene s's edges, slice g
__global__ __launch_bounds__(kT) void reproj_seg_kernel(const int32_t* __restrict__ cam,
                                                        const int32_t* __restrict__ pt,
                                                        const float* __restrict__ xy,
                                                        const int32_t* __restrict__ eoff,
                                                        const float* __restrict__ P, const float* __restrict__ X,
                                                        int64_t n, float* __restrict__ part) {
  __shared__ float sh[kT / 64];
  const int s = blockIdx.y;
  const int64_t e1 = eoff[s + 1];
  float sum = 0.f, cnt = 0.f;
  for (int64_t e = eoff[s] + int64_t(blockIdx.x) * kT + threadIdx.x; e < e1; e += int64_t(kSegG) * kT) {
    const float r = reproj_edge(cam, pt, xy, P, X, n, e);
    if (!isnan(r)) {
      sum += r;
      cnt += 1.f;
    }
  }
  sum = block_sum(sum, sh);
  cnt = block_sum(cnt, sh);
  if (threadIdx.x == 0) {
    const int64_t row = int64_t(s) * kSegG + blockIdx.x;
    part[2 * row] = sum;
    part[2 * row + 1] = cnt;
  }
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int32_t gasfm_esfm_part_rows(int64_t E) {
  const int64_t b = (E + kT - 1) / kT;
  return int32_t(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

extern "C" int gasfm_esfm_fwd(const int32_t* cam, const int32_t* pt, const float* vals, int64_t E, const float* P,
                              const float* X, int64_t n, float margin, float hinge_w, int32_t hinge, float* part,
                              void* stream) {
  GASFM_REQUIRE(E > 0 && n > 0, "gasfm_esfm_fwd: E=%lld n=%lld", (long long)E, (long long)n);
  GASFM_REQUIRE(cam && pt && vals && P && X && part, "gasfm_esfm_fwd: null pointer");
  GASFM_REQUIRE((reinterpret_cast<uintptr_t>(vals) & 7) == 0, "gasfm_esfm_fwd: vals must be 8-byte aligned");
  const EsfmConf k{margin, hinge_w, hinge, 0, 0};
  hipLaunchKernelGGL(esfm_fwd_kernel, dim3(gasfm_esfm_part_rows(E)), dim3(kT), 0,
                     reinterpret_cast<hipStream_t>(stream), cam, pt, vals, E, P, X, n, k, part);
  return launch_status("gasfm_esfm_fwd");
}

extern "C" int gasfm_esfm_bwd(const int32_t* cptr, int32_t m, const int32_t* pptr, const int32_t* perm,
                              const int32_t* cam, const int32_t* pt, const float* vals, int64_t E, int64_t E_norm,
                              const float* P, const float* X, int64_t n, float margin, float hinge_w, int32_t hinge,
                              int32_t equalize, int32_t valid_only, const float* dloss, const float* tot, float* dP,
                              float* dX, void* stream) {
  GASFM_REQUIRE(E > 0 && n > 0 && m > 0 && E_norm >= E, "gasfm_esfm_bwd: E=%lld E_norm=%lld m=%d n=%lld",
                (long long)E, (long long)E_norm, m, (long long)n);
  GASFM_REQUIRE(cptr && pptr && cam && pt && vals && P && X && dloss && tot && dP && dX, "gasfm_esfm_bwd: null pointer");
  const EsfmConf k{margin, hinge_w, hinge, equalize, valid_only};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(esfm_bwd_cam_kernel, dim3(m), dim3(kT), 0, st, cptr, pt, vals, E_norm, P, X, n, k, dloss, tot,
                     dP);
  hipLaunchKernelGGL(esfm_bwd_pt_kernel, dim3(unsigned((n + kT - 1) / kT)), dim3(kT), 0, st, pptr, perm, cam, vals,
                     E_norm, P, X, n, k, dloss, tot, dX);
  return launch_status("gasfm_esfm_bwd");
}

extern "C" int gasfm_reproj_error(const int32_t* cam, const int32_t* pt, const float* xy, int64_t E, const float* P,
                                  const float* pts3D, int64_t n, float* err, float* part, void* stream) {
  GASFM_REQUIRE(E >= 0 && n >= 0 && (E == 0 || (cam && pt && xy && P && pts3D)) && part,
                "gasfm_reproj_error: bad args");
  hipLaunchKernelGGL(reproj_kernel, dim3(gasfm_esfm_part_rows(E)), dim3(kT), 0, (hipStream_t)stream, cam, pt, xy, E,
                     P, pts3D, n, err, part);
  return launch_status("gasfm_reproj_error");
}

extern "C" int32_t gasfm_esfm_seg_part_rows(int32_t S) { return S * kSegG; }

extern "C" int gasfm_esfm_seg_fwd(const int32_t* cam, const int32_t* pt, const float* vals, const int32_t* eoff,
                                  int32_t S, const float* weight, const float* P, const float* X, int64_t n,
                                  float margin, float hinge_w, int32_t hinge, float* part, float* tot, float* loss,
                                  void* stream) {
  GASFM_REQUIRE(S > 0 && S <= kT && n > 0, "gasfm_esfm_seg_fwd: S=%d n=%lld", S, (long long)n);
  GASFM_REQUIRE(cam && pt && vals && eoff && weight && P && X && part && tot && loss, "gasfm_esfm_seg_fwd: null pointer");
  GASFM_REQUIRE((reinterpret_cast<uintptr_t>(vals) & 7) == 0, "gasfm_esfm_seg_fwd: vals must be 8-byte aligned");
  const EsfmConf k{margin, hinge_w, hinge, 0, 0};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(esfm_fwd_seg_kernel, dim3(kSegG, S), dim3(kT), 0, st, cam, pt, vals, eoff, P, X, n, k, part);
  hipLaunchKernelGGL(seg_total_kernel, dim3(1), dim3(kT), 0, st, part, S, eoff, weight, tot, loss);
  return launch_status("gasfm_esfm_seg_fwd");
}

extern "C" int gasfm_esfm_seg_bwd(const int32_t* cam_ptr, int32_t m, const int32_t* pt_ptr, const int32_t* perm,
                                  const int32_t* cam, const int32_t* pt, const float* vals, const int32_t* eoff,
                                  int32_t S, const int32_t* scene_of_cam, const int32_t* scene_of_pt,
                                  const float* weight, const float* P, const float* X, int64_t n, float margin,
                                  float hinge_w, int32_t hinge, int32_t equalize, int32_t valid_only,
                                  const float* dloss, const float* tot, float* dP, float* dX, void* stream) {
  GASFM_REQUIRE(S > 0 && m > 0 && n > 0, "gasfm_esfm_seg_bwd: S=%d m=%d n=%lld", S, m, (long long)n);
  GASFM_REQUIRE(cam_ptr && pt_ptr && cam && pt && vals && eoff && scene_of_cam && scene_of_pt && weight && P && X &&
                    dloss && tot && dP && dX,
                "gasfm_esfm_seg_bwd: null pointer");
  const EsfmConf k{margin, hinge_w, hinge, equalize, valid_only};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(esfm_bwd_cam_seg_kernel, dim3(m), dim3(kT), 0, st, cam_ptr, pt, vals, eoff, scene_of_cam, weight,
                     P, X, n, k, dloss, tot, dP);
  hipLaunchKernelGGL(esfm_bwd_pt_seg_kernel, dim3(unsigned((n + kT - 1) / kT)), dim3(kT), 0, st, pt_ptr, perm, cam,
                     vals, eoff, scene_of_pt, weight, P, X, n, k, dloss, tot, dX);
  return launch_status("gasfm_esfm_seg_bwd");
}

extern "C" int gasfm_reproj_error_seg(const int32_t* cam, const int32_t* pt, const float* xy, const int32_t* eoff,
                                      int32_t S, const float* P, const float* pts3D, int64_t n, float* part,
                                      float* tot, void* stream) {
  GASFM_REQUIRE(S > 0 && S <= kT && n > 0 && cam && pt && xy && eoff && P && pts3D && part && tot,
                "gasfm_reproj_error_seg: bad args");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(reproj_seg_kernel, dim3(kSegG, S), dim3(kT), 0, st, cam, pt, xy, eoff, P, pts3D, n, part);
  hipLaunchKernelGGL(seg_total_kernel, dim3(1), dim3(kT), 0, st, part, S, eoff, nullptr, tot, nullptr);
  return launch_status("gasfm_reproj_error_seg");
}
