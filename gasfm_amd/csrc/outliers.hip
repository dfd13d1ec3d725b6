// Outlier injection on the device, gfx950 (SURVEY.md §8(f) rank 3, config 5's per-sample transform).
//
// Replaces the reference's CPU/torch-sparse OutlierInjector (code/utils/dataset_utils.py:159-433,
// called per training sample at train.py:73-81).  The partition of the E projections is one
// byte per edge (0 fixed inlier, 1 fixed outlier, 2 free inlier, 3 free outlier; bit 0 = outlier)
// instead of four boolean masks and repeated sparse COO coalesce / sum / to_dense passes.
//
//   outlier_counts     inliers per view (one wave per camera segment: edges are camera-major)
//                      and per point (one thread per point over its CSR slots), plus the minima
//                      of both (verify_enough_points_per_view / _views_per_point, :240-251)
//   outlier_mark       init (:253-269): fixed inlier iff the point has < 3 views or the view
//                      < 9 points, else free inlier; or blacklist (:307-320): a free outlier on
//                      a point with < 2 / a view with < 8 remaining inliers becomes a fixed
//                      inlier.  Both also count the four classes.
//   outlier_moments    per view (one wave per camera): Bessel-corrected raw second moment and
//                      mean of the inliers (sparse_moment_estimation, sparse_utils.py:151-165),
//                      fp64 sums; LDL^T by LAPACK sytf2's Bunch-Kaufman rule as
//                      torch.linalg.ldl_factor, scale_tril = L sqrt(D) with the row flip of
//                      the interchanged case (:378-392)
//   outlier_apply      outlier k (edge order) <- mu[cam] + scale_tril[cam] z[k], written into the
//                      dense pixel matrix (:397-433)
// The random choices between the passes (np.random.choice over nonzero() lists) are the
// reference's numpy draws, made on the host (gasfm_amd/outliers.py).
// Integer work and a few hundred flops per camera: HBM-bound (E bytes of state + E * 16 bytes
// of indices per pass).  Deterministic: the only atomics are integer adds / mins.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kMinViewsPerPoint = 2;   // code/utils/constants.py:2
constexpr int kMinPointsPerView = 8;   // code/utils/constants.py:6

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one wave per camera c: inliers among edges cam_ptr[c] .. cam_ptr[c+1]
__global__ __launch_bounds__(256) void counts_cam_kernel(const uint8_t* __restrict__ state,
                                                         const int* __restrict__ cam_ptr, int m,
                                                         int* __restrict__ cam_in, int* __restrict__ mins) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= m) return;
  const int lane = threadIdx.x & 63;
  const int b = cam_ptr[c], e = cam_ptr[c + 1];
  int k = 0;
  for (int i = b + lane; i < e; i += 64) k += (state[i] & 1) == 0;
  k = wave_sum(k);
  if (lane == 0) {
    cam_in[c] = k;
    atomicMin(mins, k);
  }
}

// one thread per point p: inliers among its CSR slots (perm: slot -> edge; null = identity)
__global__ __launch_bounds__(256) void counts_pt_kernel(const uint8_t* __restrict__ state,
                                                        const int* __restrict__ pt_ptr,
                                                        const int* __restrict__ perm, int n,
                                                        int* __restrict__ pt_in, int* __restrict__ mins) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  int k = INT32_MAX;
  if (p < n) {
    const int b = pt_ptr[p], e = pt_ptr[p + 1];
    k = 0;
    for (int j = b; j < e; ++j) k += (state[perm ? perm[j] : j] & 1) == 0;
    pt_in[p] = k;
  }
  // wave minimum, one atomic per wave
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) k = min(k, __shfl_xor(k, o));
  if ((threadIdx.x & 63) == 0) atomicMin(mins + 1, k);
}

// grid-stride over edges; mode 0 = init, 1 = blacklist; class counts -> counts[0..3]
__global__ __launch_bounds__(256) void mark_kernel(uint8_t* __restrict__ state, const int64_t* __restrict__ cam,
                                                   const int64_t* __restrict__ pt, const int* __restrict__ cam_in,
                                                   const int* __restrict__ pt_in, int64_t E, int mode,
                                                   int* __restrict__ counts) {
  int k0 = 0, k1 = 0, k2 = 0, k3 = 0;
  for (int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x; e < E; e += int64_t(gridDim.x) * 256) {
    int s = state[e];
    if (mode == 0) {
      const bool fixed = pt_in[pt[e]] < kMinViewsPerPoint + 1 || cam_in[cam[e]] < kMinPointsPerView + 1;
      s = fixed ? 0 : 2;
      state[e] = uint8_t(s);
    } else if (s == 3) {
      if (pt_in[pt[e]] < kMinViewsPerPoint || cam_in[cam[e]] < kMinPointsPerView) {
        s = 0;
        state[e] = 0;
      }
    }
    k0 += s == 0;
    k1 += s == 1;
    k2 += s == 2;
    k3 += s == 3;
  }
  k0 = wave_sum(k0);
  k1 = wave_sum(k1);
  k2 = wave_sum(k2);
  k3 = wave_sum(k3);
  if ((threadIdx.x & 63) == 0) {
    if (k0) atomicAdd(counts + 0, k0);
    if (k1) atomicAdd(counts + 1, k1);
    if (k2) atomicAdd(counts + 2, k2);
    if (k3) atomicAdd(counts + 3, k3);
  }
}

// one wave per camera: moments of the inlier pixel values, LDL^T, scale_tril
__global__ __launch_bounds__(256) void moments_kernel(const float* __restrict__ vals, const uint8_t* __restrict__ state,
                                                      const int* __restrict__ cam_ptr, int m, float* __restrict__ mu,
                                                      float* __restrict__ sigma, float* __restrict__ tril,
                                                      int* __restrict__ piv) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= m) return;
  const int lane = threadIdx.x & 63;
  const int b = cam_ptr[c], e = cam_ptr[c + 1];
  double sx = 0, sy = 0, sxx = 0, sxy = 0, syy = 0;
  int k = 0;
  for (int i = b + lane; i < e; i += 64) {
    if (state[i] & 1) continue;
    const float2 v = reinterpret_cast<const float2*>(vals)[i];
    const float x = v.x, y = v.y;
    sx += x;
    sy += y;
    // the reference forms the fp32 outer product x x^T first (sparse_utils.py:145)
    sxx += double(x * x);
    sxy += double(x * y);
    syy += double(y * y);
    ++k;
  }
  sx = wave_sum_d(sx);
  sy = wave_sum_d(sy);
  sxx = wave_sum_d(sxx);
  sxy = wave_sum_d(sxy);
  syy = wave_sum_d(syy);
  k = wave_sum(k);
  if (lane != 0) return;
  // sparse_mean: fp32 sum / fp32 count, Bessel: / (N - 1)  (sparse_utils.py:105-125)
  const float N = float(k);
  mu[2 * c] = float(sx) / N;
  mu[2 * c + 1] = float(sy) / N;
  float a = float(sxx) / (N - 1.f), bb = float(sxy) / (N - 1.f), cc = float(syy) / (N - 1.f);
  sigma[4 * c + 0] = a;
  sigma[4 * c + 1] = bb;
  sigma[4 * c + 2] = bb;
  sigma[4 * c + 3] = cc;
  // LAPACK sytf2, lower, n = 2: alpha = (1 + sqrt(17)) / 8
  const float alpha = 0.6403882032022076f;
  const float colmax = fabsf(bb);
  int p0 = 1, p1 = 2;
  bool swap = false;
  if (!(fabsf(a) >= alpha * colmax)) {
    if (fabsf(cc) >= alpha * colmax) {  // 1x1 pivot after interchanging rows/columns 1 and 2
      p0 = 2;
      swap = true;
      const float t = a;
      a = cc;
      cc = t;
    } else {  // 2x2 pivot block: the reference asserts pivots > 0
      piv[2 * c] = -2;
      piv[2 * c + 1] = -2;
      for (int i = 0; i < 4; ++i) tril[4 * c + i] = __builtin_nanf("");
      return;
    }
  }
  piv[2 * c] = p0;
  piv[2 * c + 1] = p1;
  const float d11 = 1.f / a;
  const float d1 = cc + bb * ((-d11) * bb);  // dsyr: A22 += x * (-d11 * x)
  const float l10 = d11 * bb;                 // dscal
  const float sa = sqrtf(a), sd = sqrtf(d1);
  float t00 = sa, t01 = 0.f, t10 = l10 * sa, t11 = sd;
  if (swap) {  // scale_tril rows flipped (dataset_utils.py:391)
    float u0 = t00, u1 = t01;
    t00 = t10;
    t01 = t11;
    t10 = u0;
    t11 = u1;
  }
  tril[4 * c + 0] = t00;
  tril[4 * c + 1] = t01;
  tril[4 * c + 2] = t10;
  tril[4 * c + 3] = t11;
}

// thread = outlier k: edge idx[k] (ascending edge order), value mu + L z written into M
__global__ __launch_bounds__(256) void apply_kernel(const int64_t* __restrict__ idx, int64_t n_out,
                                                    const int64_t* __restrict__ cam, const int64_t* __restrict__ pt,
                                                    const float* __restrict__ z, const float* __restrict__ mu,
                                                    const float* __restrict__ tril, float* __restrict__ M,
                                                    int64_t ldM, float* __restrict__ pix) {
  const int64_t k = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (k >= n_out) return;
  const int64_t e = idx[k];
  const int64_t c = cam[e], p = pt[e];
  const float z0 = z[2 * k], z1 = z[2 * k + 1];
  const float* L = tril + 4 * c;
  const float x = mu[2 * c] + (L[0] * z0 + L[1] * z1);
  const float y = mu[2 * c + 1] + (L[2] * z0 + L[3] * z1);
  M[2 * c * ldM + p] = x;
  M[(2 * c + 1) * ldM + p] = y;
  if (pix) reinterpret_cast<float2*>(pix)[e] = make_float2(x, y);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_outlier_counts(const uint8_t* state, const int32_t* cam_ptr, const int32_t* pt_ptr,
                                    const int32_t* perm, int32_t m, int32_t n, int32_t* cam_in, int32_t* pt_in,
                                    int32_t* mins, void* stream) {
  GASFM_REQUIRE(m > 0 && n > 0, "gasfm_outlier_counts: m=%d n=%d", m, n);
  GASFM_REQUIRE(state && cam_ptr && pt_ptr && cam_in && pt_in && mins, "gasfm_outlier_counts: null pointer");
  hipStream_t st = (hipStream_t)stream;
  int s = hip_status(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(mins), INT32_MAX, 2, st),
                     "gasfm_outlier_counts");
  if (s) return s;
  hipLaunchKernelGGL(counts_cam_kernel, dim3((m + 3) / 4), dim3(256), 0, st, state, cam_ptr, m, cam_in, mins);
  hipLaunchKernelGGL(counts_pt_kernel, dim3((n + 255) / 256), dim3(256), 0, st, state, pt_ptr, perm, n, pt_in, mins);
  return launch_status("gasfm_outlier_counts");
}

extern "C" int gasfm_outlier_mark(uint8_t* state, const int64_t* cam, const int64_t* pt, const int32_t* cam_in,
                                  const int32_t* pt_in, int64_t E, int32_t mode, int32_t* counts, void* stream) {
  GASFM_REQUIRE(E >= 0 && (mode == 0 || mode == 1), "gasfm_outlier_mark: E=%lld mode=%d", (long long)E, mode);
  GASFM_REQUIRE(counts && (E == 0 || (state && cam && pt && cam_in && pt_in)), "gasfm_outlier_mark: null pointer");
  hipStream_t st = (hipStream_t)stream;
  int s = hip_status(hipMemsetAsync(counts, 0, 4 * sizeof(int32_t), st), "gasfm_outlier_mark");
  if (s || E == 0) return s;
  const int grid = resident_grid(reinterpret_cast<const void*>(mark_kernel), 256, 0, E, 256 * 8);
  hipLaunchKernelGGL(mark_kernel, dim3(grid), dim3(256), 0, st, state, cam, pt, cam_in, pt_in, E, mode, counts);
  return launch_status("gasfm_outlier_mark");
}

extern "C" int gasfm_outlier_moments(const float* values, const uint8_t* state, const int32_t* cam_ptr, int32_t m,
                                     float* mu, float* sigma, float* scale_tril, int32_t* pivots, void* stream) {
  GASFM_REQUIRE(m > 0, "gasfm_outlier_moments: m=%d", m);
  GASFM_REQUIRE(values && state && cam_ptr && mu && sigma && scale_tril && pivots,
                "gasfm_outlier_moments: null pointer");
  GASFM_REQUIRE((reinterpret_cast<uintptr_t>(values) & 7u) == 0, "gasfm_outlier_moments: values not 8-byte aligned");
  hipLaunchKernelGGL(moments_kernel, dim3((m + 3) / 4), dim3(256), 0, (hipStream_t)stream, values, state, cam_ptr, m,
                     mu, sigma, scale_tril, pivots);
  return launch_status("gasfm_outlier_moments");
}

extern "C" int gasfm_outlier_apply(const int64_t* idx, int64_t n_out, const int64_t* cam, const int64_t* pt,
                                   const float* z, const float* mu, const float* scale_tril, float* M, int64_t ldM,
                                   float* pix, void* stream) {
  GASFM_REQUIRE(n_out >= 0 && ldM > 0, "gasfm_outlier_apply: n_out=%lld", (long long)n_out);
  if (n_out == 0) return GASFM_OK;
  GASFM_REQUIRE(idx && cam && pt && z && mu && scale_tril && M, "gasfm_outlier_apply: null pointer");
  GASFM_REQUIRE(pix == nullptr || (reinterpret_cast<uintptr_t>(pix) & 7u) == 0,
                "gasfm_outlier_apply: pix not 8-byte aligned");
  hipLaunchKernelGGL(apply_kernel, dim3(unsigned((n_out + 255) / 256)), dim3(256), 0, (hipStream_t)stream, idx, n_out,
                     cam, pt, z, mu, scale_tril, M, ldM, pix);
  return launch_status("gasfm_outlier_apply");
}
