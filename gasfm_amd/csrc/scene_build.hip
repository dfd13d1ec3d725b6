// Device-side scene graph builder, gfx950: dense measurement matrix -> edge list + CSR/CSC.
//
// Replaces, for a measurement matrix M that is already in HBM, the reference's CPU path
//   get_M_valid_points  (code/utils/dataset_utils.py:86-113)   validity mask, >= 2 views per point
//   M2sparse            (dataset_utils.py:116-156)             cam-major nonzero() edge order
//   normalize_M         (code/utils/geo_utils.py:689-703)      values = (N_c [x, y, 1]^T)[:2]
// and the point-direction grouping that PyG's scatter did implicitly (gasfm_build_csr on the
// host: a stable counting sort of the edges by point, dataset_utils.py:531-535).
//
// Integer / byte work, HBM-bound; no float arithmetic except the 2x3 normalisation.
//   scene_mask       M [2m x n] read once (coalesced along n): one validity BIT per (camera,
//                    point) via wave ballot -> mask [m x W] uint64 (W = ceil(n/64)), plus exact
//                    per-point view counts (integer atomics, one per workgroup and point).
//   scene_ptvalid    per-point validity (count >= MIN_N_VIEWS_PER_POINT) as bits + final counts.
//   scene_tilecount  popcount of (mask & valid) per tile of 64 words of one camera row.
//   scan_i32         exclusive scan (one workgroup; tile counts, then per-point counts).
//   scene_emit       one wave per tile: word prefix by wave scan, then every set bit becomes
//                    edge e = tile base + rank: cam[e], pt[e], values[e] (row-major nonzero()
//                    order == the reference's edge order), and word_base (first edge of a word).
//   scene_point_csr  one wave per 64-point word column walks the cameras in order: the k-th
//                    camera of point p gets slot pt_ptr[p] + k, i.e. the STABLE counting sort
//                    of gasfm_build_csr, written as perm (slot -> edge) and pos (edge -> slot).
// Everything is deterministic: the only atomics are integer adds.
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kMinViewsPerPoint = 2;  // code/utils/constants.py:2
constexpr int kMaskCams = 32;         // cameras per scene_mask workgroup row
constexpr int kScanThreads = 1024;

__device__ __forceinline__ bool nonzero_bits(float v) { return (__float_as_uint(v) & 0x7fffffffu) != 0u; }

// grid (ceil(n/256), ceil(m/kMaskCams)), 256 threads: thread = point, loop over cameras.
__global__ __launch_bounds__(256) void scene_mask_kernel(const float* __restrict__ M, int64_t ldM, int m, int n,
                                                         int64_t W, unsigned long long* __restrict__ mask,
                                                         int* __restrict__ count) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int c0 = blockIdx.y * kMaskCams;
  const int c1 = min(c0 + kMaskCams, m);
  const bool live = p < n;
  const int pp = live ? p : 0;
  const int lane = threadIdx.x & 63;
  int cnt = 0;
  for (int cb = c0; cb < c1; cb += 8) {
    float x[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // all loads of the group issued before any is used
      const int c = min(cb + u, c1 - 1);
      x[u] = M[int64_t(2 * c) * ldM + pp];
      y[u] = M[int64_t(2 * c + 1) * ldM + pp];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = cb + u;
      if (c >= c1) break;
      // |x| + |y| != 0 (dataset_utils.py:97), exactly: a value is zero iff its bits are +-0
      const bool v = live && (nonzero_bits(x[u]) || nonzero_bits(y[u]));
      const unsigned long long b = __ballot(v);
      cnt += v;
      if (lane == 0 && (p >> 6) < W) mask[int64_t(c) * W + (p >> 6)] = b;
    }
  }
  if (live && cnt) atomicAdd(count + p, cnt);
}

// thread = point: validity bits (>= 2 views) and the filtered count (0 for invalid points)
__global__ __launch_bounds__(256) void scene_ptvalid_kernel(const int* __restrict__ count, int n,
                                                            unsigned long long* __restrict__ valid,
                                                            int* __restrict__ vcount) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int c = p < n ? count[p] : 0;
  const bool v = p < n && c >= kMinViewsPerPoint;
  const unsigned long long b = __ballot(v);
  if ((threadIdx.x & 63) == 0 && (p >> 6) < (n + 63) / 64) valid[p >> 6] = b;
  if (p < n) vcount[p] = v ? c : 0;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// inclusive scan over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// one wave per tile (c, t): words 64t .. 64t+63 of camera row c
__global__ __launch_bounds__(256) void scene_tilecount_kernel(const unsigned long long* __restrict__ mask,
                                                              const unsigned long long* __restrict__ valid,
                                                              int64_t W, int64_t T, int64_t ntiles,
                                                              int* __restrict__ tcount) {
  const int64_t tile = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (tile >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const int64_t c = tile / T, w = (tile % T) * 64 + lane;
  const int k = w < W ? __popcll(mask[c * W + w] & valid[w]) : 0;
  const int s = wave_sum_i(k);
  if (lane == 0) tcount[tile] = s;
}

// exclusive scan of in[0..L) into out[0..L], out[L] = total; one workgroup.  Thread i owns a
// contiguous chunk; chunk sums are scanned in LDS.
__global__ __launch_bounds__(kScanThreads) void scan_i32_kernel(const int* __restrict__ in, int64_t L,
                                                                int* __restrict__ out) {
  __shared__ int64_t sums[kScanThreads];
  const int t = threadIdx.x;
  const int64_t per = (L + kScanThreads - 1) / kScanThreads;
  const int64_t b = t * per, e = min(L, b + per);
  int64_t s = 0;
  for (int64_t i = b; i < e; ++i) s += in[i];
  sums[t] = s;
  __syncthreads();
  for (int o = 1; o < kScanThreads; o <<= 1) {  // Hillis-Steele over the chunk sums
    const int64_t v = t >= o ? sums[t - o] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int64_t run = sums[t] - s;
  for (int64_t i = b; i < e; ++i) {
    out[i] = int(run);
    run += in[i];
  }
  if (t == kScanThreads - 1) out[L] = int(sums[t]);
}

// one wave per tile: word prefix, then edges in row-major order
__global__ __launch_bounds__(256) void scene_emit_kernel(
    const float* __restrict__ M, int64_t ldM, const float* __restrict__ Ns, const unsigned long long* __restrict__ mask,
    const unsigned long long* __restrict__ valid, const int* __restrict__ tbase, int64_t W, int64_t T, int64_t ntiles,
    int64_t* __restrict__ cam, int64_t* __restrict__ pt, float* __restrict__ vals, int* __restrict__ word_base) {
  const int64_t tile = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (tile >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const int64_t c = tile / T, w = (tile % T) * 64 + lane;
  unsigned long long bits = w < W ? (mask[c * W + w] & valid[w]) : 0ull;
  const int k = __popcll(bits);
  int e = tbase[tile] + wave_incl_scan(k, lane) - k;
  if (w < W) word_base[c * W + w] = e;
  float n00 = 1.f, n01 = 0.f, n02 = 0.f, n10 = 0.f, n11 = 1.f, n12 = 0.f;
  if (Ns) {  // K^-1 of camera c (rows 0, 1 of the 3x3)
    const float* N = Ns + c * 9;
    n00 = N[0];
    n01 = N[1];
    n02 = N[2];
    n10 = N[3];
    n11 = N[4];
    n12 = N[5];
  }
  const float* Mx = M + 2 * c * ldM;
  const float* My = Mx + ldM;
  while (bits) {
    const int j = __builtin_ctzll(bits);
    bits &= bits - 1;
    const int64_t p = w * 64 + j;
    const float x = Mx[p], y = My[p];
    cam[e] = c;
    pt[e] = p;
    float2 v = make_float2(x, y);
    if (Ns) v = make_float2(n00 * x + n01 * y + n02, n10 * x + n11 * y + n12);
    reinterpret_cast<float2*>(vals)[e] = v;
    ++e;
  }
}

// one wave per word column w: lane = point 64w + lane; cameras in ascending order
__global__ __launch_bounds__(256) void scene_point_csr_kernel(const unsigned long long* __restrict__ mask,
                                                              const unsigned long long* __restrict__ valid,
                                                              const int* __restrict__ word_base,
                                                              const int* __restrict__ pt_ptr, int m, int n,
                                                              int64_t W, int* __restrict__ perm,
                                                              int* __restrict__ pos) {
  const int64_t w = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (w >= W) return;
  const int lane = threadIdx.x & 63;
  const int64_t p = w * 64 + lane;
  const unsigned long long vw = valid[w];
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int slot = p < n ? pt_ptr[p] : 0;
  for (int cb = 0; cb < m; cb += 8) {
    unsigned long long mw[8];
    int wb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = min(cb + u, m - 1);
      mw[u] = mask[int64_t(c) * W + w] & vw;
      wb[u] = word_base[int64_t(c) * W + w];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (cb + u >= m) break;
      if ((mw[u] >> lane) & 1ull) {
        const int e = wb[u] + __popcll(mw[u] & below);
        perm[slot] = e;
        pos[e] = slot;
        ++slot;
      }
    }
  }
}


// rotational homography augmentation of the image points (SceneData.apply_rotational_homography_aug,
// datasets/SceneData.py:355-440): grid (ceil(n/256), m), thread = (camera c, point p).
//   valid (c, p) (mask bit and >= 2 views): (x', y') = pflat(Ninv_c R_c Ns_c [x, y, 1]^T)
//   otherwise 0 (the reference's explicit zero-reset of ~valid_pts)
__global__ __launch_bounds__(256) void scene_homography_kernel(const float* __restrict__ M, int64_t ldM, int n,
                                                               int64_t W, const unsigned long long* __restrict__ mask,
                                                               const unsigned long long* __restrict__ valid,
                                                               const float* __restrict__ Ns, const float* __restrict__ R,
                                                               const float* __restrict__ Ninv, float* __restrict__ out,
                                                               int64_t ldO) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (p >= n) return;
  const int w = p >> 6, b = p & 63;
  const bool v = ((mask[c * W + w] >> b) & 1ull) && ((valid[w] >> b) & 1ull);
  float ox = 0.f, oy = 0.f;
  if (v) {
    const float x = M[2 * c * ldM + p], y = M[(2 * c + 1) * ldM + p];
    const float* N = Ns + c * 9;
    const float* Rc = R + c * 9;
    const float* Ni = Ninv + c * 9;
    float a[3], q[3], d[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) a[i] = N[3 * i] * x + N[3 * i + 1] * y + N[3 * i + 2];
#pragma unroll
    for (int i = 0; i < 3; ++i) q[i] = Rc[3 * i] * a[0] + Rc[3 * i + 1] * a[1] + Rc[3 * i + 2] * a[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = Ni[3 * i] * q[0] + Ni[3 * i + 1] * q[1] + Ni[3 * i + 2] * q[2];
    ox = d[0] / d[2];
    oy = d[1] / d[2];
  }
  out[2 * c * ldO + p] = ox;
  out[(2 * c + 1) * ldO + p] = oy;
}
}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int64_t gasfm_scene_mask_words(int32_t n) { return n <= 0 ? 0 : (int64_t(n) + 63) / 64; }

extern "C" int64_t gasfm_scene_tiles(int32_t m, int32_t n) {
  const int64_t W = gasfm_scene_mask_words(n);
  return int64_t(m < 0 ? 0 : m) * ((W + 63) / 64);
}

extern "C" int gasfm_scan_i32(const int32_t* in, int64_t L, int32_t* out, void* stream) {
  GASFM_REQUIRE(L >= 0 && out && (L == 0 || in), "gasfm_scan_i32: bad args");
  hipLaunchKernelGGL(scan_i32_kernel, dim3(1), dim3(kScanThreads), 0, (hipStream_t)stream, in, L, out);
  return launch_status("gasfm_scan_i32");
}

extern "C" int gasfm_scene_mask(const float* M, int64_t ldM, int32_t m, int32_t n, uint64_t* mask,
                                int32_t* view_count, uint64_t* pt_valid, int32_t* pt_count, int32_t* tile_count,
                                int32_t* tile_base, void* stream) {
  GASFM_REQUIRE(m > 0 && n > 0 && ldM >= n, "gasfm_scene_mask: m=%d n=%d ldM=%lld", m, n, (long long)ldM);
  GASFM_REQUIRE(int64_t(m) * n < INT32_MAX, "gasfm_scene_mask: m*n=%lld exceeds int32 edge ids",
                (long long)(int64_t(m) * n));
  GASFM_REQUIRE(M && mask && view_count && pt_valid && pt_count && tile_count && tile_base,
                "gasfm_scene_mask: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int64_t W = gasfm_scene_mask_words(n), T = (W + 63) / 64, ntiles = int64_t(m) * T;
  int s = hip_status(hipMemsetAsync(view_count, 0, sizeof(int32_t) * size_t(n), st), "gasfm_scene_mask");
  if (s) return s;
  hipLaunchKernelGGL(scene_mask_kernel, dim3((n + 255) / 256, (m + kMaskCams - 1) / kMaskCams), dim3(256), 0, st, M,
                     ldM, m, n, W, reinterpret_cast<unsigned long long*>(mask), view_count);
  hipLaunchKernelGGL(scene_ptvalid_kernel, dim3((n + 255) / 256), dim3(256), 0, st, view_count, n,
                     reinterpret_cast<unsigned long long*>(pt_valid), pt_count);
  hipLaunchKernelGGL(scene_tilecount_kernel, dim3(unsigned((ntiles + 3) / 4)), dim3(256), 0, st,
                     reinterpret_cast<const unsigned long long*>(mask),
                     reinterpret_cast<const unsigned long long*>(pt_valid), W, T, ntiles, tile_count);
  hipLaunchKernelGGL(scan_i32_kernel, dim3(1), dim3(kScanThreads), 0, st, tile_count, ntiles, tile_base);
  return launch_status("gasfm_scene_mask");
}

extern "C" int gasfm_scene_emit(const float* M, int64_t ldM, const float* Ns, int32_t m, int32_t n,
                                const uint64_t* mask, const uint64_t* pt_valid, const int32_t* tile_base,
                                int64_t* cam, int64_t* pt, float* values, int32_t* word_base, void* stream) {
  GASFM_REQUIRE(m > 0 && n > 0 && ldM >= n, "gasfm_scene_emit: m=%d n=%d", m, n);
  GASFM_REQUIRE(M && mask && pt_valid && tile_base && cam && pt && values && word_base,
                "gasfm_scene_emit: null pointer");
  GASFM_REQUIRE((reinterpret_cast<uintptr_t>(values) & 7u) == 0, "gasfm_scene_emit: values not 8-byte aligned");
  const int64_t W = gasfm_scene_mask_words(n), T = (W + 63) / 64, ntiles = int64_t(m) * T;
  hipLaunchKernelGGL(scene_emit_kernel, dim3(unsigned((ntiles + 3) / 4)), dim3(256), 0, (hipStream_t)stream, M, ldM,
                     Ns, reinterpret_cast<const unsigned long long*>(mask),
                     reinterpret_cast<const unsigned long long*>(pt_valid), tile_base, W, T, ntiles, cam, pt, values,
                     word_base);
  return launch_status("gasfm_scene_emit");
}

extern "C" int gasfm_scene_point_csr(const uint64_t* mask, const uint64_t* pt_valid, const int32_t* word_base,
                                     const int32_t* pt_ptr, int32_t m, int32_t n, int32_t* perm, int32_t* pos,
                                     void* stream) {
  GASFM_REQUIRE(m > 0 && n > 0, "gasfm_scene_point_csr: m=%d n=%d", m, n);
  GASFM_REQUIRE(mask && pt_valid && word_base && pt_ptr && perm && pos, "gasfm_scene_point_csr: null pointer");
  const int64_t W = gasfm_scene_mask_words(n);
  hipLaunchKernelGGL(scene_point_csr_kernel, dim3(unsigned((W + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const unsigned long long*>(mask),
                     reinterpret_cast<const unsigned long long*>(pt_valid), word_base, pt_ptr, m, n, W, perm, pos);
  return launch_status("gasfm_scene_point_csr");
}

extern "C" int gasfm_scene_homography(const float* M, int64_t ldM, int32_t m, int32_t n, const uint64_t* mask,
                                      const uint64_t* pt_valid, const float* Ns, const float* R, const float* Ninv,
                                      float* out, int64_t ldO, void* stream) {
  GASFM_REQUIRE(m > 0 && n > 0 && ldM >= n && ldO >= n, "gasfm_scene_homography: m=%d n=%d", m, n);
  GASFM_REQUIRE(M && mask && pt_valid && Ns && R && Ninv && out, "gasfm_scene_homography: null pointer");
  GASFM_REQUIRE(m <= 65535, "gasfm_scene_homography: m=%d exceeds the grid's y extent", m);
  hipLaunchKernelGGL(scene_homography_kernel, dim3((n + 255) / 256, m), dim3(256), 0, (hipStream_t)stream, M, ldM, n,
                     gasfm_scene_mask_words(n), reinterpret_cast<const unsigned long long*>(mask),
                     reinterpret_cast<const unsigned long long*>(pt_valid), Ns, R, Ninv, out, ldO);
  return launch_status("gasfm_scene_homography");
}
