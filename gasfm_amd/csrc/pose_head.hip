// Calibrated camera head: x [m x 7] = (quaternion r,i,j,k | translation) -> P = [R(q) | t] [m x 3 x 4].
//
// Replaces baseNet.extract_view_outputs for rot_representation 'quat' (code/models/baseNet.py:38-56:
// pytorch3d quaternion_to_matrix, real part first, then torch.cat with the translation), which
// aten runs as ~40 elementwise kernels forward and ~80 backward on [m] vectors.  One thread per
// camera each way.
//   R = I + s M(q),  s = 2 / |q|^2,
//   M = [[-(j2+k2), ij-kr, ik+jr], [ij+kr, -(i2+k2), jk-ir], [ik-jr, jk+ir, -(i2+j2)]]
// Backward: with G = s dR, dq = dM(q)^T G - s^2 q (dR : M).
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace gasfm {
namespace {

__global__ __launch_bounds__(256) void pose_fwd_kernel(const float* __restrict__ x, int64_t ldx, int64_t m,
                                                       float* __restrict__ P) {
  const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= m) return;
  const float* q = x + c * ldx;
  const float r = q[0], i = q[1], j = q[2], k = q[3];
  const float s = 2.f / (r * r + i * i + j * j + k * k);
  float* o = P + c * 12;
  o[0] = 1.f - s * (j * j + k * k);
  o[1] = s * (i * j - k * r);
  o[2] = s * (i * k + j * r);
  o[3] = q[4];
  o[4] = s * (i * j + k * r);
  o[5] = 1.f - s * (i * i + k * k);
  o[6] = s * (j * k - i * r);
  o[7] = q[5];
  o[8] = s * (i * k - j * r);
  o[9] = s * (j * k + i * r);
  o[10] = 1.f - s * (i * i + j * j);
  o[11] = q[6];
}

__global__ __launch_bounds__(256) void pose_bwd_kernel(const float* __restrict__ x, int64_t ldx, int64_t m,
                                                       const float* __restrict__ dP, float* __restrict__ dx,
                                                       int64_t lddx) {
  const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= m) return;
  const float* q = x + c * ldx;
  const float r = q[0], i = q[1], j = q[2], k = q[3];
  const float s = 2.f / (r * r + i * i + j * j + k * k);
  const float* g = dP + c * 12;
  const float d00 = g[0], d01 = g[1], d02 = g[2], d10 = g[4], d11 = g[5], d12 = g[6], d20 = g[8], d21 = g[9],
              d22 = g[10];
  // dL/ds = dR : M
  const float ds = d00 * -(j * j + k * k) + d01 * (i * j - k * r) + d02 * (i * k + j * r) + d10 * (i * j + k * r) +
                   d11 * -(i * i + k * k) + d12 * (j * k - i * r) + d20 * (i * k - j * r) + d21 * (j * k + i * r) +
                   d22 * -(i * i + j * j);
  const float G00 = s * d00, G01 = s * d01, G02 = s * d02, G10 = s * d10, G11 = s * d11, G12 = s * d12,
              G20 = s * d20, G21 = s * d21, G22 = s * d22;
  const float ss = -s * s * ds;  // dL/ds * ds/dq_x = -s^2 q_x dL/ds
  float* o = dx + c * lddx;
  o[0] = -k * G01 + j * G02 + k * G10 - i * G12 - j * G20 + i * G21 + ss * r;
  o[1] = j * G01 + k * G02 + j * G10 - 2.f * i * G11 - r * G12 + k * G20 + r * G21 - 2.f * i * G22 + ss * i;
  o[2] = -2.f * j * G00 + i * G01 + r * G02 + i * G10 + k * G12 - r * G20 + k * G21 - 2.f * j * G22 + ss * j;
  o[3] = -2.f * k * G00 - r * G01 + i * G02 + r * G10 - 2.f * k * G11 + j * G12 + i * G20 + j * G21 + ss * k;
  o[4] = g[3];
  o[5] = g[7];
  o[6] = g[11];
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_pose_fwd(const float* x, int64_t ldx, int64_t m, float* P, void* stream) {
  GASFM_REQUIRE(m >= 0 && ldx >= 7, "gasfm_pose_fwd: m=%lld ldx=%lld", (long long)m, (long long)ldx);
  if (m == 0) return GASFM_OK;
  GASFM_REQUIRE(x && P, "gasfm_pose_fwd: null pointer");
  hipLaunchKernelGGL(pose_fwd_kernel, dim3(unsigned((m + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, ldx, m, P);
  return launch_status("gasfm_pose_fwd");
}

extern "C" int gasfm_pose_bwd(const float* x, int64_t ldx, int64_t m, const float* dP, float* dx, int64_t lddx,
                              void* stream) {
  GASFM_REQUIRE(m >= 0 && ldx >= 7 && lddx >= 7, "gasfm_pose_bwd: m=%lld", (long long)m);
  if (m == 0) return GASFM_OK;
  GASFM_REQUIRE(x && dP && dx, "gasfm_pose_bwd: null pointer");
  hipLaunchKernelGGL(pose_bwd_kernel, dim3(unsigned((m + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, ldx, m, dP, dx, lddx);
  return launch_status("gasfm_pose_bwd");
}
