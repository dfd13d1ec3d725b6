// Adam over every parameter tensor of the model in ONE launch, gfx950.
//
// train.py (:97-100) steps torch.optim.Adam after every batch.  torch's fused multi-tensor Adam
// walks the ~880 parameter tensors (145 M values) in ~34 launches of 3-4 us set-up each and reaches
// ~2.9 TB/s (1.39 ms per step, profiles/r5_train_step_breakdown*.txt).  Here a host-built table of
// 4096-value chunks (tensor index, first value) drives one grid: each workgroup updates one chunk of
// one tensor with float4 loads / stores (a scalar tail for sizes that are not multiples of 4),
// reading p, g, m, v and writing p, m, v once: 28 bytes per parameter.
//
// Update (torch.optim.Adam, amsgrad = False, maximize = False; torch/optim/adam.py):
//   g' = g + wd p;  m = m + (1 - b1)(g' - m);  v = b2 v + (1 - b2) g'^2
//   p = p - (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr int kT = 256;

struct AdamK {
  float b1, b2, c1, c2, eps, wd, step_size, inv_bc2_sqrt;  // c1 / c2 = 1 - beta1 / 1 - beta2 (rounded from fp64)
};

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, const AdamK& k) {
  if (k.wd != 0.f) g = fmaf(k.wd, p, g);
  m = fmaf(k.c1, g - m, m);
  v = fmaf(k.b2, v, k.c2 * g * g);
  const float denom = sqrtf(v) * k.inv_bc2_sqrt + k.eps;
  p = p - k.step_size * (m / denom);
}

__global__ __launch_bounds__(kT) void adam_kernel(const gasfm_adam_tensor* __restrict__ tensors,
                                                  const gasfm_adam_chunk* __restrict__ chunks, AdamK k) {
  const gasfm_adam_chunk ch = chunks[blockIdx.x];
  const gasfm_adam_tensor t = tensors[ch.tensor];
  const int64_t end = ch.begin + GASFM_ADAM_CHUNK < t.numel ? ch.begin + GASFM_ADAM_CHUNK : t.numel;
  const bool vec = ((reinterpret_cast<uintptr_t>(t.p) | reinterpret_cast<uintptr_t>(t.g) |
                     reinterpret_cast<uintptr_t>(t.m) | reinterpret_cast<uintptr_t>(t.v)) & 15) == 0;
  if (vec) {
    const int64_t n4 = (end - ch.begin) / 4;
    for (int64_t q = threadIdx.x; q < n4; q += kT) {
      const int64_t i = ch.begin + 4 * q;
      float4 p = *reinterpret_cast<const float4*>(t.p + i);
      const float4 g = *reinterpret_cast<const float4*>(t.g + i);
      float4 m = *reinterpret_cast<const float4*>(t.m + i);
      float4 v = *reinterpret_cast<const float4*>(t.v + i);
      adam1(p.x, g.x, m.x, v.x, k);
      adam1(p.y, g.y, m.y, v.y, k);
      adam1(p.z, g.z, m.z, v.z, k);
      adam1(p.w, g.w, m.w, v.w, k);
      *reinterpret_cast<float4*>(t.p + i) = p;
      *reinterpret_cast<float4*>(t.m + i) = m;
      *reinterpret_cast<float4*>(t.v + i) = v;
    }
    for (int64_t i = ch.begin + 4 * n4 + threadIdx.x; i < end; i += kT) adam1(t.p[i], t.g[i], t.m[i], t.v[i], k);
  } else {
    for (int64_t i = ch.begin + threadIdx.x; i < end; i += kT) adam1(t.p[i], t.g[i], t.m[i], t.v[i], k);
  }
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_adam_step(const gasfm_adam_tensor* tensors, const gasfm_adam_chunk* chunks, int32_t n_chunks,
                               double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                               void* stream) {
  GASFM_REQUIRE(tensors && chunks && n_chunks > 0 && step > 0, "gasfm_adam_step: n_chunks=%d step=%lld", n_chunks,
                (long long)step);
  GASFM_REQUIRE(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0,
                "gasfm_adam_step: betas (%g, %g), eps %g", beta1, beta2, eps);
  // the hyper-parameters arrive as fp64 (torch's python floats): 1 - beta, the bias corrections
  // and the step size in fp64, then rounded (1.f - 0.999f would be 1.3e-5 off)
  const double bc1 = 1.0 - __builtin_pow(beta1, double(step));
  const double bc2 = 1.0 - __builtin_pow(beta2, double(step));
  AdamK k{float(beta1), float(beta2), float(1.0 - beta1), float(1.0 - beta2), float(eps), float(weight_decay),
          float(lr / bc1), float(1.0 / __builtin_sqrt(bc2))};
  hipLaunchKernelGGL(adam_kernel, dim3(n_chunks), dim3(kT), 0, reinterpret_cast<hipStream_t>(stream), tensors, chunks,
                     k);
  return launch_status("gasfm_adam_step");
}
