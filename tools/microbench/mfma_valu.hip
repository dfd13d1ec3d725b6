// Does VALU work overlap v_mfma_f32_16x16x4_f32 on gfx950?  Times (1) waves issuing only
// independent fp32 MFMAs, (2) waves issuing only independent VALU FMAs, (3) one MFMA wave and one
// VALU wave per SIMD, (4) one wave interleaving both.  If (3) ~ max(1, 2) the SIMD co-executes
// the two; if (3) ~ (1) + (2) the fp32 MFMA holds the vector issue.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_valu tools/microbench/mfma_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 4096;

__device__ __forceinline__ void mfma_work(f32x4 (&acc)[8], float a, float b) {
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b + k, acc[k], 0, 0, 0);
}

// the same MFMA cycles with 32x32x2 f32 (64 cycles each: 4 per iteration) or 16x16x32 bf16 (8 x 4)
__device__ __forceinline__ void mfma32_work(f32x16 (&acc)[2], float a, float b) {
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b + k, acc[k & 1], 0, 0, 0);
}
__device__ __forceinline__ void mfmabf_work(f32x4 (&acc)[8], bf16x8 a, bf16x8 b) {
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
}

__device__ __forceinline__ void valu_work(float (&v)[16], float a) {
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = fmaf(v[k], a, 1.0f);
}

// mode 0: every wave MFMA; 1: every wave VALU; 2: even waves MFMA, odd VALU (waves 2i, 2i+1 of a
// 8-wave block land on SIMDs i%4 -- checked by the timings); 3: every wave both, interleaved;
// 4: half the waves MFMA, the rest idle (one MFMA wave per SIMD); 5: half VALU, rest idle;
// KIND 0: 16x16x4 f32, 1: 32x32x2 f32, 2: 16x16x32 bf16 (8 per iteration: 1/4 of the cycles)
template <int MODE, int KIND>
__global__ __launch_bounds__(512) void bench(float* out, float a, float b) {
  const int wave = threadIdx.x / 64;
  f32x4 acc[8];
  f32x16 acc32[2];
  float v[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc32[k][r] = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = threadIdx.x * 1e-3f + k;
  bf16x8 ab, bb;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ab[k] = (__bf16)(a + k);
    bb[k] = (__bf16)(b - k);
  }
  const bool do_mfma = MODE == 0 || MODE == 3 || ((MODE == 2 || MODE == 4) && wave < 4);
  const bool do_valu = MODE == 1 || MODE == 3 || ((MODE == 2 || MODE == 5) && wave >= 4);
  auto mf = [&]() {
    if (KIND == 0) mfma_work(acc, a, b);
    else if (KIND == 1) mfma32_work(acc32, a, b);
    else mfmabf_work(acc, ab, bb);
  };
  if (do_mfma && do_valu) {
    for (int i = 0; i < kIters; ++i) {
      mf();
      valu_work(v, a);
      valu_work(v, b);
    }
  } else if (do_mfma) {
    for (int i = 0; i < kIters; ++i) mf();
  } else if (do_valu) {
    for (int i = 0; i < kIters; ++i) {
      valu_work(v, a);
      valu_work(v, b);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
#pragma unroll
  for (int k = 0; k < 2; ++k) s += acc32[k][0] + acc32[k][15];
#pragma unroll
  for (int k = 0; k < 16; ++k) s += v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int KIND>
float run(float* out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  bench<MODE, KIND><<<blocks, 512>>>(out, 1.0001f, 0.5f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) bench<MODE, KIND><<<blocks, 512>>>(out, 1.0001f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int blocks = prop.multiProcessorCount;  // one 8-wave block per CU: 2 waves per SIMD
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * 512);
  const double clk = prop.clockRate * 1e3;  // Hz
  const char* names[] = {"all MFMA (2/SIMD)", "all VALU (2/SIMD)", "MFMA wave + VALU wave per SIMD",
                         "each wave both, interleaved", "MFMA only (1/SIMD)", "VALU only (1/SIMD)"};
  const char* kinds[] = {"16x16x4 f32 (8/iter)", "32x32x2 f32 (4/iter)", "16x16x32 bf16 (8/iter)"};
  auto table = [&](auto k0, auto k1, auto k2, auto k3, auto k4, auto k5, int kind) {
    float t[6] = {k0(out, blocks), k1(out, blocks), k2(out, blocks), k3(out, blocks), k4(out, blocks), k5(out, blocks)};
    printf("MFMA %s\n", kinds[kind]);
    for (int m = 0; m < 6; ++m)
      printf("  %-34s %8.3f ms  %8.1f cycles/iter/SIMD\n", names[m], t[m], t[m] * 1e-3 * clk / kIters);
  };
  table(run<0, 0>, run<1, 0>, run<2, 0>, run<3, 0>, run<4, 0>, run<5, 0>, 0);
  table(run<0, 1>, run<1, 1>, run<2, 1>, run<3, 1>, run<4, 1>, run<5, 1>, 1);
  table(run<0, 2>, run<1, 2>, run<2, 2>, run<3, 2>, run<4, 2>, run<5, 2>, 2);
  hipFree(out);
  return 0;
}
