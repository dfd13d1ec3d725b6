// Does VALU work overlap v_mfma_f32_16x16x4_f32 on gfx950?  Times (1) waves issuing only
// independent fp32 MFMAs, (2) waves issuing only independent VALU FMAs, (3) one MFMA wave and one
// VALU wave per SIMD, (4) one wave interleaving both.  If (3) ~ max(1, 2) the SIMD co-executes
// the two; if (3) ~ (1) + (2) the fp32 MFMA holds the vector issue.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_valu tools/microbench/mfma_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

__device__ __forceinline__ void mfma_work(f32x4 (&acc)[8], float a, float b) {
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b + k, acc[k], 0, 0, 0);
}

__device__ __forceinline__ void valu_work(float (&v)[16], float a) {
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = fmaf(v[k], a, 1.0f);
}

// mode 0: every wave MFMA; 1: every wave VALU; 2: even waves MFMA, odd VALU (waves 2i, 2i+1 of a
// 8-wave block land on SIMDs i%4 -- checked by the timings); 3: every wave both, interleaved;
// 4: half the waves MFMA, the rest idle (one MFMA wave per SIMD); 5: half VALU, rest idle
template <int MODE>
__global__ __launch_bounds__(512) void bench(float* out, float a, float b) {
  const int wave = threadIdx.x / 64;
  f32x4 acc[8];
  float v[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = threadIdx.x * 1e-3f + k;
  const bool do_mfma = MODE == 0 || MODE == 3 || ((MODE == 2 || MODE == 4) && wave < 4);
  const bool do_valu = MODE == 1 || MODE == 3 || ((MODE == 2 || MODE == 5) && wave >= 4);
  if (do_mfma && do_valu) {
    for (int i = 0; i < kIters; ++i) {
      mfma_work(acc, a, b);
      valu_work(v, a);
      valu_work(v, b);
    }
  } else if (do_mfma) {
    for (int i = 0; i < kIters; ++i) mfma_work(acc, a, b);
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
  for (int k = 0; k < 16; ++k) s += v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
float run(float* out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  bench<MODE><<<blocks, 512>>>(out, 1.0001f, 0.5f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) bench<MODE><<<blocks, 512>>>(out, 1.0001f, 0.5f);
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
  float t[6] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks),
                run<3>(out, blocks), run<4>(out, blocks), run<5>(out, blocks)};
  // per SIMD per iteration: mode 0: 2 waves x 8 MFMA; mode 1: 2 x 32 VALU; mode 4: 8 MFMA; mode 5: 32 VALU
  for (int m = 0; m < 6; ++m)
    printf("%-34s %8.3f ms  %8.1f cycles/iter/SIMD\n", names[m], t[m], t[m] * 1e-3 * clk / kIters);
  hipFree(out);
  return 0;
}
