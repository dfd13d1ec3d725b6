// Per-kernel cost of short dependent kernels inside a replayed hipGraph (the node-side chains of a
// sharded step are hundreds of such kernels).  Build: hipcc --offload-arch=gfx950 -O3 -o
// gpurun_out/launch_floor tools/launch_floor.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));           \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_empty() {}
__global__ void k_copy(const float* x, float* y) { y[threadIdx.x] = x[threadIdx.x] + 1.f; }
__global__ void k_chain2(const int* ptr, const float* x, float* y) {
  y[threadIdx.x] = x[ptr[threadIdx.x]] + 1.f;
}
__global__ void k_chain3(const int* ptr, const float* x, float* y) {
  y[threadIdx.x] = x[ptr[ptr[threadIdx.x]]] + 1.f;
}
__global__ void k_wide(const float* x, float* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  y[i] = x[i] + 1.f;
}

template <class F>
float time_graph(hipStream_t st, int n, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; ++i) launch(i);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 3; ++w) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int reps = 20;
  hipEventRecord(a, st);
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1000.f / reps / n;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int N = 1 << 20;
  float *x, *y;
  int* ptr;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&y, N * 4));
  CK(hipMalloc(&ptr, N * 4));
  std::vector<int> h(N);
  for (int i = 0; i < N; ++i) h[i] = (i * 7919) % 1024;
  CK(hipMemcpy(ptr, h.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemset(x, 0, N * 4));
  const int n = 200;
  printf("us per kernel in a %d-kernel replayed graph:\n", n);
  printf("  empty 1x64            %.2f\n", time_graph(st, n, [&](int) { hipLaunchKernelGGL(k_empty, 1, 64, 0, st); }));
  printf("  empty 256x256         %.2f\n", time_graph(st, n, [&](int) { hipLaunchKernelGGL(k_empty, 256, 256, 0, st); }));
  printf("  copy 1x64 (1 load)    %.2f\n", time_graph(st, n, [&](int i) {
           hipLaunchKernelGGL(k_copy, 1, 64, 0, st, (i & 1) ? y : x, (i & 1) ? x : y);
         }));
  printf("  chain2 1x64           %.2f\n", time_graph(st, n, [&](int i) {
           hipLaunchKernelGGL(k_chain2, 1, 64, 0, st, ptr, (i & 1) ? y : x, (i & 1) ? x : y);
         }));
  printf("  chain3 1x64           %.2f\n", time_graph(st, n, [&](int i) {
           hipLaunchKernelGGL(k_chain3, 1, 64, 0, st, ptr, (i & 1) ? y : x, (i & 1) ? x : y);
         }));
  printf("  wide 1024x256 copy    %.2f\n", time_graph(st, n, [&](int i) {
           hipLaunchKernelGGL(k_wide, 1024, 256, 0, st, (i & 1) ? y : x, (i & 1) ? x : y);
         }));
  return 0;
}
