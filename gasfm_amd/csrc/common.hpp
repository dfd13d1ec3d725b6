// Shared helpers for the gasfm C ABI: status codes, thread-local error text,
// HIP error mapping.  Nothing here allocates device memory.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <cstdint>

#include "../../include/gasfm.h"

namespace gasfm {

void set_error(const char* fmt, ...);

// Kernel-choice record and run-time thresholds (dispatch.cpp; GASFM_K_* / GASFM_TUNE_* in gasfm.h).
void note_dispatch(int kernel_id);
double tune(int key);

inline int hip_status(hipError_t e, const char* where) {
  if (e == hipSuccess) return GASFM_OK;
  set_error("%s: %s", where, hipGetErrorString(e));
  return e == hipErrorOutOfMemory ? GASFM_ERR_OOM : GASFM_ERR_HIP;
}

// Status of the most recent launch on this thread (launch-config errors only;
// asynchronous faults surface at the caller's next synchronisation).
inline int launch_status(const char* where) { return hip_status(hipGetLastError(), where); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// 1 / sqrt(x) for x in the normal range -- a LayerNorm's variance + eps: the bare v_rsq_f32.
// rsqrtf's expansion only adds a denormal-input rescale around it (a compare, two multiplies and
// two selects per call) that cannot trigger here, so the result is bitwise the same (round 5).
__device__ __forceinline__ float rsq_normal(float x) { return __builtin_amdgcn_rsqf(x); }

// Workgroups of `fn` (block threads, dynamic LDS bytes) resident on the current device at once
// (occupancy x CU count; occupancy.cpp, cached).
int resident_blocks(const void* fn, int block, size_t lds);

// Grid of a grid-stride kernel: enough workgroups for `units` work units of `per_block` each,
// capped at what is resident at once.
inline int resident_grid(const void* fn, int block, size_t lds, int64_t units, int per_block) {
  const int64_t want = (units + per_block - 1) / per_block;
  const int cap = resident_blocks(fn, block, lds);
  return int(want < 1 ? 1 : (want > cap ? cap : want));
}

}  // namespace gasfm

#define GASFM_REQUIRE(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::gasfm::set_error(__VA_ARGS__);      \
      return GASFM_ERR_INVALID;             \
    }                                       \
  } while (0)
