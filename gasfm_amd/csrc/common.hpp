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

inline int hip_status(hipError_t e, const char* where) {
  if (e == hipSuccess) return GASFM_OK;
  set_error("%s: %s", where, hipGetErrorString(e));
  return e == hipErrorOutOfMemory ? GASFM_ERR_OOM : GASFM_ERR_HIP;
}

// Status of the most recent launch on this thread (launch-config errors only;
// asynchronous faults surface at the caller's next synchronisation).
inline int launch_status(const char* where) { return hip_status(hipGetLastError(), where); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace gasfm

#define GASFM_REQUIRE(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::gasfm::set_error(__VA_ARGS__);      \
      return GASFM_ERR_INVALID;             \
    }                                       \
  } while (0)
