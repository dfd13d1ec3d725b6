// Resident-workgroup counts of the grid-stride kernels (cached per kernel, block size and
// dynamic LDS).  A grid larger than what the chip holds at once leaves a second round of
// workgroups, each carrying a full share of the work (measured on the attention kernels:
// 278 us at 8192 waves vs 193 us at the 7168 that fit) and, for kernels that write one
// weight-gradient partial row per workgroup, a larger partial buffer to reduce.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.hpp"

namespace gasfm {

int resident_blocks(const void* fn, int block, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, size_t, int>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(fn, block, lds, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  (void)hipGetLastError();
  const int v = per_cu * cus;
  cache[key] = v;
  return v;
}

}  // namespace gasfm
