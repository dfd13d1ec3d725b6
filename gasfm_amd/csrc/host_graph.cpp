// Host-side (CPU) graph preprocessing for the GASFM attention kernels.
//
// The reference builds its four "axial aggregation" star graphs as PyG
// edge_index tensors (utils/dataset_utils.py:511-537) and leaves the grouping
// of edges by destination to PyG's scatter.  The kernels here instead consume
// destination-sorted edge lists: the camera direction is already CSR because
// M2sparse emits edges cam-major (dataset_utils.py:129-143), the point
// direction needs a stable counting sort (gasfm_build_csr), and long
// segments are split into pieces for load balance (gasfm_plan_work).
// Runs in DataLoader workers, so it is plain C++ with no device calls.
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"

namespace gasfm {
static thread_local char g_err[512] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace gasfm

extern "C" const char* gasfm_last_error(void) { return gasfm::g_err; }
extern "C" int gasfm_version(void) { return 1; }

extern "C" int gasfm_build_csr(const int32_t* key, int64_t E, int32_t n, int32_t* ptr,
                               int32_t* perm) {
  GASFM_REQUIRE(E >= 0 && n >= 0, "gasfm_build_csr: negative size");
  GASFM_REQUIRE(E < INT32_MAX, "gasfm_build_csr: E=%lld exceeds int32 edge ids", (long long)E);
  GASFM_REQUIRE(ptr != nullptr && (E == 0 || (key && perm)), "gasfm_build_csr: null pointer");
  std::memset(ptr, 0, sizeof(int32_t) * (size_t(n) + 1));
  for (int64_t e = 0; e < E; ++e) {
    const int32_t k = key[e];
    GASFM_REQUIRE(k >= 0 && k < n, "gasfm_build_csr: key[%lld]=%d outside [0,%d)", (long long)e, k,
                  n);
    ++ptr[k + 1];
  }
  for (int32_t i = 0; i < n; ++i) ptr[i + 1] += ptr[i];
  std::vector<int32_t> fill(ptr, ptr + n);
  for (int64_t e = 0; e < E; ++e) perm[fill[key[e]]++] = int32_t(e);
  return GASFM_OK;
}

extern "C" int gasfm_plan_work(const int32_t* seg_ptr, int32_t N, int32_t max_piece,
                               int32_t all_partial, gasfm_work_item* items, int32_t* n_items,
                               gasfm_combine_item* combine, int32_t* n_combine,
                               int32_t* n_slots) {
  GASFM_REQUIRE(seg_ptr && n_items && n_combine && n_slots, "gasfm_plan_work: null pointer");
  GASFM_REQUIRE(N >= 0 && max_piece > 0, "gasfm_plan_work: N=%d max_piece=%d", N, max_piece);
  const int32_t cap_items = *n_items, cap_comb = *n_combine;
  int64_t ni = 0, nc = 0, ns = all_partial ? N : 0;
  for (int32_t s = 0; s < N; ++s) {
    const int32_t b = seg_ptr[s], e = seg_ptr[s + 1];
    GASFM_REQUIRE(e >= b, "gasfm_plan_work: seg_ptr not monotone at %d", s);
    const int32_t len = e - b;
    if (len <= max_piece) {
      if (ni < cap_items && items) items[ni] = {s, b, e, all_partial ? s : -1};
      ++ni;
      continue;
    }
    const int32_t pieces = (len + max_piece - 1) / max_piece;
    // even split: pieces differ by at most one edge
    const int32_t base = len / pieces, rem = len % pieces;
    int32_t at = b;
    const int64_t first_slot = ns;
    for (int32_t p = 0; p < pieces; ++p) {
      const int32_t l = base + (p < rem ? 1 : 0);
      if (ni < cap_items && items) items[ni] = {s, at, at + l, int32_t(ns)};
      ++ni;
      ++ns;
      at += l;
    }
    if (nc < cap_comb && combine) combine[nc] = {s, int32_t(first_slot), pieces, 1};
    ++nc;
  }
  GASFM_REQUIRE(ni < INT32_MAX && ns < INT32_MAX, "gasfm_plan_work: too many items");
  const bool fits = ni <= cap_items && nc <= cap_comb;
  *n_items = int32_t(ni);
  *n_combine = int32_t(nc);
  *n_slots = int32_t(ns);
  if (!fits) {
    gasfm::set_error("gasfm_plan_work: capacity too small (need %lld items, %lld combine)",
                     (long long)ni, (long long)nc);
    return GASFM_ERR_INVALID;
  }
  return GASFM_OK;
}
