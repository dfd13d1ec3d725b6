// Kernel-choice record and run-time tuning knobs of the size / occupancy dependent dispatches.
//
// Several entry points pick one of a few kernels from the problem size, the alignment of the
// operands and the occupancy of the current device (e.g. gasfm_gat_attn_fwd: grouped items only
// when the wave tasks fill half the resident waves).  Parity tests must know which kernel they
// exercised, so every such dispatch bumps a counter here (host side, at launch time: a captured
// graph counts once per capture, not per replay), and the thresholds can be moved at run time
// so a small test case can force every branch.
#include <atomic>
#include <cstdlib>

#include "common.hpp"

namespace gasfm {

namespace {
std::atomic<long long> g_counts[GASFM_K_COUNT];

struct Tuning {
  double v[GASFM_TUNE_COUNT];
  Tuning() {
    auto env = [](const char* name, double dflt) {
      const char* e = std::getenv(name);
      return e ? std::atof(e) : dflt;
    };
    for (double& x : v) x = 0.0;
    v[GASFM_TUNE_ATTN_GRP_ROWS] = env("GASFM_ATTN_GRP", 4);
    v[GASFM_TUNE_ATTN_GRP_MIN_FILL] = env("GASFM_ATTN_GRP_MIN_FILL", 0.5);
    v[GASFM_TUNE_ATTN_GLDS] = env("GASFM_ATTN_GLDS", 1);
    v[GASFM_TUNE_ATTN_WAVE_CAP] = env("GASFM_ATTN_WAVES", 0);
    v[GASFM_TUNE_ATTN_GRP_SPLIT] = env("GASFM_ATTN_SPLIT", 0);
  }
};

Tuning& tuning() {
  static Tuning t;
  return t;
}
}  // namespace

void note_dispatch(int kernel_id) {
  if (kernel_id >= 0 && kernel_id < GASFM_K_COUNT) g_counts[kernel_id].fetch_add(1, std::memory_order_relaxed);
}

double tune(int key) { return (key >= 0 && key < GASFM_TUNE_COUNT) ? tuning().v[key] : 0.0; }

}  // namespace gasfm

extern "C" int gasfm_dispatch_counts(int64_t* out, int32_t n) {
  for (int k = 0; k < n && k < GASFM_K_COUNT; ++k) out[k] = gasfm::g_counts[k].load(std::memory_order_relaxed);
  return GASFM_K_COUNT;
}

extern "C" void gasfm_dispatch_reset(void) {
  for (auto& c : gasfm::g_counts) c.store(0, std::memory_order_relaxed);
}

extern "C" int gasfm_tuning_set(int32_t key, double value) {
  GASFM_REQUIRE(key >= 0 && key < GASFM_TUNE_COUNT, "gasfm_tuning_set: unknown key %d", key);
  gasfm::tuning().v[key] = value;
  return GASFM_OK;
}

extern "C" double gasfm_tuning_get(int32_t key) { return gasfm::tune(key); }
