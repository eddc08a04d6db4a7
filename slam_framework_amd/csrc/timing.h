// timing.h -- optional per-kernel HIP-event timing of the launches a context issues.
//
// When a context has timing enabled, every launch issued through SLAMGPU_LAUNCH is bracketed by
// two hipEventRecord calls on the launch stream (events come from a pre-created pool, so no
// allocation happens on the launch path). bench.py uses this to measure the dominant kernel's
// average duration live, over its timed region, on the stream the kernel runs on.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

namespace slamgpu {

struct KernelTimer {
  bool on = false;
  std::string target;              // kernel name, or "*" for every kernel
  std::vector<hipEvent_t> pool;    // 2 per recorded launch
  std::vector<const char*> names;  // name of each recorded launch
  size_t used = 0;
  bool overflow = false;

  bool wants(const char* name) const {
    return on && (target == "*" || target == name);
  }
  void begin(const char* name, hipStream_t st) {
    if (!wants(name)) return;
    if (2 * (used + 1) > pool.size()) {
      overflow = true;
      return;
    }
    (void)hipEventRecord(pool[2 * used], st);
  }
  void end(const char* name, hipStream_t st) {
    if (!wants(name) || 2 * (used + 1) > pool.size()) return;
    (void)hipEventRecord(pool[2 * used + 1], st);
    if (names.size() <= used) names.resize(used + 1);
    names[used] = name;
    used++;
  }
};

// The timer of the context currently issuing launches (set by the runtime around each call).
extern thread_local KernelTimer* g_timer;

#define SLAMGPU_LAUNCH(name, stream, ...)                    \
  do {                                                       \
    if (::slamgpu::g_timer) ::slamgpu::g_timer->begin(name, stream); \
    hipLaunchKernelGGL(__VA_ARGS__);                         \
    if (::slamgpu::g_timer) ::slamgpu::g_timer->end(name, stream);   \
  } while (0)

}  // namespace slamgpu
