// pt_prof.hip — optional per-kernel HIP-event timing of the integrator's own
// launches (the reference's equivalent is Taichi's kernel profiler,
// renderer.py:15-16 / interactive_viewer.py:241-247). Events are recorded on
// the launch stream right before and after each kernel, so elapsed times are
// the kernels' device durations; collection synchronises once at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>

#include "pt_prof.hpp"

namespace ptmi {
namespace {
struct Prof {
  bool on = false;
  std::vector<hipEvent_t> ev;   // pairs
  std::vector<int32_t> kind;    // one per pair
  size_t used = 0;              // events used
  bool overflow = false;
};
Prof g_prof;
std::mutex g_prof_mu;  // one session per process, used from any host thread
}  // namespace

int prof_begin(int32_t kind, hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_prof_mu);
  if (!g_prof.on) return -1;
  if (g_prof.used + 2 > g_prof.ev.size()) {
    g_prof.overflow = true;
    return -1;
  }
  const int slot = (int)(g_prof.used / 2);
  g_prof.kind.push_back(kind);
  g_prof.used += 2;
  (void)hipEventRecord(g_prof.ev[2 * (size_t)slot], s);
  return slot;
}

void prof_end(int slot, hipStream_t s) {
  if (slot < 0) return;
  std::lock_guard<std::mutex> lock(g_prof_mu);
  if (!g_prof.on || 2 * (size_t)slot + 1 >= g_prof.ev.size()) return;
  (void)hipEventRecord(g_prof.ev[2 * (size_t)slot + 1], s);
}

int prof_start(int32_t max_launches) {
  std::lock_guard<std::mutex> lock(g_prof_mu);
  for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
  g_prof = Prof();
  if (max_launches <= 0) return 0;
  g_prof.ev.resize(2 * (size_t)max_launches);
  for (auto& e : g_prof.ev)
    if (hipEventCreate(&e) != hipSuccess) return -1;
  g_prof.kind.reserve((size_t)max_launches);
  g_prof.on = true;
  return 0;
}

// busy (may be null): per kind, the length of the union of its launches'
// [start, end] intervals (event times relative to the session's first event).
// Launches of one kind that overlap in time (the megakernel's pipelined calls
// on two streams, the wavefront's pipes) count once there, so busy / launches
// is the GPU time per launch, while ms sums each launch's own duration.
int prof_stop(double* ms, double* busy, uint64_t* launches, int32_t n_kinds) {
  std::lock_guard<std::mutex> lock(g_prof_mu);
  for (int32_t k = 0; k < n_kinds; ++k) {
    ms[k] = 0.0;
    launches[k] = 0;
    if (busy) busy[k] = 0.0;
  }
  int rc = g_prof.overflow ? 1 : 0;
  std::vector<std::vector<std::pair<double, double>>> iv((size_t)(n_kinds > 0 ? n_kinds : 0));
  for (size_t p = 0; p + 1 < g_prof.used; p += 2) {
    float t = 0.0f;
    // launches may sit on several streams (wavefront pipes): wait for each
    if (hipEventSynchronize(g_prof.ev[p + 1]) != hipSuccess) { rc = -1; continue; }
    if (hipEventElapsedTime(&t, g_prof.ev[p], g_prof.ev[p + 1]) != hipSuccess) { rc = -1; continue; }
    int32_t k = g_prof.kind[p / 2];
    if (k >= 0 && k < n_kinds) {
      ms[k] += (double)t;
      launches[k] += 1;
      float t0 = 0.0f;
      if (busy && hipEventElapsedTime(&t0, g_prof.ev[0], g_prof.ev[p]) == hipSuccess)
        iv[(size_t)k].emplace_back((double)t0, (double)t0 + (double)t);
    }
  }
  if (busy) {
    for (int32_t k = 0; k < n_kinds; ++k) {
      auto& v = iv[(size_t)k];
      std::sort(v.begin(), v.end());
      double cur_s = 0.0, cur_e = -1.0, sum = 0.0;
      for (const auto& x : v) {
        if (x.first > cur_e) {
          if (cur_e > cur_s) sum += cur_e - cur_s;
          cur_s = x.first;
          cur_e = x.second;
        } else if (x.second > cur_e) {
          cur_e = x.second;
        }
      }
      if (cur_e > cur_s) sum += cur_e - cur_s;
      busy[k] = sum;
    }
  }
  for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
  g_prof = Prof();
  return rc;
}
}  // namespace ptmi
