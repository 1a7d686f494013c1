// pt_prof.hpp — per-kernel event timing hooks (see pt_prof.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptmi {
enum : int32_t { kProfMk = 0, kProfWfGenerate = 1, kProfWfIntersect = 2, kProfWfDrain = 3 /* wf_shade until round 3 */, kProfWfScatter = 4,
                 kProfWfResolve = 5, kProfMkResolve = 6, kProfKinds = 7 };
// prof_begin returns the launch's event slot (-1: not profiling / full);
// pass it to prof_end. Thread-safe: the session is guarded by a mutex and each
// launch owns its slot, so launches from several host threads pair correctly.
int prof_begin(int32_t kind, hipStream_t s);
void prof_end(int slot, hipStream_t s);
int prof_start(int32_t max_launches);
int prof_stop(double* ms, double* busy, uint64_t* launches, int32_t n_kinds);
}  // namespace ptmi
