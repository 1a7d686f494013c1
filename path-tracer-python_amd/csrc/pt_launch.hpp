// pt_launch.hpp — host-side launchers shared between the translation units
// of libptmi.so (pt_abi.hip calls them; pt_wavefront.hip reuses the staged
// resolve of pt_megakernel.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pt_device.hpp"

namespace ptmi {
// Megakernel, accumulating in registers straight into accum (one work unit
// per 16x16 tile for all samples of the call).
hipError_t mk_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, float* accum,
                     int32_t s_begin, int32_t s_count, unsigned long long* counters, hipStream_t stream);
// Megakernel over (tile, sample chunk) work units, colours staged per
// (sample, pixel) and resolved in sample order.
size_t mk_workspace_bytes(int32_t npix, int32_t batch);
hipError_t mk_render_staged(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws,
                            size_t ws_bytes, float* accum, int32_t s_begin, int32_t s_count,
                            unsigned long long* counters, hipStream_t stream);
// The two halves of one staged batch, for callers that schedule them
// themselves (ptmi_mk_trace_ws / ptmi_mk_resolve_ws): the megakernel into the
// workspace's staging, and the in-order resolve into accum.
hipError_t mk_trace_staged(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws,
                           int32_t s_begin, int32_t nb, unsigned long long* counters, hipStream_t stream);
int64_t mk_max_batch(const DevFrame& fr);
hipError_t wf_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws, size_t ws_bytes,
                     float* accum, int32_t s_begin, int32_t s_count, unsigned long long* counters,
                     hipStream_t stream);
size_t wf_workspace_bytes(int32_t npix, int32_t batch);
// Sets the wavefront tail threshold (capacity / divisor; 0 = no tail launch); returns the previous one.
int32_t wf_set_drain_at(int32_t divisor);
// accum[pixel] += staging[s][p] for s = 0..batch-1 in order (profiled as `prof_kind`).
hipError_t launch_stage_resolve(const DevFrame& fr, const float* staging, int32_t npix, int32_t batch,
                                float* accum, int prof_kind, hipStream_t stream);
}  // namespace ptmi
