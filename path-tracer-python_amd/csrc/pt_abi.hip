// pt_abi.hip — the extern "C" boundary of libptmi.so (declared in
// include/ptmi.h): argument validation, scene/frame conversion, launch of the
// megakernel / wavefront / tone-map / clear kernels. No device allocation
// happens inside a render call; the megakernel calls are asynchronous and
// graph-capturable, the wavefront reads its live-slot counts back every 4
// iterations (pinned 4-byte slots, allocated once).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "pt_launch.hpp"
#include "pt_prof.hpp"

namespace ptmi {

// clear_accum_buffer, kernels.py:1205-1209 (restricted to the frame's pixel set).
__global__ __launch_bounds__(kBlock) void clear_kernel(DevFrame fr, float* __restrict__ accum) {
  const int32_t npix = fr.w * fr.n_rows;
  for (int32_t i = (int32_t)(blockIdx.x * kBlock + threadIdx.x); i < npix; i += (int32_t)(gridDim.x * kBlock)) {
    int32_t lr = i / fr.w;
    int32_t px = fr.x0 + (i - lr * fr.w);
    int32_t py = frame_row(fr, lr);
    float* p = accum + 3 * ((size_t)py * (size_t)fr.width + (size_t)px);
    p[0] = 0.0f;
    p[1] = 0.0f;
    p[2] = 0.0f;
  }
}

// LivePreview.buffer_to_image, preview.py:117-132. numpy evaluates
// accum * scale in f32 (NEP 50), sqrt(max(0, x)) in f32, * 255.999 in f32,
// clip to [0, 255] and truncates to u8.
__global__ __launch_bounds__(kBlock) void tonemap_kernel(const float* __restrict__ accum, uint8_t* __restrict__ out,
                                                         int32_t n, float scale) {
  for (int32_t i = (int32_t)(blockIdx.x * kBlock + threadIdx.x); i < n; i += (int32_t)(gridDim.x * kBlock)) {
    float x = accum[i] * scale;
    float g = sqrtf(pt_maxf(x, 0.0f));
    float v = g * 255.999f;
    v = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
    out[i] = (uint8_t)(int32_t)v;
  }
}
}  // namespace ptmi

using namespace ptmi;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

static int check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(PTMI_EHIP, "%s: %s", what, hipGetErrorString(e));
  return PTMI_OK;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

static int to_dev_scene(const ptmi_scene_view* s, DevScene& d) {
  if (!s) return fail(PTMI_EINVAL, "scene is NULL");
  int32_t np = s->num_spheres + s->num_quads + s->num_triangles;
  if (s->num_spheres < 0 || s->num_quads < 0 || s->num_triangles < 0 || s->n_inner < 0)
    return fail(PTMI_EINVAL, "negative scene counts");
  if (np > 0x0fffffff) return fail(PTMI_ECAPACITY, "too many primitives (%d)", np);
  if (s->num_spheres > (1 << 25) || s->num_quads > (1 << 25) || s->num_triangles > (1 << 25))
    return fail(PTMI_ECAPACITY, "more than 2^25 primitives of one type (25-bit leaf index)");
  if (np > 0 && s->n_inner != np - 1)
    return fail(PTMI_EINVAL, "binary BVH with one primitive per leaf needs n_inner = prims - 1 (%d vs %d)",
                s->n_inner, np - 1);
  if (s->n_inner > 0 && (!s->nodes || !aligned16(s->nodes))) return fail(PTMI_EINVAL, "nodes NULL/misaligned");
  if (s->num_spheres > 0 && (!s->spheres || !aligned16(s->spheres))) return fail(PTMI_EINVAL, "spheres");
  if (s->num_quads > 0 && (!s->quads || !aligned16(s->quads))) return fail(PTMI_EINVAL, "quads");
  if (s->num_triangles > 0 && (!s->tris || !aligned16(s->tris))) return fail(PTMI_EINVAL, "tris");
  if (np > 0 && (!s->mats || !aligned16(s->mats))) return fail(PTMI_EINVAL, "mats");
  if (!s->perlin_vec || !aligned16(s->perlin_vec) || !s->perlin_perm) return fail(PTMI_EINVAL, "perlin tables");
  if (s->num_images < 0 || s->num_images > PTMI_MAX_IMAGES) return fail(PTMI_EINVAL, "num_images");
  if (s->num_images > 0 && !s->texels) return fail(PTMI_EINVAL, "texels");
  // The reference's 64-slot stack never overflows for leaf depth <= 62
  // (kernels.py:719-740); deeper BVHs run its exact walk on its own nodes,
  // silent drops included (TravRS, pt_device.hpp), which needs ref_nodes.
  if (s->max_leaf_depth < 0) return fail(PTMI_EINVAL, "negative max_leaf_depth");
  if (s->max_leaf_depth > 62 && np > 0 && !s->ref_nodes)
    return fail(PTMI_EINVAL, "BVH leaf depth %d > 62 needs ref_nodes (the reference's 64-entry stack walk)",
                s->max_leaf_depth);
  if (s->num_bvh_nodes != (np > 0 ? 2 * np - 1 : 0))
    return fail(PTMI_EINVAL, "num_bvh_nodes %d for %d primitives (expected 2N-1)", s->num_bvh_nodes, np);
  if (s->ref_nodes && !aligned16(s->ref_nodes)) return fail(PTMI_EINVAL, "ref_nodes misaligned");
  std::memset(&d, 0, sizeof d);
  d.nodes = (const float4*)s->nodes;
  d.n_inner = s->n_inner;
  d.root_ref = (np > 0) ? s->root_ref : 0;
  for (int k = 0; k < 3; ++k) {
    d.root_min[k] = s->root_min[k];
    d.root_max[k] = s->root_max[k];
  }
  d.spheres = (const float4*)s->spheres;
  d.quads = (const float4*)s->quads;
  d.tris = (const float4*)s->tris;
  d.mats = (const float4*)s->mats;
  d.mat_base[kSphere] = 0;
  d.mat_base[kQuad] = s->num_spheres;
  d.mat_base[kTriangle] = s->num_spheres + s->num_quads;
  d.texels = s->texels;
  d.num_images = s->num_images;
  for (int k = 0; k < PTMI_MAX_IMAGES; ++k) {
    d.img_offset[k] = s->img_offset[k];
    d.img_w[k] = s->img_w[k];
    d.img_h[k] = s->img_h[k];
  }
  d.perlin_vec = (const float4*)s->perlin_vec;
  d.perlin_perm = s->perlin_perm;
  d.ref_nodes = (const float4*)s->ref_nodes;
  d.n_nodes = s->num_bvh_nodes;
  return PTMI_OK;
}

static int to_dev_frame(const ptmi_frame* f, DevFrame& d) {
  if (!f) return fail(PTMI_EINVAL, "frame is NULL");
  if (f->width <= 0 || f->height <= 0 || f->w <= 0 || f->h <= 0 || f->x0 < 0 || f->y0 < 0 ||
      f->x0 + f->w > f->width || f->y0 + f->h > f->height)
    return fail(PTMI_EINVAL, "bad window %d,%d %dx%d in %dx%d", f->x0, f->y0, f->w, f->h, f->width, f->height);
  if ((int64_t)f->width * (int64_t)f->height > (int64_t)0x7fffffff / 3)
    return fail(PTMI_ECAPACITY, "image too large");
  if (f->band_rows <= 0 || f->band_stride <= 0 || f->band_offset < 0 || f->band_offset >= f->band_stride)
    return fail(PTMI_EINVAL, "bad band partition");
  if (f->max_depth < 0 || f->max_depth > 255) return fail(PTMI_EINVAL, "max_depth must be in [0, 255]");
  std::memset(&d, 0, sizeof d);
  for (int k = 0; k < 3; ++k) {
    d.center[k] = f->cam.center[k];
    d.pixel00[k] = f->cam.pixel00[k];
    d.delta_u[k] = f->cam.delta_u[k];
    d.delta_v[k] = f->cam.delta_v[k];
    d.defocus_u[k] = f->cam.defocus_u[k];
    d.defocus_v[k] = f->cam.defocus_v[k];
    d.bg[k] = f->bg[k];
  }
  d.defocus_angle = f->cam.defocus_angle;
  d.max_depth = f->max_depth;
  d.seed = f->seed;
  d.width = f->width;
  d.height = f->height;
  d.x0 = f->x0;
  d.y0 = f->y0;
  d.w = f->w;
  d.h = f->h;
  d.band_rows = f->band_rows;
  d.band_stride = f->band_stride;
  d.band_offset = f->band_offset;
  if (f->traversal != PTMI_TRAV_STACK && f->traversal != PTMI_TRAV_STACKLESS)
    return fail(PTMI_EINVAL, "unknown traversal %d", f->traversal);
  d.traversal = f->traversal;
  int32_t n = 0;
  for (int32_t r = 0; r < f->h; ++r)
    if ((r / f->band_rows) % f->band_stride == f->band_offset) ++n;
  d.n_rows = n;
  return PTMI_OK;
}

static int32_t stack_needed(const ptmi_scene_view* s) { return s->max_leaf_depth + 1; }

// The stackless traversal walks the reference-layout nodes (ref_nodes).
static int check_traversal(const DevScene& sc, const DevFrame& fr) {
  if (fr.traversal == PTMI_TRAV_STACKLESS && sc.n_nodes > 0 && !sc.ref_nodes)
    return fail(PTMI_EINVAL, "the stackless traversal needs the scene's ref_nodes");
  return PTMI_OK;
}

extern "C" {

int ptmi_version(void) { return PTMI_ABI_VERSION; }

int ptmi_node_bytes(void) { return (int)kNodeBytes; }

const char* ptmi_last_error(void) { return g_err.c_str(); }

int ptmi_scene_check(const ptmi_scene_view* scene) {
  DevScene d;
  return to_dev_scene(scene, d);
}

int ptmi_mk_render(const ptmi_scene_view* scene, const ptmi_frame* frame, float* accum, int32_t sample_begin,
                   int32_t sample_count, uint64_t* counters, void* stream) {
  DevScene sc;
  DevFrame fr;
  int rc = to_dev_scene(scene, sc);
  if (rc) return rc;
  if ((rc = to_dev_frame(frame, fr))) return rc;
  if ((rc = check_traversal(sc, fr))) return rc;
  if (!accum) return fail(PTMI_EINVAL, "accum is NULL");
  if (sample_begin < 0 || sample_count < 0) return fail(PTMI_EINVAL, "bad sample range");
  if (sample_count == 0 || fr.n_rows == 0) return PTMI_OK;
  return check_hip(mk_render(sc, fr, stack_needed(scene), accum, sample_begin, sample_count,
                             (unsigned long long*)counters, (hipStream_t)stream),
                   "mk_render launch");
}

size_t ptmi_mk_workspace_bytes(const ptmi_frame* frame, int32_t batch_samples) {
  DevFrame fr;
  if (to_dev_frame(frame, fr)) return 0;
  if (batch_samples <= 0) {
    fail(PTMI_EINVAL, "batch_samples must be > 0");
    return 0;
  }
  return mk_workspace_bytes(fr.w * fr.n_rows, batch_samples);
}

int ptmi_mk_render_ws(const ptmi_scene_view* scene, const ptmi_frame* frame, void* workspace,
                      size_t workspace_bytes, float* accum, int32_t sample_begin, int32_t sample_count,
                      uint64_t* counters, void* stream) {
  DevScene sc;
  DevFrame fr;
  int rc = to_dev_scene(scene, sc);
  if (rc) return rc;
  if ((rc = to_dev_frame(frame, fr))) return rc;
  if ((rc = check_traversal(sc, fr))) return rc;
  if (!accum) return fail(PTMI_EINVAL, "accum is NULL");
  if (sample_begin < 0 || sample_count < 0) return fail(PTMI_EINVAL, "bad sample range");
  const int32_t npix = fr.w * fr.n_rows;
  if (npix == 0) return PTMI_OK;
  if (!workspace || !aligned16(workspace) || workspace_bytes < mk_workspace_bytes(npix, 1))
    return fail(PTMI_EINVAL, "workspace too small/misaligned (%zu < %zu)", workspace_bytes,
                mk_workspace_bytes(npix, 1));
  if (sample_count == 0) return PTMI_OK;
  return check_hip(mk_render_staged(sc, fr, stack_needed(scene), workspace, workspace_bytes, accum, sample_begin,
                                    sample_count, (unsigned long long*)counters, (hipStream_t)stream),
                   "mk_render_ws");
}

int ptmi_mk_trace_ws(const ptmi_scene_view* scene, const ptmi_frame* frame, void* workspace, size_t workspace_bytes,
                     int32_t sample_begin, int32_t sample_count, uint64_t* counters, void* stream) {
  DevScene sc;
  DevFrame fr;
  int rc = to_dev_scene(scene, sc);
  if (rc) return rc;
  if ((rc = to_dev_frame(frame, fr))) return rc;
  if ((rc = check_traversal(sc, fr))) return rc;
  if (sample_begin < 0 || sample_count < 1) return fail(PTMI_EINVAL, "bad sample range");
  const int32_t npix = fr.w * fr.n_rows;
  if (npix == 0) return PTMI_OK;
  if ((int64_t)sample_count > mk_max_batch(fr))
    return fail(PTMI_ECAPACITY, "%d samples exceed one batch's 2^32 item ids", sample_count);
  const size_t need = mk_workspace_bytes(npix, sample_count);
  if (!workspace || !aligned16(workspace) || workspace_bytes < need)
    return fail(PTMI_EINVAL, "workspace too small/misaligned for one batch (%zu < %zu)", workspace_bytes, need);
  return check_hip(mk_trace_staged(sc, fr, stack_needed(scene), workspace, sample_begin, sample_count,
                                   (unsigned long long*)counters, (hipStream_t)stream),
                   "mk_trace_ws");
}

int64_t ptmi_mk_max_batch(const ptmi_frame* frame) {
  DevFrame fr;
  if (to_dev_frame(frame, fr)) return 0;
  return mk_max_batch(fr);
}

int ptmi_mk_resolve_ws(const ptmi_frame* frame, const void* workspace, size_t workspace_bytes, float* accum,
                       int32_t sample_count, void* stream) {
  DevFrame fr;
  int rc = to_dev_frame(frame, fr);
  if (rc) return rc;
  if (!accum) return fail(PTMI_EINVAL, "accum is NULL");
  if (sample_count < 1) return fail(PTMI_EINVAL, "sample_count must be >= 1");
  const int32_t npix = fr.w * fr.n_rows;
  if (npix == 0) return PTMI_OK;
  const size_t need = mk_workspace_bytes(npix, sample_count);
  if (!workspace || !aligned16(workspace) || workspace_bytes < need)
    return fail(PTMI_EINVAL, "workspace too small/misaligned for one batch (%zu < %zu)", workspace_bytes, need);
  return check_hip(launch_stage_resolve(fr, (const float*)workspace, npix, sample_count, accum, kProfMkResolve,
                                        (hipStream_t)stream),
                   "mk_resolve_ws");
}

size_t ptmi_wf_workspace_bytes(const ptmi_frame* frame, int32_t batch_samples) {
  DevFrame fr;
  if (to_dev_frame(frame, fr)) return 0;
  if (batch_samples <= 0) {
    fail(PTMI_EINVAL, "batch_samples must be > 0");
    return 0;
  }
  if ((int64_t)fr.w * fr.n_rows * batch_samples > 0x7fffffff) {
    fail(PTMI_ECAPACITY, "pixels x batch_samples exceeds 2^31 work items");
    return 0;
  }
  return wf_workspace_bytes(fr.w * fr.n_rows, batch_samples);
}

int ptmi_wf_render(const ptmi_scene_view* scene, const ptmi_frame* frame, void* workspace, size_t workspace_bytes,
                   float* accum, int32_t sample_begin, int32_t sample_count, uint64_t* counters, void* stream) {
  DevScene sc;
  DevFrame fr;
  int rc = to_dev_scene(scene, sc);
  if (rc) return rc;
  if ((rc = to_dev_frame(frame, fr))) return rc;
  if ((rc = check_traversal(sc, fr))) return rc;
  if (!accum) return fail(PTMI_EINVAL, "accum is NULL");
  if (sample_begin < 0 || sample_count < 0) return fail(PTMI_EINVAL, "bad sample range");
  int32_t npix = fr.w * fr.n_rows;
  if (npix == 0) return PTMI_OK;
  if (!workspace || !aligned16(workspace) || workspace_bytes < wf_workspace_bytes(npix, 1))
    return fail(PTMI_EINVAL, "workspace too small/misaligned (%zu < %zu)", workspace_bytes,
                wf_workspace_bytes(npix, 1));
  if (sample_count == 0) return PTMI_OK;
  return check_hip(wf_render(sc, fr, stack_needed(scene), workspace, workspace_bytes, accum, sample_begin,
                             sample_count, (unsigned long long*)counters, (hipStream_t)stream),
                   "wf_render");
}

int ptmi_wf_set_drain_at(int32_t divisor) {
  if (divisor < 0) return fail(PTMI_EINVAL, "drain divisor must be >= 0");
  return wf_set_drain_at(divisor);
}

int ptmi_clear(const ptmi_frame* frame, float* accum, void* stream) {
  DevFrame fr;
  int rc = to_dev_frame(frame, fr);
  if (rc) return rc;
  if (!accum) return fail(PTMI_EINVAL, "accum is NULL");
  int32_t npix = fr.w * fr.n_rows;
  if (npix == 0) return PTMI_OK;
  unsigned g = (unsigned)((npix + kBlock - 1) / kBlock);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(clear_kernel, dim3(g), dim3(kBlock), 0, (hipStream_t)stream, fr, accum);
  return check_hip(hipGetLastError(), "clear launch");
}

int ptmi_tonemap(const float* accum, uint8_t* out, int32_t width, int32_t height, int32_t spp, void* stream) {
  if (!accum || !out || width <= 0 || height <= 0) return fail(PTMI_EINVAL, "bad tonemap arguments");
  int64_t n = (int64_t)width * height * 3;
  if (n > 0x7fffffff) return fail(PTMI_ECAPACITY, "image too large");
  float scale = (float)(1.0 / (double)(spp > 1 ? spp : 1));  // python float -> f32 (NEP 50)
  unsigned g = (unsigned)((n + kBlock - 1) / kBlock);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(tonemap_kernel, dim3(g), dim3(kBlock), 0, (hipStream_t)stream, accum, out, (int32_t)n, scale);
  return check_hip(hipGetLastError(), "tonemap launch");
}

int ptmi_prof_start(int32_t max_launches) {
  if (max_launches < 0) return fail(PTMI_EINVAL, "max_launches < 0");
  if (prof_start(max_launches)) return fail(PTMI_EHIP, "hipEventCreate failed");
  return PTMI_OK;
}

int ptmi_prof_stop(double* ms_by_kernel, uint64_t* launches_by_kernel, int32_t n_kinds) {
  return ptmi_prof_stop_busy(ms_by_kernel, nullptr, launches_by_kernel, n_kinds);
}

int ptmi_prof_stop_busy(double* ms_by_kernel, double* busy_ms_by_kernel, uint64_t* launches_by_kernel,
                        int32_t n_kinds) {
  if (!ms_by_kernel || !launches_by_kernel || n_kinds < 0) return fail(PTMI_EINVAL, "bad arguments");
  int rc = prof_stop(ms_by_kernel, busy_ms_by_kernel, launches_by_kernel, n_kinds < kProfKinds ? n_kinds : kProfKinds);
  for (int32_t k = kProfKinds; k < n_kinds; ++k) {
    ms_by_kernel[k] = 0.0;
    launches_by_kernel[k] = 0;
    if (busy_ms_by_kernel) busy_ms_by_kernel[k] = 0.0;
  }
  if (rc < 0) return fail(PTMI_EHIP, "event timing failed");
  if (rc > 0) return fail(PTMI_ECAPACITY, "more launches than the profiling pool; counts truncated");
  return PTMI_OK;
}

}  // extern "C"
