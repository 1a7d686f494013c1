// pt_wavefront.hip — breadth-first integrator for gfx950.
//
// Replaces the wavefront stage kernels of kernels.py:1219-1418 as driven by
// TaichiRenderer.render_wavefront (renderer.py:305-334). Layout and stages
// are designed for CDNA4, not translated:
//   * ray queue = three float4 streams per slot (A = o.xyz,d.x;
//     B = d.yz,thr.xy; C = thr.z, pixel, meta) so every load/store is a
//     16-B-per-lane coalesced access; meta = depth | rng draw counter << 8
//     (the path's random stream is a function of (seed, pixel, sample, n),
//     include/ptmi_rng.h, so it travels with the ray in 24 bits);
//   * hit record = 8 B (t, leaf ref); hit point and normal are recomputed in
//     the shading kernel with the reference's own expressions;
//   * rays whose closest hit is a constant-medium boundary are compacted into
//     a separate medium queue and given their exit traversal
//     (kernels.py:417) by a dedicated kernel instead of diverging inside the
//     shading kernel;
//   * next-wave append = wave64 ballot + mbcnt prefix + ONE atomic per wave;
//     no swap copy (ping-pong pointers) and no per-wave host readback: the
//     counts stay on the device and every kernel grid-strides over them.
// Each pixel owns at most one live path per sample, so accumulator updates
// are plain read-modify-writes (no atomics) and land in the same order as
// the reference's per-pixel additions.
#include "pt_device.hpp"

namespace ptmi {

struct Queue {
  float4* a;  // o.xyz, d.x
  float4* b;  // d.y, d.z, thr.x, thr.y
  float4* c;  // thr.z, pixel (bits), meta (bits), unused
};

struct WfBufs {
  Queue q[2];
  float2* hit;       // t, ref (bits)
  int32_t* medq;     // indices into the current queue
  int32_t* counts;   // [0],[1] queue sizes, [2] medium queue size, [3] pad
  int32_t capacity;
};

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Wave-aggregated append: returns this lane's slot (valid only if want).
__device__ __forceinline__ int32_t wave_append(bool want, int32_t* counter) {
  unsigned long long mask = __ballot(want);
  if (mask == 0ull) return -1;
  int32_t prefix = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
  int32_t leader = __ffsll((long long)mask) - 1;
  int32_t base = 0;
  if (lane_id() == leader) base = atomicAdd(counter, (int32_t)__popcll(mask));
  base = __shfl(base, leader);
  return base + prefix;
}

__device__ __forceinline__ void store_ray(const Queue& q, int32_t i, pt_v3 o, pt_v3 d, pt_v3 thr, uint32_t pixel,
                                          uint32_t meta) {
  q.a[i] = make_float4(o.x, o.y, o.z, d.x);
  q.b[i] = make_float4(d.y, d.z, thr.x, thr.y);
  q.c[i] = make_float4(thr.z, __uint_as_float(pixel), __uint_as_float(meta), 0.0f);
}

__device__ __forceinline__ void accum_add(float* __restrict__ accum, uint32_t pixel, pt_v3 v) {
  float* p = accum + 3 * (size_t)pixel;
  p[0] += v.x;
  p[1] += v.y;
  p[2] += v.z;
}

// generate_camera_rays, kernels.py:1219-1239 (direction left unnormalized, Q1).
__global__ __launch_bounds__(kBlock) void wf_generate(DevFrame fr, WfBufs wb, int32_t s) {
  const int32_t npix = fr.w * fr.n_rows;
  for (int32_t i = (int32_t)(blockIdx.x * kBlock + threadIdx.x); i < npix; i += (int32_t)(gridDim.x * kBlock)) {
    int32_t lr = i / fr.w;
    int32_t px = fr.x0 + (i - lr * fr.w);
    int32_t py = frame_row(fr, lr);
    uint32_t pixel = (uint32_t)(py * fr.width + px);
    Rng r{pt_path_key(fr.seed, pixel, (uint32_t)s), 0u};
    pt_v3 o, d;
    get_ray(fr, px, py, r, o, d);
    store_ray(wb.q[0], i, o, d, pt_v3f(1.0f, 1.0f, 1.0f), pixel, r.n << 8);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    wb.counts[0] = npix;
    wb.counts[1] = 0;
    wb.counts[2] = 0;
  }
}

// intersect_rays, kernels.py:1242-1263.
template <int STACK>
__global__ __launch_bounds__(kBlock) void wf_intersect(DevScene sc, WfBufs wb, int32_t cur,
                                                       unsigned long long* __restrict__ counters) {
  __shared__ uint32_t lds_ref[STACK * kBlock];
  __shared__ float lds_t[STACK * kBlock];
  const int tid = threadIdx.x;
  Stack st{lds_ref + tid, lds_t + tid};
  const int32_t n = wb.counts[cur];
  if (blockIdx.x == 0 && tid == 0) {
    wb.counts[cur ^ 1] = 0;  // next queue (last read by the previous wave's kernels)
    wb.counts[2] = 0;
    if (counters && n > 0) atomicAdd(counters + 0, (unsigned long long)n);
  }
  const Queue q = wb.q[cur];
  for (int32_t i = (int32_t)(blockIdx.x * kBlock + tid); i < n; i += (int32_t)(gridDim.x * kBlock)) {
    float4 a = q.a[i], b = q.b[i];
    pt_v3 o = pt_v3f(a.x, a.y, a.z), d = pt_v3f(a.w, b.x, b.y);
    float t;
    int32_t ref;
    bool hit = traverse<STACK>(sc, o, d, kTMin, kTMax, st, t, ref);
    wb.hit[i] = make_float2(t, __int_as_float(hit ? ref : 0x7fffffff));
  }
}

// Shared epilogue of shade_and_scatter (kernels.py:1365-1399): emission,
// throughput update, Russian roulette, enqueue.
struct ShadeOut {
  bool enqueue;
  pt_v3 o, d, thr;
  uint32_t meta;
};

__device__ __forceinline__ void finish_scatter(const DevFrame& fr, bool scattered, pt_v3 hp, pt_v3 sdir,
                                               pt_v3 att, pt_v3 thr, int32_t depth, Rng& r, ShadeOut& out) {
  out.enqueue = false;
  if (!scattered) return;
  pt_v3 nthr = pt_mul(thr, att);
  int32_t nd = depth + 1;
  if (nd >= fr.max_depth) return;
  if (nd >= kRRMinDepth) {
    float sp = pt_minf(pt_maxf(pt_maxf(nthr.x, nthr.y), nthr.z), kRRMaxProb);
    if (r.next() > sp) return;
    nthr = pt_divs(nthr, sp);
  }
  out.enqueue = true;
  out.o = hp;
  out.d = sdir;
  out.thr = nthr;
  out.meta = (uint32_t)nd;
}

// shade_miss_rays + shade_and_scatter for non-medium hits (kernels.py:1266-1399);
// medium-boundary hits are compacted into the medium queue.
__global__ __launch_bounds__(kBlock) void wf_shade(DevScene sc, DevFrame fr, WfBufs wb, int32_t cur, int32_t s,
                                                   float* __restrict__ accum) {
  const int32_t n = wb.counts[cur];
  const Queue q = wb.q[cur];
  const Queue qo = wb.q[cur ^ 1];
  const pt_v3 bg = pt_v3f(fr.bg[0], fr.bg[1], fr.bg[2]);
  const int32_t stride = (int32_t)(gridDim.x * kBlock);
  for (int32_t base = (int32_t)(blockIdx.x * kBlock); base < n; base += stride) {
    const int32_t i = base + (int32_t)threadIdx.x;
    const bool active = i < n;
    bool to_medium = false;
    ShadeOut out;
    out.enqueue = false;
    uint32_t pixel = 0;
    if (active) {
      float2 h = wb.hit[i];
      int32_t ref = __float_as_int(h.y);
      float4 a = q.a[i], b = q.b[i], c = q.c[i];
      pt_v3 o = pt_v3f(a.x, a.y, a.z), d = pt_v3f(a.w, b.x, b.y), thr = pt_v3f(b.z, b.w, c.x);
      pixel = __float_as_uint(c.y);
      uint32_t meta = __float_as_uint(c.z);
      if (ref == 0x7fffffff) {
        accum_add(accum, pixel, pt_mul(thr, bg));  // shade_miss_rays :1280
      } else {
        const int32_t g = mat_index(sc, ref);
        if ((mat_flags(sc, g) >> 8) & 1u) {
          to_medium = true;
        } else {
          Rng r{pt_path_key(fr.seed, pixel, (uint32_t)s), meta >> 8};
          const Mat m = load_mat(sc, g);
          pt_v3 hp = pt_add(o, pt_scale(d, h.x));
          pt_v3 nrm = hit_normal(sc, ref, hp, d);
          pt_v3 emit = emitted(m);
          pt_v3 sdir, att;
          bool sc_ok = scatter(sc, ref, m, d, hp, nrm, r, sdir, att);
          if (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) accum_add(accum, pixel, pt_mul(thr, emit));
          finish_scatter(fr, sc_ok, hp, sdir, att, thr, (int32_t)(meta & 0xffu), r, out);
          out.meta |= r.n << 8;
        }
      }
    }
    int32_t mslot = wave_append(to_medium, wb.counts + 2);
    if (to_medium) wb.medq[mslot] = i;
    int32_t slot = wave_append(out.enqueue, wb.counts + (cur ^ 1));
    if (out.enqueue) store_ray(qo, slot, out.o, out.d, out.thr, pixel, out.meta);
  }
}

// Constant-medium rays: exit traversal + free flight (apply_constant_medium,
// kernels.py:365-450) and the volume branch of shade_and_scatter
// (kernels.py:1326-1357).
template <int STACK>
__global__ __launch_bounds__(kBlock) void wf_medium(DevScene sc, DevFrame fr, WfBufs wb, int32_t cur, int32_t s,
                                                    float* __restrict__ accum,
                                                    unsigned long long* __restrict__ counters) {
  __shared__ uint32_t lds_ref[STACK * kBlock];
  __shared__ float lds_t[STACK * kBlock];
  Stack st{lds_ref + threadIdx.x, lds_t + threadIdx.x};
  const int32_t n = wb.counts[2];
  if (blockIdx.x == 0 && threadIdx.x == 0 && counters && n > 0) atomicAdd(counters + 1, (unsigned long long)n);
  const Queue q = wb.q[cur];
  const Queue qo = wb.q[cur ^ 1];
  const int32_t stride = (int32_t)(gridDim.x * kBlock);
  for (int32_t base = (int32_t)(blockIdx.x * kBlock); base < n; base += stride) {
    const int32_t j = base + (int32_t)threadIdx.x;
    const bool active = j < n;
    ShadeOut out;
    out.enqueue = false;
    uint32_t pixel = 0;
    if (active) {
      const int32_t i = wb.medq[j];
      float2 h = wb.hit[i];
      int32_t ref = __float_as_int(h.y);
      float4 a = q.a[i], b = q.b[i], c = q.c[i];
      pt_v3 o = pt_v3f(a.x, a.y, a.z), d = pt_v3f(a.w, b.x, b.y), thr = pt_v3f(b.z, b.w, c.x);
      pixel = __float_as_uint(c.y);
      uint32_t meta = __float_as_uint(c.z);
      int32_t depth = (int32_t)(meta & 0xffu);
      float t_entry = h.x;
      float te;
      int32_t rex;
      bool hx = traverse<STACK>(sc, o, d, t_entry + 0.0001f, kTMax, st, te, rex);
      const Mat m = load_mat(sc, mat_index(sc, ref));
      Rng r{pt_path_key(fr.seed, pixel, (uint32_t)s), meta >> 8};
      float t_exit;
      pt_v3 mp;
      if (medium_step(hx, te, t_entry, m.m3.w, o, d, r, mp, t_exit)) {
        pt_v3 sdir = random_unit_vector(r);
        finish_scatter(fr, true, mp, sdir, pt_v3f(m.m4.x, m.m4.y, m.m4.z), thr, depth, r, out);
        out.meta |= r.n << 8;
      } else if (t_exit > 0.0f) {  // passthrough: re-enqueue, same depth (kernels.py:1342-1350)
        float eps_t = 0.001f / sqrtf(pt_dot(d, d));
        out.enqueue = true;
        out.o = pt_add(o, pt_scale(d, t_exit + eps_t));
        out.d = d;
        out.thr = thr;
        out.meta = (uint32_t)depth | (r.n << 8);
      } else {  // fallback (kernels.py:1352-1357)
        pt_v3 hp = pt_add(o, pt_scale(d, t_entry));
        pt_v3 nrm = hit_normal(sc, ref, hp, d);
        pt_v3 emit = emitted(m);
        pt_v3 sdir, att;
        bool sc_ok = scatter(sc, ref, m, d, hp, nrm, r, sdir, att);
        if (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) accum_add(accum, pixel, pt_mul(thr, emit));
        finish_scatter(fr, sc_ok, hp, sdir, att, thr, depth, r, out);
        out.meta |= r.n << 8;
      }
    }
    int32_t slot = wave_append(out.enqueue, wb.counts + (cur ^ 1));
    if (out.enqueue) store_ray(qo, slot, out.o, out.d, out.thr, pixel, out.meta);
  }
}

static inline unsigned grid_for(int32_t n) {
  int64_t b = ((int64_t)n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (unsigned)b;
}

template <int STACK>
static hipError_t wf_run(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, float* accum, int32_t s_begin,
                         int32_t s_count, unsigned long long* counters, hipStream_t stream) {
  const int32_t npix = fr.w * fr.n_rows;
  const unsigned g = grid_for(npix);
  for (int32_t s = s_begin; s < s_begin + s_count; ++s) {
    hipLaunchKernelGGL(wf_generate, dim3(g), dim3(kBlock), 0, stream, fr, wb, s);
    int32_t cur = 0;
    // renderer.py:313 — at most max_depth waves; leftover rays are dropped (Q14).
    for (int32_t wave = 0; wave < fr.max_depth; ++wave) {
      hipLaunchKernelGGL(wf_intersect<STACK>, dim3(g), dim3(kBlock), 0, stream, sc, wb, cur, counters);
      hipLaunchKernelGGL(wf_shade, dim3(g), dim3(kBlock), 0, stream, sc, fr, wb, cur, s, accum);
      hipLaunchKernelGGL(wf_medium<STACK>, dim3(g), dim3(kBlock), 0, stream, sc, fr, wb, cur, s, accum, counters);
      cur ^= 1;
    }
  }
  return hipGetLastError();
}

size_t wf_workspace_bytes(int32_t capacity) {
  size_t cap = (size_t)(capacity > 0 ? capacity : 1);
  size_t q = 3 * sizeof(float4) * cap;
  return 2 * q + sizeof(float2) * cap + sizeof(int32_t) * cap + 64;
}

hipError_t wf_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws, int32_t capacity,
                     float* accum, int32_t s_begin, int32_t s_count, unsigned long long* counters,
                     hipStream_t stream) {
  char* p = (char*)ws;
  size_t cap = (size_t)capacity;
  WfBufs wb;
  for (int k = 0; k < 2; ++k) {
    wb.q[k].a = (float4*)p; p += sizeof(float4) * cap;
    wb.q[k].b = (float4*)p; p += sizeof(float4) * cap;
    wb.q[k].c = (float4*)p; p += sizeof(float4) * cap;
  }
  wb.hit = (float2*)p; p += sizeof(float2) * cap;
  wb.medq = (int32_t*)p; p += sizeof(int32_t) * cap;
  p = (char*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
  wb.counts = (int32_t*)p;
  wb.capacity = capacity;
  if (stack_needed <= 16) return wf_run<16>(sc, fr, wb, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= 24) return wf_run<24>(sc, fr, wb, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= 32) return wf_run<32>(sc, fr, wb, accum, s_begin, s_count, counters, stream);
  return wf_run<64>(sc, fr, wb, accum, s_begin, s_count, counters, stream);
}

}  // namespace ptmi
