// pt_wavefront.hip — breadth-first (wavefront) integrator for gfx950.
//
// Replaces the wavefront stage kernels of kernels.py:1219-1418 as driven by
// TaichiRenderer.render_wavefront (renderer.py:305-334). Stages and layout
// are designed for CDNA4, not translated:
//   * ray queue = three float4 streams per slot (A = o.xyz,d.x;
//     B = d.yz,thr.xy; C = thr.z, pixel, rng draw counter, meta) so every
//     load/store is a 16-B-per-lane coalesced access; meta = depth |
//     wave << 8 | sample << 16 (sample relative to the call's first);
//   * hit record = 8 B (t, leaf ref); hit point and normal are recomputed in
//     the shading kernel with the reference's own expressions;
//   * rays whose closest hit is a constant-medium boundary are compacted into
//     a separate medium queue and get their exit traversal (kernels.py:417)
//     from a dedicated kernel instead of diverging inside shading;
//   * next-queue append = wave64 ballot + mbcnt prefix + ONE atomic per wave;
//     ping-pong queues (no swap copy, kernels.py:1402-1418 removed);
//   * STREAMING: the reference runs one sample at a time through max_depth
//     bounce-synchronous waves (renderer.py:305-334), so after a few bounces
//     its queues are nearly empty. Here a path that ends is immediately
//     replaced in the queue by the camera ray of the same pixel's next
//     sample, so every launch works on a full queue. Each ray carries its
//     own wave count and is dropped when it reaches max_depth waves, exactly
//     the reference's per-path budget (Q14, incl. passthrough waves Q11), and
//     a pixel's samples still run one after another, so per-path results
//     and the per-pixel accumulation order are those of the reference loop.
// Each pixel owns at most one live path at a time, so accumulator updates
// are plain read-modify-writes (no atomics).
#include "pt_device.hpp"
#include "pt_prof.hpp"

namespace ptmi {

struct Queue {
  float4* a;  // o.xyz, d.x
  float4* b;  // d.y, d.z, thr.x, thr.y
  float4* c;  // thr.z, pixel, rng counter, meta (bits)
};

struct WfBufs {
  Queue q[2];
  float2* hit;       // t, ref (bits); ref 0x7fffffff = miss
  int32_t* medq;     // indices into the current queue
  int32_t* counts;   // [0],[1] queue sizes, [2] medium queue size, [3] pad
  int32_t capacity;
};

constexpr int32_t kMissRef = 0x7fffffff;

__device__ __forceinline__ uint32_t pack_meta(int32_t depth, int32_t wave, int32_t srel) {
  return (uint32_t)depth | ((uint32_t)wave << 8) | ((uint32_t)srel << 16);
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Wave-aggregated append: returns this lane's slot (meaningful only if want).
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

__device__ __forceinline__ void wave_count(bool flag, unsigned long long* counter) {
  unsigned long long mask = __ballot(flag);
  if (counter && mask && lane_id() == __ffsll((long long)mask) - 1)
    atomicAdd(counter, (unsigned long long)__popcll(mask));
}

struct Ray {
  pt_v3 o, d, thr;
  uint32_t pixel, ctr, meta;
};

__device__ __forceinline__ void store_ray(const Queue& q, int32_t i, const Ray& r) {
  q.a[i] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
  q.b[i] = make_float4(r.d.y, r.d.z, r.thr.x, r.thr.y);
  q.c[i] = make_float4(r.thr.z, __uint_as_float(r.pixel), __uint_as_float(r.ctr), __uint_as_float(r.meta));
}

__device__ __forceinline__ Ray load_ray(const Queue& q, int32_t i) {
  float4 a = q.a[i], b = q.b[i], c = q.c[i];
  Ray r;
  r.o = pt_v3f(a.x, a.y, a.z);
  r.d = pt_v3f(a.w, b.x, b.y);
  r.thr = pt_v3f(b.z, b.w, c.x);
  r.pixel = __float_as_uint(c.y);
  r.ctr = __float_as_uint(c.z);
  r.meta = __float_as_uint(c.w);
  return r;
}

__device__ __forceinline__ void accum_add(float* __restrict__ accum, uint32_t pixel, pt_v3 v) {
  float* p = accum + 3 * (size_t)pixel;
  p[0] += v.x;
  p[1] += v.y;
  p[2] += v.z;
}

// generate_camera_rays, kernels.py:1219-1239 (direction left unnormalized, Q1).
__device__ __forceinline__ Ray camera_ray(const DevFrame& fr, uint32_t pixel, int32_t s_begin, int32_t srel) {
  int32_t py = (int32_t)(pixel / (uint32_t)fr.width);
  int32_t px = (int32_t)(pixel - (uint32_t)py * (uint32_t)fr.width);
  Rng rng{pt_path_key(fr.seed, pixel, (uint32_t)(s_begin + srel)), 0u};
  Ray r;
  get_ray(fr, px, py, rng, r.o, r.d);
  r.thr = pt_v3f(1.0f, 1.0f, 1.0f);
  r.pixel = pixel;
  r.ctr = rng.n;
  r.meta = pack_meta(0, 0, srel);
  return r;
}

__global__ __launch_bounds__(kBlock) void wf_generate(DevFrame fr, WfBufs wb, int32_t s_begin) {
  const int32_t npix = fr.w * fr.n_rows;
  for (int32_t i = (int32_t)(blockIdx.x * kBlock + threadIdx.x); i < npix; i += (int32_t)(gridDim.x * kBlock)) {
    int32_t lr = i / fr.w;
    int32_t px = fr.x0 + (i - lr * fr.w);
    int32_t py = frame_row(fr, lr);
    store_ray(wb.q[0], i, camera_ray(fr, (uint32_t)(py * fr.width + px), s_begin, 0));
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
    wb.counts[cur ^ 1] = 0;  // next queue: last read by the previous iteration's kernels
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
    wb.hit[i] = make_float2(t, __int_as_float(hit ? ref : kMissRef));
  }
}

// Continuation of a ray after shading (kernels.py:1377-1399 + the per-path
// wave budget of renderer.py:313), or regeneration of the pixel's next
// sample when the path ends.
struct Next {
  bool enqueue;
  bool ended;
  Ray ray;
};

__device__ __forceinline__ void continue_or_regen(const DevFrame& fr, int32_t s_begin, int32_t s_count, bool go,
                                                  const Ray& cont, const Ray& cur, Next& nx) {
  const int32_t wave = (int32_t)((cur.meta >> 8) & 0xffu);
  const int32_t srel = (int32_t)(cur.meta >> 16);
  nx.enqueue = false;
  nx.ended = false;
  if (go && wave + 1 < fr.max_depth) {  // waves beyond max_depth are dropped (Q14)
    nx.enqueue = true;
    nx.ray = cont;
    return;
  }
  nx.ended = true;
  if (srel + 1 < s_count) {
    nx.enqueue = true;
    nx.ray = camera_ray(fr, cur.pixel, s_begin, srel + 1);
  }
}

// scatter epilogue of shade_and_scatter (kernels.py:1377-1391).
__device__ __forceinline__ bool scatter_epilogue(const DevFrame& fr, bool scattered, pt_v3 hp, pt_v3 sdir, pt_v3 att,
                                                 const Ray& cur, Rng& r, Ray& out) {
  if (!scattered) return false;
  pt_v3 nthr = pt_mul(cur.thr, att);
  int32_t nd = (int32_t)(cur.meta & 0xffu) + 1;
  if (nd >= fr.max_depth) return false;
  if (nd >= kRRMinDepth) {
    float sp = pt_minf(pt_maxf(pt_maxf(nthr.x, nthr.y), nthr.z), kRRMaxProb);
    if (r.next() > sp) return false;
    nthr = pt_divs(nthr, sp);
  }
  int32_t wave = (int32_t)((cur.meta >> 8) & 0xffu);
  out.o = hp;
  out.d = sdir;
  out.thr = nthr;
  out.pixel = cur.pixel;
  out.ctr = r.n;
  out.meta = pack_meta(nd, wave + 1, (int32_t)(cur.meta >> 16));
  return true;
}

// shade_miss_rays + shade_and_scatter for non-medium hits (kernels.py:1266-1399);
// medium-boundary hits are compacted into the medium queue.
__global__ __launch_bounds__(kBlock) void wf_shade(DevScene sc, DevFrame fr, WfBufs wb, int32_t cur,
                                                   int32_t s_begin, int32_t s_count, float* __restrict__ accum,
                                                   unsigned long long* __restrict__ counters) {
  const int32_t n = wb.counts[cur];
  const Queue q = wb.q[cur];
  const Queue qo = wb.q[cur ^ 1];
  const pt_v3 bg = pt_v3f(fr.bg[0], fr.bg[1], fr.bg[2]);
  const int32_t stride = (int32_t)(gridDim.x * kBlock);
  for (int32_t base = (int32_t)(blockIdx.x * kBlock); base < n; base += stride) {
    const int32_t i = base + (int32_t)threadIdx.x;
    bool to_medium = false;
    Next nx;
    nx.enqueue = false;
    nx.ended = false;
    if (i < n) {
      const float2 h = wb.hit[i];
      const int32_t ref = __float_as_int(h.y);
      const Ray ray = load_ray(q, i);
      Ray cont;
      bool go = false;
      if (ref == kMissRef) {
        accum_add(accum, ray.pixel, pt_mul(ray.thr, bg));  // shade_miss_rays :1280
      } else {
        const int32_t g = mat_index(sc, ref);
        if ((mat_flags(sc, g) >> 8) & 1u) {
          to_medium = true;
        } else {
          Rng r{pt_path_key(fr.seed, ray.pixel, (uint32_t)(s_begin + (int32_t)(ray.meta >> 16))), ray.ctr};
          const Mat m = load_mat(sc, g);
          pt_v3 hp = pt_add(ray.o, pt_scale(ray.d, h.x));
          pt_v3 nrm = hit_normal(sc, ref, hp, ray.d);
          pt_v3 emit = emitted(m);
          pt_v3 sdir, att;
          bool sc_ok = scatter(sc, ref, m, ray.d, hp, nrm, r, sdir, att);
          if (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) accum_add(accum, ray.pixel, pt_mul(ray.thr, emit));
          go = scatter_epilogue(fr, sc_ok, hp, sdir, att, ray, r, cont);
        }
      }
      if (!to_medium) continue_or_regen(fr, s_begin, s_count, go, cont, ray, nx);
    }
    wave_count(nx.ended, counters ? counters + 2 : nullptr);
    const int32_t mslot = wave_append(to_medium, wb.counts + 2);
    if (to_medium) wb.medq[mslot] = i;
    const int32_t slot = wave_append(nx.enqueue, wb.counts + (cur ^ 1));
    if (nx.enqueue) store_ray(qo, slot, nx.ray);
  }
}

// Constant-medium rays: exit traversal + free flight (apply_constant_medium,
// kernels.py:365-450) and the volume branch of shade_and_scatter
// (kernels.py:1326-1357).
template <int STACK>
__global__ __launch_bounds__(kBlock) void wf_medium(DevScene sc, DevFrame fr, WfBufs wb, int32_t cur,
                                                    int32_t s_begin, int32_t s_count, float* __restrict__ accum,
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
    Next nx;
    nx.enqueue = false;
    nx.ended = false;
    if (j < n) {
      const int32_t i = wb.medq[j];
      const float2 h = wb.hit[i];
      const int32_t ref = __float_as_int(h.y);
      const Ray ray = load_ray(q, i);
      const float t_entry = h.x;
      float te;
      int32_t rex;
      const bool hx = traverse<STACK>(sc, ray.o, ray.d, t_entry + 0.0001f, kTMax, st, te, rex);
      const Mat m = load_mat(sc, mat_index(sc, ref));
      Rng r{pt_path_key(fr.seed, ray.pixel, (uint32_t)(s_begin + (int32_t)(ray.meta >> 16))), ray.ctr};
      float t_exit;
      pt_v3 mp;
      Ray cont;
      bool go;
      if (medium_step(hx, te, t_entry, m.m3.w, ray.o, ray.d, r, mp, t_exit)) {
        pt_v3 sdir = random_unit_vector(r);
        go = scatter_epilogue(fr, true, mp, sdir, pt_v3f(m.m4.x, m.m4.y, m.m4.z), ray, r, cont);
      } else if (t_exit > 0.0f) {  // passthrough: same depth, next wave (kernels.py:1342-1350)
        float eps_t = 0.001f / sqrtf(pt_dot(ray.d, ray.d));
        cont = ray;
        cont.o = pt_add(ray.o, pt_scale(ray.d, t_exit + eps_t));
        cont.ctr = r.n;
        cont.meta = ray.meta + (1u << 8);
        go = true;
      } else {  // fallback (kernels.py:1352-1357)
        pt_v3 hp = pt_add(ray.o, pt_scale(ray.d, t_entry));
        pt_v3 nrm = hit_normal(sc, ref, hp, ray.d);
        pt_v3 emit = emitted(m);
        pt_v3 sdir, att;
        bool sc_ok = scatter(sc, ref, m, ray.d, hp, nrm, r, sdir, att);
        if (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) accum_add(accum, ray.pixel, pt_mul(ray.thr, emit));
        go = scatter_epilogue(fr, sc_ok, hp, sdir, att, ray, r, cont);
      }
      continue_or_regen(fr, s_begin, s_count, go, cont, ray, nx);
    }
    wave_count(nx.ended, counters ? counters + 2 : nullptr);
    const int32_t slot = wave_append(nx.enqueue, wb.counts + (cur ^ 1));
    if (nx.enqueue) store_ray(qo, slot, nx.ray);
  }
}

static inline unsigned grid_for(int32_t n) {
  int64_t b = ((int64_t)n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (unsigned)b;
}

namespace {
int32_t* g_pinned_count = nullptr;  // host-pinned readback slot for the live-ray count
}

template <int STACK>
static hipError_t wf_run(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, float* accum, int32_t s_begin,
                         int32_t s_count, unsigned long long* counters, hipStream_t stream) {
  const int32_t npix = fr.w * fr.n_rows;
  const unsigned g = grid_for(npix);
  if (!g_pinned_count) {
    hipError_t e = hipHostMalloc((void**)&g_pinned_count, sizeof(int32_t), hipHostMallocDefault);
    if (e != hipSuccess) return e;
  }
  prof_begin(kProfWfGenerate, stream);
  hipLaunchKernelGGL(wf_generate, dim3(g), dim3(kBlock), 0, stream, fr, wb, s_begin);
  prof_end(kProfWfGenerate, stream);
  // Every path lives at most max_depth waves and a pixel's samples run back
  // to back, so s_count * max_depth iterations drain every queue.
  const int64_t max_iters = (int64_t)s_count * (int64_t)(fr.max_depth > 0 ? fr.max_depth : 1) + 1;
  int32_t cur = 0;
  int64_t it = 0;
  int32_t chunk = 4;
  while (it < max_iters) {
    int64_t n = max_iters - it < chunk ? max_iters - it : chunk;
    for (int64_t j = 0; j < n; ++j) {
      prof_begin(kProfWfIntersect, stream);
      hipLaunchKernelGGL(wf_intersect<STACK>, dim3(g), dim3(kBlock), 0, stream, sc, wb, cur, counters);
      prof_end(kProfWfIntersect, stream);
      prof_begin(kProfWfShade, stream);
      hipLaunchKernelGGL(wf_shade, dim3(g), dim3(kBlock), 0, stream, sc, fr, wb, cur, s_begin, s_count, accum,
                         counters);
      prof_end(kProfWfShade, stream);
      prof_begin(kProfWfMedium, stream);
      hipLaunchKernelGGL(wf_medium<STACK>, dim3(g), dim3(kBlock), 0, stream, sc, fr, wb, cur, s_begin, s_count,
                         accum, counters);
      prof_end(kProfWfMedium, stream);
      cur ^= 1;
    }
    it += n;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // live-ray count of the queue the next iteration would consume
    e = hipMemcpyAsync(g_pinned_count, wb.counts + cur, sizeof(int32_t), hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return e;
    if (*g_pinned_count == 0) break;
    if (chunk < 16) chunk *= 2;
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
  // sample index relative to the call's first travels in 16 bits of meta
  for (int32_t b = 0; b < s_count; b += 65535) {
    int32_t c = s_count - b < 65535 ? s_count - b : 65535;
    hipError_t e;
    if (stack_needed <= 16) e = wf_run<16>(sc, fr, wb, accum, s_begin + b, c, counters, stream);
    else if (stack_needed <= 24) e = wf_run<24>(sc, fr, wb, accum, s_begin + b, c, counters, stream);
    else if (stack_needed <= 32) e = wf_run<32>(sc, fr, wb, accum, s_begin + b, c, counters, stream);
    else e = wf_run<64>(sc, fr, wb, accum, s_begin + b, c, counters, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ptmi
