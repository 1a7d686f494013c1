// pt_wavefront.hip — breadth-first (wavefront) integrator for gfx950.
//
// Replaces the wavefront stage kernels of kernels.py:1219-1418 as driven by
// TaichiRenderer.render_wavefront (renderer.py:305-334). Stages and layout
// are designed for CDNA4, not translated:
//   * ray queue = three float4 streams per slot (A = o.xyz,d.x;
//     B = d.yz,thr.xy; C = thr.z, work item, rng draw counter, meta) so every
//     load/store is a 16-B-per-lane coalesced access; meta = depth | wave << 8;
//   * hit record = 8 B (t, leaf ref); hit point and normal are recomputed in
//     the shading kernel with the reference's own expressions;
//   * rays whose closest hit is a constant-medium boundary are compacted into
//     a separate medium queue and get their exit traversal (kernels.py:417)
//     from a dedicated kernel instead of diverging inside shading;
//   * WORK POOL, IN-PLACE SLOTS: the reference pushes one sample of every
//     pixel through max_depth bounce-synchronous waves (renderer.py:305-334)
//     and compacts survivors into a next queue with one atomic per ray, so
//     after a few bounces its queues are nearly empty. Here the (sample,
//     pixel) pairs of a batch are work items: a queue slot keeps its ray in
//     place from bounce to bounce (no append, no swap copy: kernels.py:
//     1402-1418 removed) and, when the path ends, waits for the next
//     wf_intersect, which hands it the camera ray of the next work item — so
//     every launch works on a full queue until the batch runs out.
//   * Work is handed out per 64-slot group (one wave): a group draws 64-item
//     units (one 8x8 pixel square x one sample) in chunks of a few samples of
//     the same square, so a wave's rays stay coherent. Unit counters are
//     sharded 8 ways by slot block (blocks b and b+8 share an XCD), one
//     atomic per chunk, each counter on its own 256-B line, because a single
//     device-wide counter saturates near 88 returning atomics/us on MI355X
//     (MI355X_MICROARCH.md, "dequeue") and was measured at 97 % wait cycles.
//   * PIPES: the queue is split into 4 independent parts, each looping
//     intersect -> shade -> medium on its own stream, so the drain at the end
//     of one pipe's launch is filled by another's (+21 % over one pipe).
//   * The host learns that a pipe has drained from a 4-byte live count read
//     back every 8 iterations, and waits for chunk k's counts only after
//     chunk k + 1 is queued, so no pipe idles through the host round trip
//     (the reference reads its ray count back every bounce, renderer.py:315).
//   * Each ray carries its own wave count and is dropped at max_depth waves,
//     exactly the reference's per-path budget (Q14, incl. passthrough Q11).
//   * A path adds at most one colour to its pixel, when it ends (a miss, or an
//     emissive hit, which never scatters: kernels.py:1266-1280, 1365-1375,
//     906), so each path writes that colour (or 0) to a staging slot
//     [sample][pixel]; a resolve kernel then adds the slots into the
//     accumulator in sample order — the same float additions, in the same
//     order, as the reference's per-sample accumulation, with no atomics and
//     no ordering constraint between concurrent paths of one pixel.
#include "pt_launch.hpp"
#include "pt_prof.hpp"

#include <mutex>

namespace ptmi {

constexpr int kShards = 8;
#ifndef PTMI_WF_CHUNK_SAMPLES
#define PTMI_WF_CHUNK_SAMPLES 4  // samples per work chunk (one 8x8 pixel square each)
#endif
#ifndef PTMI_WF_TAIL
#define PTMI_WF_TAIL 2  // a shard hands out single units once it has < TAIL chunks per group left
#endif
#ifndef PTMI_WF_BLOCK
#define PTMI_WF_BLOCK 128  // threads per block of the queue kernels (A/B on MI355X, parity-identical: 128 vs 256
                           // C3 +1.2 %, mesh fog +1.7 %; 64: C3 -6 %, mesh fog +2.3 %; profiles/r02/ab/ab_wf_block.log)
#endif
constexpr int kWfBlock = PTMI_WF_BLOCK;
constexpr uint32_t kDead = 0xffffffffu;     // item of a retired slot
constexpr uint32_t kPending = 0xfffffffeu;  // item of a slot waiting for work (assigned in wf_intersect)

struct Queue {
  float4* a;  // o.xyz, d.x
  float4* b;  // d.y, d.z, thr.x, thr.y
  float4* c;  // thr.z, item, rng counter, meta (bits)
};

struct WfBufs {
  Queue q;
  float2* hit;        // t, ref (bits); ref kMissRef = miss
  int32_t* medq;      // kShards segments of medseg slot indices
  float* staging;     // [batch][npix][3] path colours
  int32_t* ctl;       // this pipe's counters, one per 256-B line (see ctl_*)
  int32_t* next;      // next-unit counters shared by the pipes, one per 256-B line
  int32_t capacity;   // queue slots (multiple of kShards * kWfBlock)
  int32_t medseg;     // slots per shard
  int2* grp;          // per 64-slot group (one wave in wf_intersect): {next item, end} of its fetched units
  int32_t npix;       // pixels of the frame's pixel set
  int32_t sq_x, nsq;  // 8x8 pixel squares covering the pixel set: per row, total
  int32_t csamp;      // samples per chunk: a chunk is one square x csamp samples (64 * csamp items)
  int32_t batch;      // samples of the batch
  int32_t nunits;     // 64-item units of the batch (one square x one sample; csamp per chunk)
  int32_t shard_len;  // units per shard (a multiple of csamp): shard s owns [s*len, min((s+1)*len, nunits))
  int32_t shard_groups; // 64-slot groups drawing from each shard
  int32_t s_begin;    // first sample of the batch
};

constexpr int32_t kMissRef = 0x7fffffff;

// Pipes: the queue is split into PTMI_WF_PIPES independent halves, each
// driven through its own intersect/shade/medium loop on its own stream, so
// one pipe's kernels fill the drain at the end of the other's. They share the
// work pool (next-unit counters) and the staging buffer.
#ifndef PTMI_WF_PIPES
#define PTMI_WF_PIPES 4  // A/B on MI355X: 1 -> 2 pipes +15 % (C3), 2 -> 4 +5 %
#endif
constexpr int32_t kPipes = PTMI_WF_PIPES;

// Device-scope atomics are performed per cache line at the memory side, so
// counters sharing a line serialize as one: every counter gets its own
// 256-B line. Lines 0-7: next unit per shard (shared); then per pipe 17 lines:
// medium-queue count per shard, live slots (read by the host), deferred-
// shading count per shard.
constexpr int32_t kLine = 64;
constexpr int32_t kPipeLines = 17;
constexpr int32_t kCtlWords = (8 + kPipeLines * kPipes) * kLine;
__host__ __device__ __forceinline__ int32_t* ctl_medium(const WfBufs& wb, int32_t s) { return wb.ctl + s * kLine; }
__host__ __device__ __forceinline__ int32_t* ctl_next(const WfBufs& wb, int32_t s) { return wb.next + s * kLine; }
__host__ __device__ __forceinline__ int32_t* ctl_live(const WfBufs& wb) { return wb.ctl + 8 * kLine; }
// deferred-shading (Perlin-textured surface hits) count per shard: lines 9-16
__host__ __device__ __forceinline__ int32_t* ctl_noise(const WfBufs& wb, int32_t s) { return wb.ctl + (9 + s) * kLine; }

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Slot i is processed by block (i / kWfBlock) % grid, grid a multiple of
// kShards, so block b's slots draw chunks from shard b % kShards (blocks b and
// b + 8 share an XCD). A 64-slot group is always one wave of wf_intersect.
__device__ __forceinline__ int32_t slot_shard(int32_t i) { return (i / kWfBlock) % kShards; }

// Wave-aggregated counter increment: this lane's ticket (meaningful only if want).
__device__ __forceinline__ int32_t wave_ticket(bool want, int32_t* counter) {
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

__device__ __forceinline__ void wave_add(bool flag, int32_t* counter, int32_t sign) {
  unsigned long long mask = __ballot(flag);
  if (mask && lane_id() == __ffsll((long long)mask) - 1) atomicAdd(counter, sign * (int32_t)__popcll(mask));
}

// Statistics counters: each thread tallies in a register over its grid-stride
// loop; at kernel end the block sums through LDS and adds once. `scratch` may
// alias LDS the kernel used before (the traversal stack): no extra LDS, which
// would push a 32 KiB-stack block past 160 KiB / 5 and cost a wave per SIMD.
template <int N>
__device__ __forceinline__ void block_flush(const uint32_t (&vals)[N], void* scratch, unsigned long long* counter) {
  unsigned int* lds = static_cast<unsigned int*>(scratch);
  uint32_t v[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    v[k] = vals[k];
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
  }
  __syncthreads();
  if (threadIdx.x < N) lds[threadIdx.x] = 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (lane_id() == 0 && v[k]) atomicAdd(lds + k, v[k]);
  __syncthreads();
  if (threadIdx.x < N && lds[threadIdx.x]) atomicAdd(counter + threadIdx.x, (unsigned long long)lds[threadIdx.x]);
}

struct Ray {
  pt_v3 o, d, thr;
  uint32_t item, ctr, meta;
};

// Streamed buffers (queue records, hit records, medium lists, staging) go
// through these helpers. PMC: wf_intersect's L2 hit rate is 60 % against the
// megakernel's 96 % (L1 hit rates 96 % / 98 %), the queue stream evicting BVH
// lines. But the stage kernels re-read what the previous one wrote, and that
// reuse is worth more than streaming hints: A/B on MI355X (parity-identical),
// `nt` loads + stores / `nt` stores / `sc1` stores, C3 -10 % / -5 % / -5 %
// (profiles/r02/ab/ab_nontemporal.log, profiles/r02/pmc_cache/).
typedef float pt_qf4 __attribute__((ext_vector_type(4)));
typedef float pt_qf2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ T s_load(const T* p) {
  return *p;
}
template <typename T>
__device__ __forceinline__ void s_store(T* p, T v) {
  *p = v;
}
__device__ __forceinline__ float4 q_load(const float4* p) {
  const pt_qf4 v = s_load((const pt_qf4*)p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void q_store(float4* p, float4 v) { s_store((pt_qf4*)p, pt_qf4{v.x, v.y, v.z, v.w}); }
__device__ __forceinline__ float2 h_load(const float2* p) {
  const pt_qf2 v = s_load((const pt_qf2*)p);
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ void h_store(float2* p, float2 v) { s_store((pt_qf2*)p, pt_qf2{v.x, v.y}); }

__device__ __forceinline__ void store_ray(const Queue& q, int32_t i, const Ray& r) {
  q_store(q.a + i, make_float4(r.o.x, r.o.y, r.o.z, r.d.x));
  q_store(q.b + i, make_float4(r.d.y, r.d.z, r.thr.x, r.thr.y));
  q_store(q.c + i, make_float4(r.thr.z, __uint_as_float(r.item), __uint_as_float(r.ctr), __uint_as_float(r.meta)));
}

__device__ __forceinline__ void kill_slot(const Queue& q, int32_t i) {
  s_store(reinterpret_cast<uint32_t*>(q.c + i) + 1, kDead);
}

__device__ __forceinline__ uint32_t slot_item(const Queue& q, int32_t i) {
  return s_load(reinterpret_cast<const uint32_t*>(q.c + i) + 1);
}

__device__ __forceinline__ Ray load_ray(const Queue& q, int32_t i) {
  float4 a = q_load(q.a + i), b = q_load(q.b + i), c = q_load(q.c + i);
  Ray r;
  r.o = pt_v3f(a.x, a.y, a.z);
  r.d = pt_v3f(a.w, b.x, b.y);
  r.thr = pt_v3f(b.z, b.w, c.x);
  r.item = __float_as_uint(c.y);
  r.ctr = __float_as_uint(c.z);
  r.meta = __float_as_uint(c.w);
  return r;
}

// Work items come in chunks of one 8x8 pixel square x csamp samples. Chunk c
// is square c % nsq of sample block c / nsq (so early chunks cover every
// square); item j of a chunk is pixel j % 64 of the square, sample j / 64 of
// the block. Each 64-slot group works through one chunk at a time, so a
// wave's rays come from one pixel square — the coherence the megakernel's
// waves get from their 8x8 squares. Items outside the frame or past the
// batch are skipped. it.p is the row-major pixel index (staging).
struct Item {
  int32_t srel, p, px, py;
  bool valid;
};
__device__ __forceinline__ Item decode_item(const DevFrame& fr, const WfBufs& wb, uint32_t k) {
  Item it;
  const uint32_t per = 64u * (uint32_t)wb.csamp;
  const uint32_t c = k / per, j = k - c * per;
  const uint32_t blk = c / (uint32_t)wb.nsq, q = c - blk * (uint32_t)wb.nsq;
  const int32_t qy = (int32_t)(q / (uint32_t)wb.sq_x), qx = (int32_t)q - qy * wb.sq_x;
  const int32_t lx = qx * 8 + (int32_t)(j & 7u), lr = qy * 8 + (int32_t)((j >> 3) & 7u);
  it.srel = (int32_t)blk * wb.csamp + (int32_t)(j >> 6);
  it.valid = lx < fr.w && lr < fr.n_rows && it.srel < wb.batch;
  it.p = lr * fr.w + lx;
  it.px = fr.x0 + lx;
  it.py = it.valid ? frame_row(fr, lr) : 0;
  return it;
}

__device__ __forceinline__ uint32_t path_key(const DevFrame& fr, const WfBufs& wb, const Item& it) {
  return pt_path_key(fr.seed, (uint32_t)(it.py * fr.width + it.px), (uint32_t)(wb.s_begin + it.srel));
}

// generate_camera_rays, kernels.py:1219-1239 (direction left unnormalized, Q1).
__device__ __forceinline__ Ray camera_ray(const DevFrame& fr, const WfBufs& wb, uint32_t k) {
  Item it = decode_item(fr, wb, k);
  Rng rng{path_key(fr, wb, it), 0u};
  Ray r;
  get_ray(fr, it.px, it.py, rng, r.o, r.d);
  r.thr = pt_v3f(1.0f, 1.0f, 1.0f);
  r.item = k;
  r.ctr = rng.n;
  r.meta = 0u;
  return r;
}

__device__ __forceinline__ void stage(const DevFrame& fr, const WfBufs& wb, uint32_t k, pt_v3 c) {
  const Item it = decode_item(fr, wb, k);
  float* p = wb.staging + 3 * ((size_t)it.srel * (size_t)wb.npix + (size_t)it.p);
  s_store(p, c.x);
  s_store(p + 1, c.y);
  s_store(p + 2, c.z);
}

__device__ __forceinline__ int32_t shard_end(const WfBufs& wb, int32_t s) {
  int64_t e = (int64_t)(s + 1) * wb.shard_len;
  return e < wb.nunits ? (int32_t)e : wb.nunits;
}

// Next units for a group of shard `shard` (one lane calls it), stealing from
// the other shards once its own range is spent: {first, end} unit, or
// first = -1 when the batch is done. A whole chunk (csamp units of one
// square) while the shard has plenty left; single units in its tail, so no
// group is left with a long private queue while the others retire.
__device__ __forceinline__ int2 fetch_units(const WfBufs& wb, int32_t shard) {
  for (int32_t a = 0; a < kShards; ++a) {
    const int32_t s = (shard + a) % kShards;
    const int32_t e = shard_end(wb, s);
    const int32_t cur = __hip_atomic_load(ctl_next(wb, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur >= e) continue;
    const int32_t take = (e - cur) >= PTMI_WF_TAIL * wb.shard_groups * wb.csamp ? wb.csamp : 1;
    const int32_t t = atomicAdd(ctl_next(wb, s), take);
    if (t < e) return make_int2(t, t + take < e ? t + take : e);
  }
  return make_int2(-1, -1);
}

// Initial state: every slot waits for work; groups own no units yet; shard s
// starts at its first unit.
__global__ __launch_bounds__(kWfBlock) void wf_generate(DevFrame fr, WfBufs wb, int32_t init_next) {
  for (int32_t i = (int32_t)(blockIdx.x * kWfBlock + threadIdx.x); i < wb.capacity; i += (int32_t)(gridDim.x * kWfBlock)) {
    reinterpret_cast<uint32_t*>(wb.q.c + i)[1] = kPending;
    if ((i & 63) == 0) wb.grp[i >> 6] = make_int2(0, 0);
  }
  if (init_next && blockIdx.x < kShards && threadIdx.x == 0) {
    const int32_t s = (int32_t)blockIdx.x;
    *ctl_next(wb, s) = min(s * wb.shard_len, wb.nunits);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctl_live(wb) = wb.capacity;
}

// Hand the group's (this wave's) next items to its slots waiting for work,
// taking a new chunk when the current one runs out; slots that find no work
// retire. Wave-uniform: called by all 64 lanes of the group.
__device__ __forceinline__ void assign_work(const DevFrame& fr, const WfBufs& wb, int32_t i, uint32_t& item) {
  const bool pending = item == kPending;
  const unsigned long long pm = __ballot(pending);
  if (pm == 0ull) return;
  const int32_t g = i >> 6;
  const uint32_t n = (uint32_t)__popcll(pm);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
  const int2 gs = wb.grp[g];
  uint32_t nxt = (uint32_t)gs.x, end = (uint32_t)gs.y;
  const uint32_t avail = end - nxt;
  uint32_t my = kDead;
  if (rank < avail) my = nxt + rank;
  if (n > avail) {  // the group needs new units (>= 64 items: one fetch is enough)
    int2 u = make_int2(0, 0);
    const int32_t leader = __ffsll((long long)pm) - 1;
    if (lane_id() == leader) u = fetch_units(wb, slot_shard(i));
    u.x = __shfl(u.x, leader);
    u.y = __shfl(u.y, leader);
    if (u.x >= 0) {
      const uint32_t cb = 64u * (uint32_t)u.x;
      if (rank >= avail) my = cb + (rank - avail);
      nxt = cb + (n - avail);
      end = 64u * (uint32_t)u.y;
    } else {
      nxt = end;
    }
  } else {
    nxt += n;
  }
  if (lane_id() == 0) wb.grp[g] = make_int2((int32_t)nxt, (int32_t)end);
  if (pending) {
    if (my == kDead) {
      kill_slot(wb.q, i);
      item = kDead;
    } else if (decode_item(fr, wb, my).valid) {
      store_ray(wb.q, i, camera_ray(fr, wb, my));
      item = my;
    }  // an item outside the frame / batch: the slot stays pending
  }
  wave_add(pending && my == kDead, ctl_live(wb), -1);
}

// intersect_rays, kernels.py:1242-1263.
template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock) void wf_intersect(DevScene sc, DevFrame fr, WfBufs wb,
                                                       unsigned long long* __restrict__ counters) {
  __shared__ uint2 lds_stack[STACK * kWfBlock];
  const int tid = threadIdx.x;
  Stack st{lds_stack + tid};
  if (blockIdx.x < kShards && tid == 0) {  // medium and deferred-shading counts of this iteration
    *ctl_medium(wb, blockIdx.x) = 0;
    *ctl_noise(wb, blockIdx.x) = 0;
  }
  const Queue q = wb.q;
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  uint32_t n_live = 0;
  for (int32_t i = (int32_t)(blockIdx.x * kWfBlock + tid); i < wb.capacity; i += stride) {
    uint32_t item = slot_item(q, i);
    assign_work(fr, wb, i, item);  // generate_camera_rays (kernels.py:1219-1239) for slots that need work
    if (item >= kPending) continue;
    ++n_live;
    float4 a = q_load(q.a + i), b = q_load(q.b + i);
    pt_v3 o = pt_v3f(a.x, a.y, a.z), d = pt_v3f(a.w, b.x, b.y);
    float t;
    int32_t ref;
    bool hit = traverse<STACK, kWfBlock, TRAV>(sc, o, d, kTMin, kTMax, st, t, ref);
    h_store(wb.hit + i, make_float2(t, __int_as_float(hit ? ref : kMissRef)));
  }
  if (counters) block_flush<1>({n_live}, lds_stack, counters + 0);
}

// scatter epilogue of shade_and_scatter (kernels.py:1377-1399) plus the
// per-path wave budget of renderer.py:313. A path it ends is counted in
// ends[0] (Russian roulette) or ends[1] (depth or wave budget).
__device__ __forceinline__ bool scatter_epilogue(const DevFrame& fr, bool scattered, pt_v3 hp, pt_v3 sdir, pt_v3 att,
                                                 const Ray& cur, Rng& r, Ray& out, uint32_t (&ends)[2]) {
  if (!scattered) return false;
  pt_v3 nthr = pt_mul(cur.thr, att);
  int32_t nd = (int32_t)(cur.meta & 0xffu) + 1;
  if (nd >= fr.max_depth) {
    ++ends[1];
    return false;
  }
  if (nd >= kRRMinDepth) {
    float sp = pt_minf(pt_maxf(pt_maxf(nthr.x, nthr.y), nthr.z), kRRMaxProb);
    if (r.next() > sp) {
      ++ends[0];
      return false;
    }
    nthr = pt_divs(nthr, sp);
  }
  int32_t wave = (int32_t)((cur.meta >> 8) & 0xffu);
  if (wave + 1 >= fr.max_depth) {  // Q14: no wave left for the continuation
    ++ends[1];
    return false;
  }
  out.o = hp;
  out.d = sdir;
  out.thr = nthr;
  out.item = cur.item;
  out.ctr = r.n;
  out.meta = (uint32_t)nd | ((uint32_t)(wave + 1) << 8);
  return true;
}

// One scatter site and one random_unit_vector site per shading kernel
// (scatter_begin / scatter_end, pt_device.hpp): wf_medium's deferred
// Perlin-textured surfaces, boundary fallbacks and medium scatters share them,
// so each divergent piece (material scatter, rejection loop) runs once per
// wave. A/B on MI355X against separate sites, parity-identical: C3 +0.8 %,
// mesh fog +0.6 % (profiles/r02/ab/ab_one_scatter.log).

// Per-lane tail of both shading kernels: keep a continuing ray in its slot,
// or mark the slot of an ended path as waiting for work (the next
// wf_intersect hands it the next item of its group's chunk).
__device__ __forceinline__ void finish_lane(const WfBufs& wb, int32_t i, bool ended, bool go, const Ray& cont) {
  if (go) store_ray(wb.q, i, cont);
  if (ended) s_store(reinterpret_cast<uint32_t*>(wb.q.c + i) + 1, kPending);
}

// Surface branch of shade_and_scatter (kernels.py:1359-1399) for slot ray
// `ray` whose closest hit (t, ref) has material g.
__device__ __forceinline__ void shade_surface(const DevScene& sc, const DevFrame& fr, const WfBufs& wb,
                                              const Ray& ray, float t, int32_t ref, int32_t g, bool& ended,
                                              bool& go, Ray& cont, uint32_t (&ends)[2]) {
  Item it = decode_item(fr, wb, ray.item);
  Rng r{path_key(fr, wb, it), ray.ctr};
  const Mat m = load_mat(sc, g);
  pt_v3 hp = pt_add(ray.o, pt_scale(ray.d, t));
  pt_v3 nrm = hit_normal(sc, ref, hp, ray.d);
  pt_v3 emit = emitted(m);
  pt_v3 sdir, att;
  bool sc_ok;  // one unit-vector site for metal and isotropic lanes
  const int32_t ruv = scatter_begin(sc, ref, m, ray.d, hp, nrm, r, sdir, att, sc_ok);
  if (ruv != kRuvNone) sc_ok = scatter_end(sc, ruv, ref, m, hp, nrm, random_unit_vector(r), sdir, att);
  go = scatter_epilogue(fr, sc_ok, hp, sdir, att, ray, r, cont, ends);
  if (!go) {
    ended = true;  // an emissive hit is the path's only contribution (:1368-1375)
    stage(fr, wb, ray.item, (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) ? pt_mul(ray.thr, emit)
                                                                          : pt_v3f(0.0f, 0.0f, 0.0f));
  }
}

// Surface hits whose scatter evaluates Perlin turbulence (a noise texture on
// a Lambertian or isotropic material, kernels.py:1013-1015): deferred to a
// compacted list shaded by wf_medium, so one such lane no longer puts three
// octaves of table round trips into every wave of wf_shade that holds it.
__device__ __forceinline__ bool noise_shaded(uint32_t flags) {
  const uint32_t mt = flags & 0xfu, tx = (flags >> 4) & 0xfu;
  return tx == 3u && (mt == 0u || mt == 4u);
}

// A/B, not kept: wf_shade writing its block's continuing rays back sorted by
// direction octant (a ray record is self-contained, so its slot is free to
// change): -8 % C3 and mesh fog. A wave's rays come from one pixel square, and
// that origin coherence is worth more than the direction coherence the sort
// buys (profiles/r02/ab/ab_wf_octant_sort.log).

// shade_miss_rays + shade_and_scatter for non-medium hits (kernels.py:1266-1399);
// medium-boundary hits go to their shard's medium queue segment.
#ifndef PTMI_WF_SHADE_MIN_WAVES
#define PTMI_WF_SHADE_MIN_WAVES 5  // 96 VGPRs, no spills: A/B C3 +0.8 %; 6 waves (48 B spills) -2.7 % (profiles/r02/ab/ab_wf_occupancy.log)
#endif
__global__ __launch_bounds__(kWfBlock, PTMI_WF_SHADE_MIN_WAVES) void wf_shade(DevScene sc, DevFrame fr, WfBufs wb,
                                                   unsigned long long* __restrict__ counters) {
  const Queue q = wb.q;
  const pt_v3 bg = pt_v3f(fr.bg[0], fr.bg[1], fr.bg[2]);
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  const int32_t shard = (int32_t)(blockIdx.x % kShards);
  __shared__ unsigned int tally[3];
  uint32_t n_ended = 0, ends[2] = {0u, 0u};
  for (int32_t base = (int32_t)(blockIdx.x * kWfBlock); base < wb.capacity; base += stride) {
    const int32_t i = base + (int32_t)threadIdx.x;
    bool to_medium = false, to_noise = false, ended = false, go = false;
    Ray cont;
    const bool live = i < wb.capacity && slot_item(q, i) < kPending;
    if (live) {
      const float2 h = h_load(wb.hit + i);
      const int32_t ref = __float_as_int(h.y);
      const Ray ray = load_ray(q, i);
      if (ref == kMissRef) {
        stage(fr, wb, ray.item, pt_mul(ray.thr, bg));  // shade_miss_rays :1280
        ended = true;
      } else {
        const int32_t g = mat_index(sc, ref);
        const uint32_t fl = mat_flags(sc, g);
        if ((fl >> 8) & 1u) {
          to_medium = true;
        } else if (noise_shaded(fl)) {
          to_noise = true;
        } else {
          shade_surface(sc, fr, wb, ray, h.x, ref, g, ended, go, cont, ends);
        }
      }
    }
    const int32_t mslot = wave_ticket(to_medium, ctl_medium(wb, shard));
    if (to_medium) s_store(wb.medq + shard * wb.medseg + mslot, i);
    // deferred hits fill the shard's segment from the top; a slot is in at
    // most one of the two lists, so together they never exceed the segment
    const int32_t nslot = wave_ticket(to_noise, ctl_noise(wb, shard));
    if (to_noise) s_store(wb.medq + shard * wb.medseg + wb.medseg - 1 - nslot, i);
    finish_lane(wb, i, ended, go, cont);
    n_ended += ended ? 1u : 0u;
  }
  if (counters) block_flush<3>({n_ended, ends[0], ends[1]}, tally, counters + 2);
}

// Constant-medium rays: exit traversal + free flight (apply_constant_medium,
// kernels.py:365-450) and the volume branch of shade_and_scatter
// (kernels.py:1326-1357). Work index j runs over the concatenated shard segments.
template <int STACK, int TRAV = PTMI_TRAV_STACK>
#ifndef PTMI_WF_MEDIUM_MIN_WAVES
#define PTMI_WF_MEDIUM_MIN_WAVES 4  // <= 128 VGPRs: with the deferred shading list it needs 131 otherwise (3 waves/SIMD)
#endif
__global__ __launch_bounds__(kWfBlock, PTMI_WF_MEDIUM_MIN_WAVES) void wf_medium(DevScene sc, DevFrame fr, WfBufs wb,
                                                    unsigned long long* __restrict__ counters) {
  __shared__ uint2 lds_stack[STACK * kWfBlock];
  Stack st{lds_stack + threadIdx.x};
  int32_t cnt[kShards];  // per-shard medium counts (wave-uniform)
  int32_t n = 0;
#pragma unroll
  for (int s = 0; s < kShards; ++s) {
    cnt[s] = __builtin_amdgcn_readfirstlane(*ctl_medium(wb, s));
    n += cnt[s];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && counters && n > 0) atomicAdd(counters + 1, (unsigned long long)n);
  int32_t nn = 0;  // deferred surface hits (wf_shade), after the medium rays in the index space
  int32_t cntn[kShards];
#pragma unroll
  for (int s = 0; s < kShards; ++s) {
    cntn[s] = __builtin_amdgcn_readfirstlane(*ctl_noise(wb, s));
    nn += cntn[s];
  }
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  uint32_t n_ended = 0, ends[2] = {0u, 0u};
  for (int32_t base = (int32_t)(blockIdx.x * kWfBlock); base < n + nn; base += stride) {
    const int32_t j = base + (int32_t)threadIdx.x;
    bool ended = false, go = false;
    Ray cont;
    int32_t i = -1, shard = 0;
    const bool is_noise = j >= n && j < n + nn;
    if (j < n) {  // medium-queue slot
      int32_t off = j;
#pragma unroll
      for (int s = 0; s + 1 < kShards; ++s) {
        if (shard == s && off >= cnt[s]) {
          off -= cnt[s];
          shard = s + 1;
        }
      }
      i = s_load(wb.medq + shard * wb.medseg + off);
    } else if (is_noise) {  // deferred surface slot (wf_shade), from the top of the segment
      int32_t off = j - n;
#pragma unroll
      for (int s = 0; s + 1 < kShards; ++s) {
        if (shard == s && off >= cntn[s]) {
          off -= cntn[s];
          shard = s + 1;
        }
      }
      i = s_load(wb.medq + shard * wb.medseg + wb.medseg - 1 - off);
    }
    if (i >= 0) {
      const float2 h = h_load(wb.hit + i);
      const int32_t ref = __float_as_int(h.y);
      const Ray ray = load_ray(wb.q, i);
      float te = 0.0f;
      int32_t rex = 0;
      bool hx = false;
      if (!is_noise)  // the exit search from t_entry + 1e-4 (kernels.py:417-419)
        hx = traverse<STACK, kWfBlock, TRAV>(sc, ray.o, ray.d, h.x + 0.0001f, kTMax, st, te, rex);
      const Mat m = load_mat(sc, mat_index(sc, ref));
      Item it = decode_item(fr, wb, ray.item);
      Rng r{path_key(fr, wb, it), ray.ctr};
      bool surface = is_noise, scattered = false, passthrough = false;
      int32_t ruv = kRuvNone;
      pt_v3 hp, nrm, sdir, att, emit = pt_v3f(0.0f, 0.0f, 0.0f);
      if (!is_noise) {
        float t_exit;
        pt_v3 mp;
        if (medium_step(hx, te, h.x, m.m3.w, ray.o, ray.d, r, mp, t_exit)) {
          hp = mp;
          att = pt_v3f(m.m4.x, m.m4.y, m.m4.z);
          ruv = kRuvMedium;
          scattered = true;
        } else if (t_exit > 0.0f) {  // passthrough: same depth, next wave (kernels.py:1342-1350)
          passthrough = true;
          int32_t wave = (int32_t)((ray.meta >> 8) & 0xffu);
          if (wave + 1 >= fr.max_depth) {
            ++ends[1];  // Q14: no wave left for the passthrough
          } else {
            float eps_t = 0.001f / sqrtf(pt_dot(ray.d, ray.d));
            cont = ray;
            cont.o = pt_add(ray.o, pt_scale(ray.d, t_exit + eps_t));
            cont.ctr = r.n;
            cont.meta = ray.meta + (1u << 8);
            go = true;
          }
        } else {  // fallback: the boundary as a surface (kernels.py:1352-1357)
          surface = true;
        }
      }
      if (surface) {  // one scatter site: deferred Perlin-textured hits and boundary fallbacks
        hp = pt_add(ray.o, pt_scale(ray.d, h.x));
        nrm = hit_normal(sc, ref, hp, ray.d);
        emit = emitted(m);
        ruv = scatter_begin(sc, ref, m, ray.d, hp, nrm, r, sdir, att, scattered);
      }
      if (ruv != kRuvNone) {  // one random_unit_vector site
        const pt_v3 v = random_unit_vector(r);
        if (ruv == kRuvMedium) sdir = v;
        else scattered = scatter_end(sc, ruv, ref, m, hp, nrm, v, sdir, att);
      }
      if (!passthrough) go = scatter_epilogue(fr, scattered, hp, sdir, att, ray, r, cont, ends);
      if (!go) {
        ended = true;  // emissive surfaces add their emission once (:1368-1375); other ends add 0
        stage(fr, wb, ray.item, (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) ? pt_mul(ray.thr, emit)
                                                                              : pt_v3f(0.0f, 0.0f, 0.0f));
      }
    }
    finish_lane(wb, i, ended, go, cont);
    n_ended += ended ? 1u : 0u;
  }
  if (counters) block_flush<3>({n_ended, ends[0], ends[1]}, lds_stack, counters + 2);
}

namespace {
// Library-owned state of one device, created on first use: the streams and
// fork/join events of pipes 1.., the live-count readback events and their
// host-pinned slots [2][kPipes]. `mu` serialises ptmi_wf_render calls on the
// device (each call drives all pipes and reads their counts back), so two
// host threads rendering on one device never share readback slots; calls on
// different devices run concurrently.
struct PipeStreams {
  std::mutex mu;
  hipStream_t s[kPipes] = {};
  hipEvent_t fork = nullptr, join[kPipes] = {};
  hipEvent_t rb[2][kPipes] = {};  // live-count readbacks of two consecutive chunks
  int32_t* pinned_live = nullptr;
  bool ok = false;
};
constexpr int kMaxDevices = 64;
PipeStreams g_pipes[kMaxDevices];

// Called with ps->mu held.
hipError_t pipe_streams_init(PipeStreams* ps) {
  if (ps->ok) return hipSuccess;
  hipError_t e = hipSuccess;
  if (!ps->pinned_live) e = hipHostMalloc((void**)&ps->pinned_live, 2 * kPipes * sizeof(int32_t), hipHostMallocDefault);
  if (e == hipSuccess && !ps->fork) e = hipEventCreateWithFlags(&ps->fork, hipEventDisableTiming);
  for (int p = 1; p < kPipes && e == hipSuccess; ++p) {
    if (!ps->s[p]) e = hipStreamCreateWithFlags(&ps->s[p], hipStreamNonBlocking);
    if (e == hipSuccess && !ps->join[p]) e = hipEventCreateWithFlags(&ps->join[p], hipEventDisableTiming);
  }
  for (int k = 0; k < 2; ++k)
    for (int p = 0; p < kPipes && e == hipSuccess; ++p)
      if (!ps->rb[k][p]) e = hipEventCreateWithFlags(&ps->rb[k][p], hipEventDisableTiming);
  ps->ok = e == hipSuccess;
  return e;
}
#ifndef PTMI_WF_RB_CHUNK
#define PTMI_WF_RB_CHUNK 8
#endif
#ifndef PTMI_WF_CAPACITY_LOG2
#define PTMI_WF_CAPACITY_LOG2 21  // queue slots (all pipes); A/B: 2^21 +3 % over 2^20 (C3, mesh fog)
#endif
constexpr int32_t kMaxCapacity = 1 << PTMI_WF_CAPACITY_LOG2;
constexpr int32_t kSlotQuantum = kShards * kWfBlock;

struct Layout {
  int32_t capacity, medseg;
  size_t q, hit, medq, grp, staging, ctl, total;
};

Layout layout(int32_t npix, int32_t batch) {
  Layout L;
  int64_t items = (int64_t)npix * batch;
  int64_t cap = npix > kMaxCapacity ? npix : kMaxCapacity;
  if (items < cap) cap = items;
  cap = (cap + kPipes * kSlotQuantum - 1) / (kPipes * kSlotQuantum) * (kPipes * kSlotQuantum);
  L.capacity = (int32_t)cap;  // all pipes; each pipe has capacity / kPipes slots
  L.medseg = (int32_t)(cap / kPipes / kShards);
  size_t c = (size_t)cap;
  L.q = 0;
  L.hit = L.q + 3 * sizeof(float4) * c;
  L.medq = L.hit + sizeof(float2) * c;
  L.grp = (L.medq + sizeof(int32_t) * c + 15) & ~(size_t)15;
  L.staging = (L.grp + sizeof(int2) * (c / 64) + 15) & ~(size_t)15;
  L.ctl = (L.staging + 3 * sizeof(float) * (size_t)items + 255) & ~(size_t)255;
  L.total = L.ctl + kCtlWords * sizeof(int32_t);
  return L;
}
}  // namespace

#ifndef PTMI_WF_MAX_BLOCKS
#define PTMI_WF_MAX_BLOCKS (2048 * 256 / PTMI_WF_BLOCK)  // all pipes together; A/B: 4096 -1.5 %, 8192 -3.5 % (C3)
#endif
static_assert((PTMI_WF_MAX_BLOCKS / kPipes) % kShards == 0, "a pipe's grid must be a multiple of the shard count");

// One batch: generate on the caller's stream, fork the pipes, run each pipe's
// intersect -> shade -> medium loop on its own stream until its slots have all
// retired, join, resolve.
template <int STACK, int TRAV = PTMI_TRAV_STACK>
static hipError_t wf_batch(const DevScene& sc, const DevFrame& fr, const WfBufs* wbs, float* accum, int32_t batch,
                           unsigned long long* counters, hipStream_t stream, const PipeStreams& ps) {
  // a pipe's grid = multiple of kShards and of the slot quantum, so its slot i
  // always maps to block (i / kWfBlock) % grid with shard (i / kWfBlock) % kShards
  int64_t blocks = wbs[0].capacity / kWfBlock;
  if (blocks > PTMI_WF_MAX_BLOCKS / kPipes) blocks = PTMI_WF_MAX_BLOCKS / kPipes;
  const unsigned g = (unsigned)blocks;
  (void)hipMemsetAsync(wbs[0].next, 0, kCtlWords * sizeof(int32_t), stream);
  for (int p = 0; p < kPipes; ++p) {
    prof_begin(kProfWfGenerate, stream);
    hipLaunchKernelGGL(wf_generate, dim3(g), dim3(kWfBlock), 0, stream, fr, wbs[p], (int32_t)(p == 0));
    prof_end(kProfWfGenerate, stream);
  }
  hipStream_t st[kPipes];
  st[0] = stream;
  for (int p = 1; p < kPipes; ++p) st[p] = ps.s[p];
  if (kPipes > 1) {
    hipError_t e = hipEventRecord(ps.fork, stream);
    for (int p = 1; p < kPipes && e == hipSuccess; ++p) e = hipStreamWaitEvent(st[p], ps.fork, 0);
    if (e != hipSuccess) return e;
  }
  // Each item needs at most max_depth waves and every iteration advances every
  // live ray by one wave (or hands a waiting slot an item), so this many
  // iterations always drain a pipe.
  const int64_t max_iters = (int64_t)wbs[0].nunits * 64 * (int64_t)(fr.max_depth > 0 ? fr.max_depth : 1) + 2;
  bool live[kPipes];
  for (int p = 0; p < kPipes; ++p) live[p] = true;
  int64_t it = 0;
  const int32_t chunk = PTMI_WF_RB_CHUNK;  // iterations between live-count readbacks
  hipError_t err = hipSuccess;
  // The host reads chunk k's live counts only after chunk k + 1 is queued, so
  // the pipes never idle through the readback's host round trip. Iterations
  // on a drained pipe are no-ops (no slot holds or receives work), so the one
  // extra chunk a pipe may run after draining changes nothing.
  bool inflight[2][kPipes] = {};
  int cur = 0;
  while (it < max_iters) {
    const int64_t n = max_iters - it < chunk ? max_iters - it : chunk;
    for (int64_t j = 0; j < n; ++j) {
      for (int p = 0; p < kPipes; ++p) {
        if (!live[p]) continue;
        const WfBufs& wb = wbs[p];
        prof_begin(kProfWfIntersect, st[p]);
        hipLaunchKernelGGL((wf_intersect<STACK, TRAV>), dim3(g), dim3(kWfBlock), 0, st[p], sc, fr, wb, counters);
        prof_end(kProfWfIntersect, st[p]);
        prof_begin(kProfWfShade, st[p]);
        hipLaunchKernelGGL(wf_shade, dim3(g), dim3(kWfBlock), 0, st[p], sc, fr, wb, counters);
        prof_end(kProfWfShade, st[p]);
        prof_begin(kProfWfMedium, st[p]);
        hipLaunchKernelGGL((wf_medium<STACK, TRAV>), dim3(g), dim3(kWfBlock), 0, st[p], sc, fr, wb, counters);
        prof_end(kProfWfMedium, st[p]);
      }
    }
    it += n;
    err = hipGetLastError();
    for (int p = 0; p < kPipes && err == hipSuccess; ++p) {
      inflight[cur][p] = live[p];
      if (!live[p]) continue;
      err = hipMemcpyAsync(ps.pinned_live + cur * kPipes + p, ctl_live(wbs[p]), sizeof(int32_t),
                           hipMemcpyDeviceToHost, st[p]);
      if (err == hipSuccess) err = hipEventRecord(ps.rb[cur][p], st[p]);
    }
    const int prev = cur ^ 1;
    cur = prev;
    bool waited = false;
    for (int p = 0; p < kPipes && err == hipSuccess; ++p)
      if (inflight[prev][p]) {
        err = hipEventSynchronize(ps.rb[prev][p]);
        waited = true;
      }
    if (err != hipSuccess) break;
    if (!waited) continue;  // first chunk: nothing read back yet
    bool any = false;
    for (int p = 0; p < kPipes; ++p) {
      if (inflight[prev][p]) live[p] = live[p] && ps.pinned_live[prev * kPipes + p] != 0;
      inflight[prev][p] = false;
      any = any || live[p];
    }
    if (!any) break;
  }
  // the last chunk's readbacks may still be in flight: finish them before the
  // pinned slots are reused
  for (int k = 0; k < 2; ++k)
    for (int p = 0; p < kPipes; ++p)
      if (inflight[k][p]) {
        hipError_t e = hipEventSynchronize(ps.rb[k][p]);
        if (err == hipSuccess) err = e;
      }
  for (int p = 1; p < kPipes; ++p) {  // join (also on error: the caller's stream must not run ahead)
    hipError_t e = hipEventRecord(ps.join[p], st[p]);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, ps.join[p], 0);
    if (err == hipSuccess) err = e;
  }
  if (err != hipSuccess) return err;
  return launch_stage_resolve(fr, wbs[0].staging, wbs[0].npix, batch, accum, kProfWfResolve, stream);
}

size_t wf_workspace_bytes(int32_t npix, int32_t batch) {
  if (npix <= 0 || batch <= 0) return 0;
  return layout(npix, batch).total;
}

hipError_t wf_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws, size_t ws_bytes,
                     float* accum, int32_t s_begin, int32_t s_count, unsigned long long* counters,
                     hipStream_t stream) {
  const int32_t npix = fr.w * fr.n_rows;
  // work items (sample, pixel) of a batch are 32-bit ids: at most 2^31 - 1
  int32_t batch = s_count;
  if ((int64_t)npix * batch > 0x7fffffffll) batch = (int32_t)(0x7fffffffll / npix);
  if (batch < 1) return hipErrorInvalidValue;
  while (batch > 1 && layout(npix, batch).total > ws_bytes) batch = (batch + 1) / 2;
  if (layout(npix, batch).total > ws_bytes) return hipErrorInvalidValue;
  int dev = 0;
  {
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  }
  PipeStreams* ps = &g_pipes[dev];
  std::lock_guard<std::mutex> lock(ps->mu);
  {
    hipError_t e = pipe_streams_init(ps);  // pipes 1.. streams, fork/join and readback events, pinned slots
    if (e != hipSuccess) return e;
  }
  for (int32_t b0 = 0; b0 < s_count; b0 += batch) {
    const int32_t nb = s_count - b0 < batch ? s_count - b0 : batch;
    const Layout L = layout(npix, nb);
    char* base = (char*)ws;
    const size_t c = (size_t)L.capacity, cp = c / kPipes;
    WfBufs wbs[kPipes];
    for (int p = 0; p < kPipes; ++p) {
      WfBufs& wb = wbs[p];
      wb.q.a = (float4*)(base + L.q) + p * cp;
      wb.q.b = (float4*)(base + L.q + sizeof(float4) * c) + p * cp;
      wb.q.c = (float4*)(base + L.q + 2 * sizeof(float4) * c) + p * cp;
      wb.hit = (float2*)(base + L.hit) + p * cp;
      wb.medq = (int32_t*)(base + L.medq) + p * cp;
      wb.grp = (int2*)(base + L.grp) + p * (cp / 64);
      wb.staging = (float*)(base + L.staging);
      wb.next = (int32_t*)(base + L.ctl);
      wb.ctl = wb.next + (8 + p * kPipeLines) * kLine;
      wb.capacity = (int32_t)cp;
      wb.medseg = L.medseg;
      wb.npix = npix;
      wb.sq_x = (fr.w + 7) / 8;
      wb.nsq = wb.sq_x * ((fr.n_rows + 7) / 8);
      wb.batch = nb;
      wb.csamp = nb < PTMI_WF_CHUNK_SAMPLES ? nb : PTMI_WF_CHUNK_SAMPLES;
      wb.nunits = wb.nsq * ((nb + wb.csamp - 1) / wb.csamp) * wb.csamp;
      wb.shard_len = (wb.nunits / wb.csamp + kShards - 1) / kShards * wb.csamp;
      wb.shard_groups = L.capacity / 64 / kShards;  // all pipes draw on every shard
      wb.s_begin = s_begin + b0;
    }
    hipError_t e;
    if (fr.traversal == PTMI_TRAV_STACKLESS) e = wf_batch<1, PTMI_TRAV_STACKLESS>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 16) e = wf_batch<16>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 20) e = wf_batch<20>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 24) e = wf_batch<24>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 32) e = wf_batch<32>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else e = wf_batch<64>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ptmi
