// pt_wavefront.hip — breadth-first (wavefront) integrator for gfx950.
//
// Replaces the wavefront stage kernels of kernels.py:1219-1418 as driven by
// TaichiRenderer.render_wavefront (renderer.py:305-334). Stages and layout
// are designed for CDNA4, not translated:
//   * ray queue = five streams per slot (A = o.xyz,d.x; D = d.yz; C =
//     thr.xyz, meta; the work-item word; the rng draw counter), each read
//     only by the stage that needs it, every access a coalesced per-lane
//     vector load/store; meta = depth | wave << 8. wf_intersect reads the
//     item word and the ray (24 B); a fresh camera ray is not stored at all
//     (wf_scatter regenerates it from its item);
//   * hit record = 8 B (t, leaf ref); hit point and normal are recomputed in
//     the shading kernel with the reference's own expressions;
//   * CLOSEST-HIT CLASSIFICATION: wf_intersect ends the paths a hit or miss
//     ends without a scatter (miss: shade_miss_rays, kernels.py:1266-1280;
//     emissive: kernels.py:1365-1375) and compacts every other slot, by its
//     hit's material, into one of five lists with wave64 ballot + mbcnt (one
//     atomic per wave and list): Lambertian, metal/isotropic, dielectric,
//     constant-medium boundary, Perlin-textured surface;
//   * PER-MATERIAL SHADING: one wf_scatter launch walks the medium, Perlin,
//     Lambertian, glossy and dielectric lists in turn, each padded to whole
//     waves, so every wave runs one list's code only: the constant-medium
//     exit traversal (kernels.py:417) and free flight, the Perlin-textured
//     surfaces (three octaves of table gathers, kernels.py:1013-1015), or one
//     material's scatter (kernels.py:817-917). Separate launches per material
//     lost 6 %, separate shading and medium launches 5 %: a launch costs
//     ~7.5 us per pipe and iteration even when its lists are empty;
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
//     intersect -> scatter on its own stream, so
//     the drain at the end of one pipe's launch is filled by another's (+21 %
//     over one pipe).
//   * THE TAIL: once a pipe's live count falls below capacity / 16
//     (PTMI_WF_DRAIN_AT, or ptmi_wf_set_drain_at; the work pool is then
//     empty), one wf_drain launch finishes its remaining paths and the items
//     its groups still hold, each lane looping intersect -> shade over its
//     own slot, instead of ~50 nearly empty intersect + scatter launches;
//   * The host learns that a pipe has drained from a 4-byte live count read
//     back every PTMI_WF_RB_CHUNK (4) iterations, and waits for chunk k's counts only after
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

#include <atomic>
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
#ifndef PTMI_WF_ISECT_LDS
// Stack slots wf_intersect keeps in LDS when its stack is deeper than 16
// slots; the deeper slots spill to global memory (Stack, pt_device.hpp). Its
// LDS stacks set its occupancy: the 20-slot kernel (leaf depth 16-19, e.g.
// the mesh-fog torus) fits 4 waves/SIMD with all slots in LDS, 7 with 11
// (67 VGPRs). A/B on MI355X, parity-identical (also with 3 LDS slots, where
// most pushes spill): mesh fog +2.2 %; for the 16-slot kernel (vol2, C3: 5
// waves/SIMD) 7 waves gained nothing (-1.5 %; 6 waves -2.5 %; larger pipe
// grids -1 to -5 %), so it keeps all 16 in LDS
// (profiles/r03/ab/ab_wf_spill.log). A 16-slot wf_intersect padded down to 4
// waves/SIMD loses 8 % (3 waves: 18 %).
#define PTMI_WF_ISECT_LDS 11
#endif
#ifndef PTMI_WF_SPILL_MAX_STACK
#define PTMI_WF_SPILL_MAX_STACK 20  // kernels of 17 to this many stack slots spill; deeper ones keep them all in LDS
#endif
constexpr int kSpillSlots = PTMI_WF_SPILL_MAX_STACK > PTMI_WF_ISECT_LDS ? PTMI_WF_SPILL_MAX_STACK - PTMI_WF_ISECT_LDS : 0;
template <int STACK, int TRAV>
constexpr int isect_lds() {
  return (TRAV == PTMI_TRAV_STACK && STACK > 16 && STACK <= PTMI_WF_SPILL_MAX_STACK && PTMI_WF_ISECT_LDS < STACK)
             ? PTMI_WF_ISECT_LDS
             : STACK;
}
#ifndef PTMI_WF_MAX_BLOCKS
#define PTMI_WF_MAX_BLOCKS (2048 * 256 / PTMI_WF_BLOCK)  // all pipes together; A/B: 4096 -1.5 %, 8192 -3.5 % (C3)
#endif
constexpr uint32_t kDead = 0xffffffffu;     // item of a retired slot
constexpr uint32_t kPending = 0xfffffffeu;  // item of a slot waiting for work (assigned in wf_intersect)
// A slot whose camera ray was generated and traced in this iteration's
// wf_intersect holds its item | kFresh and nothing else: the ray is not
// stored, wf_scatter regenerates it from the item (get_ray, kernels.py:
// 176-201: the same draws from the same counter-based stream), with
// throughput 1 and depth 0. Items are < 2^31 (wf_render bounds them).
constexpr uint32_t kFresh = 0x80000000u;

// Ray queue: five streams per slot, each read only by the stage that needs
// it. wf_intersect reads the item word (4 B) of every slot and the ray
// (o, d: A + D, 24 B) of a traced one; wf_scatter reads the rest.
struct Queue {
  float4* a;      // o.xyz, d.x
  float2* d;      // d.y, d.z
  float4* c;      // thr.xyz, meta (bits)
  uint32_t* item; // work item (| kFresh), kPending or kDead
  uint32_t* ctr;  // rng draw counter
};

// Closest-hit lists (wf_intersect fills them, wf_scatter drains them).
// Each list holds kShards segments of medseg slot indices; the medium and
// Perlin lists share one array, the Perlin one filling its segments from the
// top (a slot is in at most one list, so together they never exceed a segment).
// Misses and emissive hits (class kListEnded) end in wf_intersect: a lane
// that finishes its traversal early ends its path while the wave's longest
// traversal runs, nearly for free. A/B on MI355X (round 4): an ended list
// drained by wf_scatter instead cost wf_scatter +19 % for wf_intersect -2.4 %,
// C3 -5 % (profiles/r04/ab/). kListEnded is a class, not a list.
enum : int32_t { kListLambertian = 0, kListGlossy = 1, kListDielectric = 2, kListMedium = 3, kListNoise = 4,
                 kListEnded = 5, kLists = 5 };

struct WfBufs {
  Queue q;
  float2* hit;        // t, leaf ref (bits) of a traced slot's closest hit; ref 0 for a miss
  int32_t* lists;     // 4 arrays of capacity indices: Lambertian, glossy + ended, dielectric, medium + Perlin
  float* staging;     // [batch][npix][3] path colours
  int32_t* ctl;       // this pipe's counters, one per 256-B line (see ctl_*)
  char* spill;        // this pipe's spilled stack slots of wf_intersect (kSpillSlots rows of its grid's threads)
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
  FastDiv by_per, by_nsq, by_sqx;  // item decode: / (64 * csamp), / nsq, / sq_x
};

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
// 256-B line. Lines 0-7: next unit per shard (shared); then per pipe 81
// lines: live slots (read by the host), and two sets (by iteration parity)
// of one count per list and shard. wf_intersect of iteration k appends to set
// k & 1 and wf_scatter reads it and zeroes set (k + 1) & 1 for the next
// iteration's wf_intersect.
constexpr int32_t kLine = 64;
constexpr int32_t kPipeLines = 1 + 2 * kLists * 8;
constexpr int32_t kCtlWords = (8 + kPipeLines * kPipes) * kLine;
__host__ __device__ __forceinline__ int32_t* ctl_next(const WfBufs& wb, int32_t s) { return wb.next + s * kLine; }
__host__ __device__ __forceinline__ int32_t* ctl_live(const WfBufs& wb) { return wb.ctl; }
__host__ __device__ __forceinline__ int32_t* ctl_list(const WfBufs& wb, int32_t par, int32_t list, int32_t s) {
  return wb.ctl + (1 + (par * kLists + list) * 8 + s) * kLine;
}
// slot-index entry k of shard s's segment of a list
__device__ __forceinline__ int32_t* list_slot(const WfBufs& wb, int32_t list, int32_t s, int32_t k) {
  const int32_t arr = list < kListMedium ? list : kListMedium;
  int32_t* seg = wb.lists + (size_t)arr * (size_t)wb.capacity + (size_t)s * (size_t)wb.medseg;
  return list == kListNoise ? seg + wb.medseg - 1 - k : seg + k;
}

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
  uint32_t item, ctr, meta;  // item without kFresh
  bool fresh;                // a camera ray regenerated from its item (its slot holds only the item word)
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

// A continuing ray back into its slot; a fresh ray's slot also gets its item
// word without kFresh (the other streams were never written for it).
__device__ __forceinline__ void store_ray_v(const Queue& q, int32_t i, pt_v3 o, pt_v3 d, pt_v3 thr, uint32_t item,
                                            bool was_fresh, uint32_t ctr, uint32_t meta) {
  s_store((pt_qf4*)(q.a + i), pt_qf4{o.x, o.y, o.z, d.x});
  s_store((pt_qf2*)(q.d + i), pt_qf2{d.y, d.z});
  s_store((pt_qf4*)(q.c + i), pt_qf4{thr.x, thr.y, thr.z, __uint_as_float(meta)});
  s_store(q.ctr + i, ctr);
  if (was_fresh) s_store(q.item + i, item);
}

// The slot's state lives in its work-item word: an item (| kFresh), kPending or kDead.
__device__ __forceinline__ void set_slot_item(const Queue& q, int32_t i, uint32_t v) { s_store(q.item + i, v); }

__device__ __forceinline__ uint32_t slot_item(const Queue& q, int32_t i) { return s_load(q.item + i); }

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
  // multiply-shift divisions (exact: items < 2^31, FastDiv)
  const uint32_t per = 64u * (uint32_t)wb.csamp;
  const uint32_t c = fdiv(k, wb.by_per), j = k - c * per;
  const uint32_t blk = fdiv(c, wb.by_nsq), q = c - blk * (uint32_t)wb.nsq;
  const int32_t qy = (int32_t)fdiv(q, wb.by_sqx), qx = (int32_t)q - qy * wb.sq_x;
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

// The ray of slot i for wf_scatter, with its decoded work item. A fresh
// camera ray (generated and traced in this iteration's wf_intersect, not
// stored) is regenerated from its item: the same get_ray draws
// (kernels.py:1219-1239, direction unnormalized, Q1), throughput 1, depth and
// wave 0.
__device__ __forceinline__ Ray load_ray(const DevFrame& fr, const WfBufs& wb, int32_t i, Item& it) {
  const Queue& q = wb.q;
  Ray r;
  const uint32_t w = s_load(q.item + i);
  r.fresh = (w & kFresh) != 0u;
  r.item = w & ~kFresh;
  it = decode_item(fr, wb, r.item);
  if (r.fresh) {
    // (storing it in wf_intersect instead, 28 B, measured 1-2 % slower on C3)
    Rng rng{path_key(fr, wb, it), 0u};
    get_ray(fr, it.px, it.py, rng, r.o, r.d);
    r.ctr = rng.n;
    r.thr = pt_v3f(1.0f, 1.0f, 1.0f);
    r.meta = 0u;
  } else {
    const float4 a = q_load(q.a + i), c = q_load(q.c + i);
    const float2 d = h_load(q.d + i);
    r.o = pt_v3f(a.x, a.y, a.z);
    r.d = pt_v3f(a.w, d.x, d.y);
    r.ctr = s_load(q.ctr + i);
    r.thr = pt_v3f(c.x, c.y, c.z);
    r.meta = __float_as_uint(c.w);
  }
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
    wb.q.item[i] = kPending;
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
// retire. Wave-uniform: called by all 64 lanes of the group. A slot given a
// camera ray gets its origin and direction in (o, d) (true returned); only
// its item word is stored, marked kFresh (wf_scatter regenerates the ray).
__device__ __forceinline__ bool assign_work(const DevFrame& fr, const WfBufs& wb, int32_t i, uint32_t& item,
                                            pt_v3& o, pt_v3& d) {
  const bool pending = item == kPending;
  const unsigned long long pm = __ballot(pending);
  if (pm == 0ull) return false;
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
  bool fresh = false;
  if (pending) {
    if (my == kDead) {
      set_slot_item(wb.q, i, kDead);
      item = kDead;
    } else if (decode_item(fr, wb, my).valid) {
      // generate_camera_rays, kernels.py:1219-1239 (direction left unnormalized, Q1)
      const Item it = decode_item(fr, wb, my);
      Rng rng{path_key(fr, wb, it), 0u};
      get_ray(fr, it.px, it.py, rng, o, d);
      item = my | kFresh;
      set_slot_item(wb.q, i, item);
      fresh = true;
    }  // an item outside the frame / batch: the slot stays pending
  }
  wave_add(pending && my == kDead, ctl_live(wb), -1);
  return fresh;
}

// Path end without a scatter (a miss, or an emissive / absorbing hit): its
// one colour (or 0) to the staging slot, and the slot waits for work.
__device__ __forceinline__ void end_path(const DevFrame& fr, const WfBufs& wb, int32_t i, uint32_t item, pt_v3 c) {
  stage(fr, wb, item, c);
  set_slot_item(wb.q, i, kPending);
}

// A path that ends without a scatter (its traced segment has class
// kListEnded): a miss adds thr * background (shade_miss_rays, kernels.py:
// 1266-1280), an emissive hit thr * emit when the emit colour is non-zero
// (kernels.py:1365-1375). w = the slot's item word (a fresh camera ray's
// throughput is 1: no C record was stored for it), ref = the hit's leaf code,
// 0 for a miss.
__device__ __forceinline__ void end_unscattered(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, int32_t i,
                                                uint32_t w, int32_t ref) {
  pt_v3 thr = pt_v3f(1.0f, 1.0f, 1.0f);
  if (!(w & kFresh)) {
    const float4 c = q_load(wb.q.c + i);
    thr = pt_v3f(c.x, c.y, c.z);
  }
  pt_v3 col = pt_mul(thr, pt_v3f(fr.bg[0], fr.bg[1], fr.bg[2]));
  if (ref != 0) {
    const float4 e = sc.mats[5 * mat_index(sc, ref) + 1];  // emit colour (Mat::m1)
    col = (e.x > 0.0f || e.y > 0.0f || e.z > 0.0f) ? pt_mul(thr, pt_v3f(e.x, e.y, e.z)) : pt_v3f(0.0f, 0.0f, 0.0f);
  }
  end_path(fr, wb, i, w & ~kFresh, col);
}

// Closest-hit classes (PTMI_CLASS_*, include/ptmi.h) are packed into the
// leaf codes by the host, so a hit's list is known without a material load.
// Surface hits whose scatter evaluates Perlin turbulence (a noise texture on
// a Lambertian or isotropic material, kernels.py:1013-1015) have their own
// class, with its own list in wf_scatter: a marble lane would otherwise put three octaves
// of table round trips into every Lambertian wave that holds it.
static_assert(PTMI_CLASS_LAMBERTIAN == kListLambertian && PTMI_CLASS_GLOSSY == kListGlossy &&
                  PTMI_CLASS_DIELECTRIC == kListDielectric && PTMI_CLASS_MEDIUM == kListMedium &&
                  PTMI_CLASS_NOISE == kListNoise && PTMI_CLASS_EMISSIVE == kListEnded,
              "leaf classes are list ids");

// intersect_rays, kernels.py:1242-1263, plus the closest-hit classification:
// a miss (shade_miss_rays, kernels.py:1266-1280) or an emissive hit
// (kernels.py:1365-1375) ends its path here; every other traced slot is
// appended to the list of its hit's material class. Its streams: the item
// word of every slot, o and d of a traced one (24 B), the hit record (8 B)
// and one list entry (4 B); a path end reads thr (16 B) and writes its
// staging slot and item word. A fresh camera ray is not stored.
template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock) void wf_intersect(DevScene sc, DevFrame fr, WfBufs wb, int32_t par,
                                                       unsigned long long* __restrict__ counters) {
  constexpr int LDS = isect_lds<STACK, TRAV>();
  __shared__ uint2 lds_stack[LDS * kWfBlock];
  const int tid = threadIdx.x;
  Stack st{lds_stack + tid, wb.spill, (uint32_t)(blockIdx.x * kWfBlock + tid) * 8u, gridDim.x * kWfBlock * 8u};
  const Queue q = wb.q;
  const int32_t shard = (int32_t)(blockIdx.x % kShards);
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  uint32_t n_live = 0, n_ended = 0;
  for (int32_t i = (int32_t)(blockIdx.x * kWfBlock + tid); i < wb.capacity; i += stride) {
    uint32_t item = s_load(q.item + i);
    pt_v3 o = pt_v3f(0.0f, 0.0f, 0.0f), d = o;
    // generate_camera_rays (kernels.py:1219-1239) for slots that need work
    const bool fresh = assign_work(fr, wb, i, item, o, d);
    int32_t list = -1;
    if (item < kPending) {
      ++n_live;
      if (!fresh) {
        const float4 a = q_load(q.a + i);
        const float2 dyz = h_load(q.d + i);
        o = pt_v3f(a.x, a.y, a.z);
        d = pt_v3f(a.w, dyz.x, dyz.y);
      }
      float t = 0.0f;
      int32_t ref = 0;
      const bool hit = traverse<STACK, kWfBlock, TRAV, LDS>(sc, o, d, kTMin, kTMax, st, t, ref);
      if (!hit) ref = 0;  // a miss: no leaf code
      list = hit ? leaf_class(ref) : kListEnded;
      if (list == kListEnded) {
        end_unscattered(sc, fr, wb, i, item, ref);
        ++n_ended;
        list = -1;
      } else {
        h_store(wb.hit + i, make_float2(t, __int_as_float(ref)));
      }
    }
    // wave-uniform appends, one atomic per wave and non-empty list; lane 0
    // issues them all before it waits for any (independent round trips)
    unsigned long long m[kLists];
    int32_t got[kLists];
#pragma unroll
    for (int32_t l = 0; l < kLists; ++l) {
      m[l] = pt_ballot(list == l);
      got[l] = 0;
    }
    if (lane_id() == 0) {
#pragma unroll
      for (int32_t l = 0; l < kLists; ++l)
        if (m[l]) got[l] = atomicAdd(ctl_list(wb, par, l, shard), (int32_t)__popcll(m[l]));
    }
    // broadcast lane 0's bases: in converged code (every lane of the wave
    // active here), so that lane 0 takes part whatever its own list
    int32_t b0 = 0;
    unsigned long long ml = 0ull;
#pragma unroll
    for (int32_t l = 0; l < kLists; ++l) {
      const int32_t bl = __shfl(got[l], 0);
      if (list == l) {
        b0 = bl;
        ml = m[l];
      }
    }
    if (list >= 0) {
      const int32_t k = b0 + (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(ml >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)ml, 0u));
      if (k < wb.medseg) s_store(list_slot(wb, list, shard, k), i);  // always true: a shard has medseg slots
    }
  }
  if (counters) {
    block_flush<1>({n_live}, lds_stack, counters + 0);
    block_flush<1>({n_ended}, lds_stack, counters + 2);
  }
}

// scatter epilogue of shade_and_scatter (kernels.py:1377-1399) plus the
// per-path wave budget of renderer.py:313: a continuing ray is stored back
// into its slot i (true returned). A path it ends is counted in ends[0]
// (Russian roulette) or ends[1] (depth or wave budget).
__device__ __forceinline__ bool scatter_epilogue(const DevFrame& fr, const WfBufs& wb, int32_t i, bool scattered,
                                                 pt_v3 hp, pt_v3 sdir, pt_v3 att, const Ray& cur, Rng& r,
                                                 uint32_t (&ends)[2]) {
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
  store_ray_v(wb.q, i, hp, sdir, nthr, cur.item, cur.fresh, r.n, (uint32_t)nd | ((uint32_t)(wave + 1) << 8));
  return true;
}

// Per-lane tail of wf_scatter for a path a scatter ended: stage its colour
// (0 unless it ended on an emissive boundary fallback; misses and emissive
// surface hits end in wf_intersect, end_unscattered) and mark the slot as
// waiting for work (the next wf_intersect hands it the next item).
__device__ __forceinline__ void finish_ended(const DevFrame& fr, const WfBufs& wb, int32_t i, const Ray& ray,
                                             pt_v3 emit) {
  end_path(fr, wb, i, ray.item,
           (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) ? pt_mul(ray.thr, emit) : pt_v3f(0.0f, 0.0f, 0.0f));
}

// Shard s and offset of entry j of a list whose shard segments hold cnt[s]
// entries (cnt wave-uniform).
__device__ __forceinline__ int32_t list_entry(const WfBufs& wb, int32_t list, const int32_t (&cnt)[kShards], int32_t j) {
  int32_t off = j, shard = 0;
#pragma unroll
  for (int s = 0; s + 1 < kShards; ++s) {
    if (shard == s && off >= cnt[s]) {
      off -= cnt[s];
      shard = s + 1;
    }
  }
  return s_load(list_slot(wb, list, shard, off));
}

__device__ __forceinline__ int32_t list_counts(const WfBufs& wb, int32_t par, int32_t list, int32_t (&cnt)[kShards]) {
  int32_t n = 0;
#pragma unroll
  for (int s = 0; s < kShards; ++s) {
    cnt[s] = __builtin_amdgcn_readfirstlane(*ctl_list(wb, par, list, s));
    n += cnt[s];
  }
  return n;
}


// One entry i of the Lambertian, glossy or dielectric list (`list`,
// wave-uniform): shade_and_scatter for a surface hit (kernels.py:1359-1399).
__device__ __forceinline__ void shade_entry(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, int32_t list,
                                            int32_t i, uint32_t& n_ended, uint32_t (&ends)[2]) {
  const float2 h = h_load(wb.hit + i);
  const int32_t ref = __float_as_int(h.y);
  Item it;
  const Ray ray = load_ray(fr, wb, i, it);
  const Mat m = load_mat(sc, mat_index(sc, ref));
  Rng r{path_key(fr, wb, it), ray.ctr};
  const pt_v3 hp = pt_add(ray.o, pt_scale(ray.d, h.x));
  const pt_v3 nrm = hit_normal(sc, ref, hp, ray.d);
  pt_v3 sdir = pt_v3f(0.0f, 0.0f, 0.0f), att = pt_v3f(1.0f, 1.0f, 1.0f);
  bool sc_ok = true;
  if (list == kListLambertian) {  // kernels.py:829-849
    att = eval_texture(sc, ref, m, hp);
    sdir = random_cosine_direction(nrm, r);
  } else if (list == kListDielectric) {  // kernels.py:876-903
    sdir = scatter_dielectric(m, ray.d, nrm, r);
  } else {
    sc_ok = scatter(sc, ref, m, ray.d, hp, nrm, r, sdir, att);
  }
  const bool go = scatter_epilogue(fr, wb, i, sc_ok, hp, sdir, att, ray, r, ends);
  if (!go) {
    finish_ended(fr, wb, i, ray, emitted(m));
    ++n_ended;
  }
}

// One entry i of the constant-medium list (exit traversal + free flight,
// apply_constant_medium kernels.py:365-450, and the volume branch of
// shade_and_scatter, kernels.py:1326-1357) or, is_noise, of the Perlin list.
template <int STACK, int TRAV>
__device__ __forceinline__ void medium_entry(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, Stack st,
                                             int32_t i, bool is_noise, uint32_t& n_ended, uint32_t (&ends)[2]) {
  bool ended = false, go = false;
  pt_v3 emit = pt_v3f(0.0f, 0.0f, 0.0f);
  const float2 h = h_load(wb.hit + i);
  const int32_t ref = __float_as_int(h.y);
  Item it;
  const Ray ray = load_ray(fr, wb, i, it);
  float te = 0.0f;
  int32_t rex = 0;
  bool hx = false;
  if (!is_noise)  // the exit search from t_entry + 1e-4 (kernels.py:417-419)
    hx = traverse<STACK, kWfBlock, TRAV>(sc, ray.o, ray.d, h.x + 0.0001f, kTMax, st, te, rex);
  const Mat m = load_mat(sc, mat_index(sc, ref));
  Rng r{path_key(fr, wb, it), ray.ctr};
  bool surface = is_noise, scattered = false, passthrough = false;
  int32_t ruv = kRuvNone;
  pt_v3 hp, nrm, sdir, att;
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
        store_ray_v(wb.q, i, pt_add(ray.o, pt_scale(ray.d, t_exit + eps_t)), ray.d, ray.thr, ray.item, ray.fresh,
                    r.n, ray.meta + (1u << 8));
        go = true;
      }
    } else {  // fallback: the boundary as a surface (kernels.py:1352-1357)
      surface = true;
    }
  }
  if (surface) {  // one scatter site: Perlin-textured hits and boundary fallbacks
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
  if (!passthrough) go = scatter_epilogue(fr, wb, i, scattered, hp, sdir, att, ray, r, ends);
  ended = !go;
  if (ended) finish_ended(fr, wb, i, ray, emit);
  n_ended += ended ? 1u : 0u;
}

// shade_and_scatter (kernels.py:1289-1399) and the constant-medium exit
// search and free flight (apply_constant_medium, kernels.py:365-450) in one
// launch per iteration and pipe: the work index runs over the medium, Perlin,
// Lambertian, glossy and dielectric lists in turn (the traversing medium
// waves first: they are the longest), each padded to whole waves, so every
// wave runs one list's code only — Lambertian (scatter kernels.py:829-849 +
// its texture, :924-1017), dielectric (:876-903), glossy (metal :853-871,
// isotropic :905-915, and anything else scatter() receives), the medium
// (:1326-1357) or the Perlin-textured surfaces. A/B on MI355X against a
// shading launch and a medium launch per iteration (parity-identical): C3
// +4.8 %, mesh fog -1.8 % (the shading waves run at the medium's 4
// waves/SIMD; profiles/r03/ab/ab_wf_fused.log). The surface hit point and
// normal are the reference's (kernels.py:1359-1364); every draw keeps the
// reference's order.
#ifndef PTMI_WF_SCATTER_MIN_WAVES
// 5 waves/SIMD: <= 96 VGPRs (the 16-slot kernel: 96, 72 B/lane of scratch, against 116 VGPRs and 52 B at 4
// waves). A/B on MI355X, parity-identical: C3 +2.1 %, mesh fog +3 % (profiles/r03/ab/ab_wf_scatter_waves.log).
// Kernels of more than 16 stack slots stay at 4 (their 20+ KB LDS stacks allow no more).
#define PTMI_WF_SCATTER_MIN_WAVES 5
#endif
// The medium waves' LDS stacks cap this kernel at 5 waves/SIMD. A/B on
// MI355X (round 4): split into a medium launch (5 waves) and a launch for the
// Perlin and surface lists without LDS stacks (5 / 6 waves), C3 -4 %
// (profiles/r04/ab/ab_r04i_split_knobs_ruv.log).
constexpr int32_t kScatterOrder[kLists] = {kListMedium, kListNoise, kListLambertian, kListGlossy, kListDielectric};

template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock, PTMI_WF_SCATTER_MIN_WAVES) void wf_scatter(DevScene sc, DevFrame fr, WfBufs wb,
                                                    int32_t par, unsigned long long* __restrict__ counters) {
  __shared__ uint2 lds_stack[STACK * kWfBlock];
  Stack st{lds_stack + threadIdx.x};
  int32_t cnt[kLists][kShards], num[kLists], span[kLists];  // wave-uniform
  int32_t n = 0;
#pragma unroll
  for (int l = 0; l < kLists; ++l) {
    num[l] = list_counts(wb, par, kScatterOrder[l], cnt[l]);
    span[l] = (num[l] + 63) & ~63;
    n += span[l];
  }
  if (blockIdx.x < kShards && threadIdx.x < kLists)  // the next iteration's lists start empty
    *ctl_list(wb, par ^ 1, (int32_t)threadIdx.x, (int32_t)blockIdx.x) = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && counters && num[0] > 0)
    atomicAdd(counters + 1, (unsigned long long)num[0]);  // medium exit traversals
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  uint32_t n_ended = 0, ends[2] = {0u, 0u};
  for (int32_t base = (int32_t)(blockIdx.x * kWfBlock); base < n; base += stride) {
    // wave-uniform list of this wave's 64 entries
    int32_t j = base + (int32_t)threadIdx.x, l = 0;
#pragma unroll
    for (int k = 0; k + 1 < kLists; ++k)
      if (l == k && j >= span[k]) {
        j -= span[k];
        l = k + 1;
      }
    int32_t i = -1;
#pragma unroll
    for (int k = 0; k < kLists; ++k)
      if (l == k && j < num[k]) i = list_entry(wb, kScatterOrder[k], cnt[k], j);
    if (i < 0) continue;  // the list's padding
    int32_t lid = kScatterOrder[0];  // this wave's list (wave-uniform select, no indexed table)
#pragma unroll
    for (int k = 1; k < kLists; ++k)
      if (l == k) lid = kScatterOrder[k];
    if (lid == kListMedium || lid == kListNoise) medium_entry<STACK, TRAV>(sc, fr, wb, st, i, lid == kListNoise, n_ended, ends);
    else shade_entry(sc, fr, wb, lid, i, n_ended, ends);
  }
  if (counters) block_flush<3>({n_ended, ends[0], ends[1]}, lds_stack, counters + 2);
}

// The tail of a batch (wf_batch switches a pipe to it once its live slots fall
// below 1 / drain_at of its capacity, i.e. after the work pool ran dry: a
// slot retires only when fetch_units finds every shard empty): one launch
// finishes every path still in the pipe, each lane looping intersect ->
// classify -> shade over its own slot until the path ends — exactly the
// per-path steps of wf_intersect and wf_scatter (the same entry functions,
// reading and writing the same slot), so every path, its draws, its wave
// budget (Q14) and the counters are unchanged. The shards are empty, but a
// group may still hold items it fetched and has not handed out yet
// (wb.grp[g]: up to 63 of a single tail unit, more after a whole-chunk
// fetch): a lane whose slot waits for work, or whose path ends, claims the
// group's next item with an atomic on wb.grp[g].x and traces its camera ray
// (generate_camera_rays, kernels.py:1219-1239) in the same loop, until the
// group's range is spent. What changes is the schedule: instead of one
// intersect and one scatter launch per remaining wave (~7.5 us each even when
// nearly empty, and ~50 of them for the longest Russian-roulette survivors),
// the tail is one launch whose length is the longest remaining chain of
// paths of one slot. Launched on the pipe's stream after a wf_scatter, so no
// slot is fresh and the lists are not used.
__device__ __forceinline__ bool drain_claim(const DevFrame& fr, const WfBufs& wb, int32_t i, uint32_t& w, pt_v3& o,
                                            pt_v3& d) {
  int32_t* const nxt = &wb.grp[i >> 6].x;
  const int32_t end = wb.grp[i >> 6].y;  // not changed by this launch
  for (;;) {
    const int32_t k = atomicAdd(nxt, 1);
    if (k >= end) {
      set_slot_item(wb.q, i, kDead);
      return false;
    }
    const Item it = decode_item(fr, wb, (uint32_t)k);
    if (!it.valid) continue;  // padding of a square outside the frame / past the batch
    Rng rng{path_key(fr, wb, it), 0u};
    get_ray(fr, it.px, it.py, rng, o, d);
    w = (uint32_t)k | kFresh;  // wf_scatter's entry functions regenerate the ray from it (load_ray)
    set_slot_item(wb.q, i, w);
    return true;
  }
}

template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock) void wf_drain(DevScene sc, DevFrame fr, WfBufs wb,
                                                   unsigned long long* __restrict__ counters) {
  __shared__ uint2 lds_stack[STACK * kWfBlock];
  Stack st{lds_stack + threadIdx.x};
  const Queue q = wb.q;
  uint32_t n_seg = 0, n_med = 0, n_ended = 0, ends[2] = {0u, 0u};
  for (int32_t i = (int32_t)(blockIdx.x * kWfBlock + threadIdx.x); i < wb.capacity;
       i += (int32_t)(gridDim.x * kWfBlock)) {
    uint32_t w = s_load(q.item + i);
    if (w == kDead) continue;  // retired: its group's items are all handed out
    for (;;) {
      pt_v3 o, d;
      if (w == kPending) {  // waiting for work: the group's next item, if any
        if (!drain_claim(fr, wb, i, w, o, d)) break;
      } else {
        const float4 a = q_load(q.a + i);
        const float2 dyz = h_load(q.d + i);
        o = pt_v3f(a.x, a.y, a.z);
        d = pt_v3f(a.w, dyz.x, dyz.y);
      }
      // intersect_rays (kernels.py:1242-1263) for this slot
      float t = 0.0f;
      int32_t ref = 0;
      const bool hit = traverse<STACK, kWfBlock, TRAV>(sc, o, d, kTMin, kTMax, st, t, ref);
      ++n_seg;
      if (!hit) ref = 0;
      h_store(wb.hit + i, make_float2(t, __int_as_float(ref)));
      const int32_t list = hit ? leaf_class(ref) : kListEnded;
      const uint32_t before = n_ended;
      if (list == kListEnded) {
        end_unscattered(sc, fr, wb, i, w, ref);
        ++n_ended;
      } else if (list == kListMedium || list == kListNoise) {
        n_med += list == kListMedium ? 1u : 0u;
        medium_entry<STACK, TRAV>(sc, fr, wb, st, i, list == kListNoise, n_ended, ends);
      } else {
        shade_entry(sc, fr, wb, list, i, n_ended, ends);
      }
      // the path ended (its slot now waits for work), or continues from its
      // stored ray (the item word holds the item without kFresh)
      w = n_ended != before ? kPending : (w & ~kFresh);
    }
  }
  if (counters) {
    block_flush<2>({n_seg, n_med}, lds_stack, counters + 0);
    block_flush<3>({n_ended, ends[0], ends[1]}, lds_stack, counters + 2);
    block_flush<1>({n_seg}, lds_stack, counters + PTMI_COUNTER_TAIL_SEGMENTS);
  }
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
#define PTMI_WF_RB_CHUNK 4  // A/B r04j: 4 +1.7 % C3, +1 % mesh fog over 8
#endif
#ifndef PTMI_WF_DRAIN_AT
// A pipe whose read-back live count falls below capacity / drain_at finishes
// its paths in one wf_drain launch (0 = never: one intersect and one scatter
// launch per wave until the pipe is empty). The default; ptmi_wf_set_drain_at
// changes it at run time (tests drive the tail with 1: drain as soon as the
// pool is dry, while most groups still hold fetched items).
#define PTMI_WF_DRAIN_AT 16
#endif
#ifndef PTMI_WF_CAPACITY_LOG2
#define PTMI_WF_CAPACITY_LOG2 21  // queue slots (all pipes); A/B: 2^21 +3 % over 2^20 (C3, mesh fog)
#endif
constexpr int32_t kMaxCapacity = 1 << PTMI_WF_CAPACITY_LOG2;
std::atomic<int32_t> g_drain_at{PTMI_WF_DRAIN_AT};
constexpr int32_t kSlotQuantum = kShards * kWfBlock;

constexpr size_t kQueueBytesPerSlot = 48;
struct Layout {
  int32_t capacity, medseg;
  size_t q, hit, lists, grp, staging, spill, ctl, total;
};
constexpr size_t kSpillPipeBytes = (size_t)kSpillSlots * (PTMI_WF_MAX_BLOCKS / kPipes) * kWfBlock * 8;

Layout layout(int32_t npix, int32_t batch) {
  Layout L;
  int64_t items = (int64_t)npix * batch;
  int64_t cap = npix > kMaxCapacity ? npix : kMaxCapacity;
  if (items < cap) cap = items;
  cap = (cap + kPipes * kSlotQuantum - 1) / (kPipes * kSlotQuantum) * (kPipes * kSlotQuantum);
  L.capacity = (int32_t)cap;  // all pipes; each pipe has capacity / kPipes slots
  L.medseg = (int32_t)(cap / kPipes / kShards);
  size_t c = (size_t)cap;
  L.q = 0;  // queue streams: A (16 B), D (8 B), C (16 B), item (4 B), ctr (4 B) per slot
  L.hit = L.q + kQueueBytesPerSlot * c;
  L.lists = L.hit + sizeof(float2) * c;
  L.grp = (L.lists + 4 * sizeof(int32_t) * c + 15) & ~(size_t)15;
  L.staging = (L.grp + sizeof(int2) * (c / 64) + 15) & ~(size_t)15;
  L.spill = (L.staging + 3 * sizeof(float) * (size_t)items + 255) & ~(size_t)255;
  L.ctl = L.spill + kPipes * kSpillPipeBytes;
  L.total = L.ctl + kCtlWords * sizeof(int32_t);
  return L;
}
}  // namespace

static_assert((PTMI_WF_MAX_BLOCKS / kPipes) % kShards == 0, "a pipe's grid must be a multiple of the shard count");

// One batch: generate on the caller's stream, fork the pipes, run each pipe's
// intersect -> scatter loop on its own stream until its slots have all
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
    const int pslot = prof_begin(kProfWfGenerate, stream);
    hipLaunchKernelGGL(wf_generate, dim3(g), dim3(kWfBlock), 0, stream, fr, wbs[p], (int32_t)(p == 0));
    prof_end(pslot, stream);
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
  const int64_t drain_at = g_drain_at.load(std::memory_order_relaxed);
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
        const int32_t par = (int32_t)((it + j) & 1);  // which list counters this iteration uses
        const int ps_i = prof_begin(kProfWfIntersect, st[p]);
        hipLaunchKernelGGL((wf_intersect<STACK, TRAV>), dim3(g), dim3(kWfBlock), 0, st[p], sc, fr, wb, par, counters);
        prof_end(ps_i, st[p]);
        const int ps_s = prof_begin(kProfWfScatter, st[p]);
        hipLaunchKernelGGL((wf_scatter<STACK, TRAV>), dim3(g), dim3(kWfBlock), 0, st[p], sc, fr, wb, par, counters);
        prof_end(ps_s, st[p]);
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
    for (int p = 0; p < kPipes && err == hipSuccess; ++p) {
      if (inflight[prev][p]) {
        const int32_t n_live = ps.pinned_live[prev * kPipes + p];
        live[p] = live[p] && n_live != 0;
        if (live[p] && drain_at > 0 && (int64_t)n_live * drain_at < (int64_t)wbs[p].capacity) {
          // the pool is empty (some slot found no work) and few paths are left:
          // finish them, and the items groups still hold, in one launch,
          // queued behind the iterations in flight
          const int pd = prof_begin(kProfWfDrain, st[p]);
          hipLaunchKernelGGL((wf_drain<STACK, TRAV>), dim3((unsigned)(wbs[p].capacity / kWfBlock)), dim3(kWfBlock), 0,
                             st[p], sc, fr, wbs[p], counters);
          prof_end(pd, st[p]);
          err = hipGetLastError();
          live[p] = false;
        }
      }
      inflight[prev][p] = false;
      any = any || live[p];
    }
    if (err != hipSuccess) break;
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

int32_t wf_set_drain_at(int32_t divisor) { return g_drain_at.exchange(divisor); }

size_t wf_workspace_bytes(int32_t npix, int32_t batch) {
  if (npix <= 0 || batch <= 0) return 0;
  return layout(npix, batch).total;
}

hipError_t wf_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws, size_t ws_bytes,
                     float* accum, int32_t s_begin, int32_t s_count, unsigned long long* counters,
                     hipStream_t stream) {
  const int32_t npix = fr.w * fr.n_rows;
  // work items (sample, pixel) of a batch are ids below 2^31 (FastDiv's
  // range), padded ids included: 64 per 8x8 pixel square, and the batch's
  // samples rounded up to whole chunks (wb.nunits below)
  const int64_t sq_items = 64ll * ((fr.w + 7) / 8) * ((fr.n_rows + 7) / 8);
  int32_t batch = s_count;
  const int64_t max_batch = sq_items > 0 ? 0x7fffffffll / sq_items - (PTMI_WF_CHUNK_SAMPLES - 1) : 0;
  if (batch > max_batch) batch = (int32_t)max_batch;
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
      wb.q.d = (float2*)(base + L.q + 16 * c) + p * cp;
      wb.q.c = (float4*)(base + L.q + 24 * c) + p * cp;
      wb.q.item = (uint32_t*)(base + L.q + 40 * c) + p * cp;
      wb.q.ctr = (uint32_t*)(base + L.q + 44 * c) + p * cp;
      wb.hit = (float2*)(base + L.hit) + p * cp;
      wb.lists = (int32_t*)(base + L.lists) + p * 4 * cp;
      wb.grp = (int2*)(base + L.grp) + p * (cp / 64);
      wb.staging = (float*)(base + L.staging);
      wb.next = (int32_t*)(base + L.ctl);
      wb.ctl = wb.next + (8 + p * kPipeLines) * kLine;
      wb.spill = base + L.spill + p * kSpillPipeBytes;
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
      wb.by_per = fast_div(64u * (uint32_t)wb.csamp);
      wb.by_nsq = fast_div((uint32_t)wb.nsq);
      wb.by_sqx = fast_div((uint32_t)wb.sq_x);
    }
    hipError_t e;
    if (fr.traversal == PTMI_TRAV_STACKLESS) e = wf_batch<1, PTMI_TRAV_STACKLESS>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 16) e = wf_batch<16>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 20) e = wf_batch<20>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 24) e = wf_batch<24>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= 32) e = wf_batch<32>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else if (stack_needed <= kRefStackSlots - 1) e = wf_batch<64>(sc, fr, wbs, accum, nb, counters, stream, *ps);
    else e = wf_batch<kRefStackSlots, kTravRefStack>(sc, fr, wbs, accum, nb, counters, stream, *ps);  // leaf depth > 62
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ptmi
