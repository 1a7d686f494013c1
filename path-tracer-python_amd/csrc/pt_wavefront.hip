// pt_wavefront.hip — breadth-first (wavefront) integrator for gfx950.
//
// Replaces the wavefront stage kernels of kernels.py:1219-1418 as driven by
// TaichiRenderer.render_wavefront (renderer.py:305-334). Stages and layout
// are designed for CDNA4, not translated:
//   * RAY BUFFERS, COMPACTED AND SORTED BY DIRECTION (round 5): every
//     iteration traces up to `capacity` rays per pipe from one of two ray
//     buffers (by iteration parity). The rays that continue are written by
//     wf_scatter into the other buffer, appended (wave64 ballot + one atomic
//     per wave and bin) to the segment of their direction octant, so one
//     wf_intersect wave traces 64 rays of one octant that left neighbouring
//     surfaces (one wf_scatter wave's worth of shading): the traversal visits
//     similar nodes in the same order across the wave. Segments are also
//     sharded by the producing block's XCD (8 shards), so the appends of one
//     launch spread over 64 counters; a wave reads all 64 counts at once and
//     maps its work index to (bin, shard, offset) with a scan. A segment that
//     overflows its region spills into an unsorted overflow region. The
//     reference appends continuing rays to one next queue with one atomic per
//     ray and copies it back (kernels.py:1377-1418);
//   * FRESH CAMERA RAYS fill the buffer back up to `capacity` every
//     iteration: the lanes past the continuing rays claim consecutive work
//     items (one 8x8 pixel square x one sample per 64 items) with one atomic
//     per wave on their XCD's shard of the work pool (stealing from the other
//     shards when it is empty) and trace their camera rays
//     (generate_camera_rays, kernels.py:1219-1239); a fresh ray is not
//     stored, only its item word (| kFresh): wf_scatter regenerates it;
//   * ray record = five streams (A = o.xyz,d.x; D = d.yz; C = thr.xyz, meta;
//     the work-item word; the rng draw counter), each read only by the stage
//     that needs it, every access a per-lane vector load/store, coalesced
//     along a segment; meta = depth | wave << 8;
//   * hit record = 8 B (t, leaf ref); hit point and normal are recomputed in
//     the shading kernel with the reference's own expressions;
//   * CLOSEST-HIT CLASSIFICATION: wf_intersect ends the paths a hit or miss
//     ends without a scatter (miss: shade_miss_rays, kernels.py:1266-1280;
//     emissive: kernels.py:1365-1375) and compacts every other ray, by its
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
//   * WORK POOL: the reference pushes one sample of every pixel through
//     max_depth bounce-synchronous waves (renderer.py:305-334), so after a
//     few bounces its queues are nearly empty. Here the (sample, pixel)
//     pairs of a batch are work items, handed out as rays end, so every
//     launch works on a full buffer until the batch runs out. Item counters
//     are sharded 8 ways (blocks b and b+8 share an XCD), each counter on its
//     own 256-B line, because a single device-wide counter saturates near 88
//     returning atomics/us on MI355X (MI355X_MICROARCH.md, "dequeue");
//   * PIPES: the rays are split into 4 independent parts, each looping
//     intersect -> scatter on its own stream, so the drain at the end of one
//     pipe's launch is filled by another's (+21 % over one pipe);
//   * THE TAIL: once the pool is empty and a pipe traces fewer than
//     capacity / 16 rays per iteration (PTMI_WF_DRAIN_AT, or
//     ptmi_wf_set_drain_at), one wf_drain launch finishes its remaining
//     paths, each lane looping intersect -> scatter over its own ray, instead
//     of ~50 nearly empty intersect + scatter launches;
//   * The host learns that a pipe has drained from its status word (rays
//     traced, pool empty) read back every PTMI_WF_RB_CHUNK (4) iterations,
//     and waits for chunk k's status only after chunk k + 1 is queued, so no
//     pipe idles through the host round trip (the reference reads its ray
//     count back every bounce, renderer.py:315).
//   * Each ray carries its own wave count and is dropped at max_depth waves,
//     exactly the reference's per-path budget (Q14, incl. passthrough Q11).
//   * A path adds at most one colour to its pixel, when it ends (a miss, or an
//     emissive hit, which never scatters: kernels.py:1266-1280, 1365-1375,
//     906), so each path writes that colour (or 0) to a staging slot
//     [sample][pixel]; a resolve kernel then adds the slots into the
//     accumulator in sample order — the same float additions, in the same
//     order, as the reference's per-sample accumulation, with no atomics and
//     no ordering constraint between concurrent paths of one pixel. Which
//     ray is traced in which lane, and when, therefore changes nothing.
#include "pt_launch.hpp"
#include "pt_prof.hpp"

#include <atomic>
#include <mutex>

namespace ptmi {

constexpr int kShards = 8;
#ifndef PTMI_WF_CHUNK_SAMPLES
#define PTMI_WF_CHUNK_SAMPLES 4  // samples per work chunk (one 8x8 pixel square each)
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
// most pushes spill): mesh fog +2.2 %; for the 16-slot kernel (vol2, C3) 7
// waves measured -1.5 % on round 3's in-place slots (profiles/r03/ab/ab_wf_spill.log)
// and +0.8 % on round 5's compacted buffers (PTMI_WF_SPILL_MIN_STACK below). A
// 16-slot wf_intersect padded down to 4 waves/SIMD loses 8 % (3 waves: 18 %).
#define PTMI_WF_ISECT_LDS 10
#endif
#ifndef PTMI_WF_SPILL_MAX_STACK
#define PTMI_WF_SPILL_MAX_STACK 20  // kernels of 17 to this many stack slots spill; deeper ones keep them all in LDS
#endif
constexpr int kSpillSlots = PTMI_WF_SPILL_MAX_STACK > PTMI_WF_ISECT_LDS ? PTMI_WF_SPILL_MAX_STACK - PTMI_WF_ISECT_LDS : 0;
#ifndef PTMI_WF_SPILL_MIN_STACK
// Kernels of this many stack slots up to PTMI_WF_SPILL_MAX_STACK spill. Round 5,
// on the compacted buffers: the 16-slot kernel (vol2) with 11 slots in LDS and
// 5 spilled runs at 7 waves/SIMD instead of 5: C3 +0.8 % over three A/B runs
// (1946-1961 vs 1927-1944; 13 slots, 6 waves: -0.5 %), the mesh fog's 20-slot
// kernel unchanged (profiles/r05/ab/ab_wf_lds_slots16.log, ab_wf_prio_block.log).
// Round 3 had measured it -1.5 % on the in-place slots.
#define PTMI_WF_SPILL_MIN_STACK 16
#endif
template <int STACK, int TRAV>
constexpr int isect_lds() {
  return (TRAV == PTMI_TRAV_STACK && STACK >= PTMI_WF_SPILL_MIN_STACK && STACK <= PTMI_WF_SPILL_MAX_STACK &&
          PTMI_WF_ISECT_LDS < STACK)
             ? PTMI_WF_ISECT_LDS
             : STACK;
}
// ... and with 10 LDS slots (10 KiB per 2-wave block: 8 waves/SIMD) the
// kernel is held to the 8-wave VGPR budget (64 VGPRs; 100 B/lane of scratch
// instead of 52): A/B on MI355X, parity-identical, against 11 slots at 7 waves
// (70 VGPRs): C3 +1.5 % (bench.py 2033 vs 2003), mesh fog +0.7 %
// (profiles/r05/ab/ab_wf_isect_8waves.log). Kernels that keep more slots in
// LDS (and the stackless walk) get no bound.
#ifndef PTMI_WF_ISECT_MIN_WAVES
#define PTMI_WF_ISECT_MIN_WAVES 8
#endif
template <int STACK, int TRAV>
constexpr int isect_min_waves() {
  return (isect_lds<STACK, TRAV>() < STACK && isect_lds<STACK, TRAV>() <= 10) ? PTMI_WF_ISECT_MIN_WAVES : 1;
}
#ifndef PTMI_WF_MAX_BLOCKS
#define PTMI_WF_MAX_BLOCKS (2048 * 256 / PTMI_WF_BLOCK)  // all pipes together; A/B: 4096 -1.5 %, 8192 -3.5 % (C3)
#endif
// A fresh camera ray (generated and traced in this iteration's wf_intersect)
// is stored as its item | kFresh and nothing else: wf_scatter regenerates it
// from the item (get_ray, kernels.py:176-201: the same draws from the same
// counter-based stream), with throughput 1 and depth 0. Items are < 2^31
// (wf_render bounds them).
constexpr uint32_t kFresh = 0x80000000u;

// Continuing-ray segments: kBins direction bins x kShards producer shards,
// one counter each (kSegs <= 64: one wave holds them all, one per lane).
// Sorting by octant, A/B on MI355X (round 5, parity-identical;
// profiles/r05/ab/ab_wf_sort.log): against the round-4 in-place slots
// (1685-1694 Msamples/s on C3, 705-708 on mesh fog) the compacted buffers
// alone (one bin) give 1889-1900 / 847-849, sorted by octant 1914-1923 /
// 850-854; wf_intersect's lane efficiency 0.43 unsorted, 0.45 sorted.
constexpr int kBins = 8;
constexpr int kSegs = kBins * kShards;
#ifndef PTMI_WF_SEG_DIV
#define PTMI_WF_SEG_DIV 16  // a segment's region holds capacity / this rays (4x an even share of 64 segments)
#endif

// Ray buffer of one iteration parity: positions [0, npos) of six streams.
// Segment s holds positions [s * seg_cap, (s + 1) * seg_cap), the overflow
// region the next `capacity`, the fresh camera rays the last `capacity`.
struct RayBuf {
  float4* a;       // o.xyz, d.x
  float4* c;       // thr.xyz, meta (bits)
  float2* d;       // d.y, d.z
  float2* hit;     // t, leaf ref (bits) of the closest hit (wf_intersect -> wf_scatter)
  uint32_t* item;  // work item (| kFresh)
  uint32_t* ctr;   // rng draw counter
};

// Closest-hit lists (wf_intersect fills them, wf_scatter drains them).
// Each list holds kShards segments of medseg ray positions; the medium and
// Perlin lists share one array, the Perlin one filling its segments from the
// top (a ray is in at most one list, so together they never exceed a segment).
// Misses and emissive hits (class kListEnded) end in wf_intersect: a lane
// that finishes its traversal early ends its path while the wave's longest
// traversal runs, nearly for free. A/B on MI355X (round 4): an ended list
// drained by wf_scatter instead cost wf_scatter +19 % for wf_intersect -2.4 %,
// C3 -5 % (profiles/r04/ab/). kListEnded is a class, not a list.
enum : int32_t { kListLambertian = 0, kListGlossy = 1, kListDielectric = 2, kListMedium = 3, kListNoise = 4,
                 kListEnded = 5, kLists = 5 };

struct WfBufs {
  RayBuf rb[2];       // by iteration parity: wf_intersect(k) and wf_scatter(k) read rb[k & 1], wf_scatter(k) writes rb[(k + 1) & 1]
  int32_t* lists;     // 4 arrays of kShards x medseg positions: Lambertian, glossy, dielectric, medium + Perlin
  float* staging;     // [batch][npix][3] path colours
  int32_t* ctl;       // this pipe's counters, one per 256-B line (see ctl_*)
  char* spill;        // this pipe's spilled stack slots of wf_intersect (kSpillSlots rows of its grid's threads)
  int32_t* next;      // next-item counters of the work pool shards, shared by the pipes, one per 256-B line
  int32_t capacity;   // rays traced per iteration (this pipe)
  int32_t seg_cap;    // positions per continuing-ray segment
  int32_t medseg;     // positions per shard segment of a material list
  int32_t npix;       // pixels of the frame's pixel set
  int32_t sq_x, nsq;  // 8x8 pixel squares covering the pixel set: per row, total
  int32_t csamp;      // samples per chunk: a chunk is one square x csamp samples (64 * csamp items)
  int32_t batch;      // samples of the batch
  int32_t nitems;     // work items of the batch, padded to whole squares and chunks
  int32_t shard_len;  // items per pool shard (whole chunks): shard s owns [s*len, min((s+1)*len, nitems))
  int32_t s_begin;    // first sample of the batch
  FastDiv by_per, by_nsq, by_sqx;  // item decode: / (64 * csamp), / nsq, / sq_x
};

// Pipes: the rays are split into PTMI_WF_PIPES independent parts, each
// driven through its own intersect/scatter loop on its own stream, so one
// pipe's kernels fill the drain at the end of another's. They share the work
// pool (next-item counters) and the staging buffer.
#ifndef PTMI_WF_PIPES
#define PTMI_WF_PIPES 4  // A/B on MI355X: 1 -> 2 pipes +15 % (C3), 2 -> 4 +5 %
#endif
constexpr int32_t kPipes = PTMI_WF_PIPES;

// Device-scope atomics are performed per cache line at the memory side, so
// counters sharing a line serialize as one: every counter gets its own
// 256-B line. Lines 0-7: next item per pool shard (shared); then per pipe:
// its status ([2]: the pool was empty after the last wf_scatter's iteration,
// written by that wf_scatter; [0], [1]: the continuing rays of the last
// wf_intersect and the [2] it saw, for the host), two sets (by
// iteration parity) of kSegs segment counts and one overflow count, and two
// sets of one count per material list and shard.
constexpr int32_t kLine = 64;
constexpr int32_t kPipeLines = 3 + 2 * kSegs + 2 * kLists * kShards;
constexpr int32_t kCtlWords = (8 + kPipeLines * kPipes) * kLine;
__host__ __device__ __forceinline__ int32_t* ctl_next(const WfBufs& wb, int32_t s) { return wb.next + s * kLine; }
__host__ __device__ __forceinline__ int32_t* ctl_status(const WfBufs& wb) { return wb.ctl; }
__device__ __forceinline__ int32_t* ctl_seg(const WfBufs& wb, int32_t par, int32_t s) {
  return wb.ctl + (1 + par * kSegs + s) * kLine;
}
__device__ __forceinline__ int32_t* ctl_ovf(const WfBufs& wb, int32_t par) { return wb.ctl + (1 + 2 * kSegs + par) * kLine; }
__device__ __forceinline__ int32_t* ctl_list(const WfBufs& wb, int32_t par, int32_t list, int32_t s) {
  return wb.ctl + (3 + 2 * kSegs + (par * kLists + list) * kShards + s) * kLine;
}
// entry k of shard s's segment of a list
__device__ __forceinline__ int32_t* list_slot(const WfBufs& wb, int32_t list, int32_t s, int32_t k) {
  const int32_t arr = list < kListMedium ? list : kListMedium;
  int32_t* seg = wb.lists + ((size_t)arr * kShards + (size_t)s) * (size_t)wb.medseg;
  return list == kListNoise ? seg + wb.medseg - 1 - k : seg + k;
}
__device__ __forceinline__ int32_t ovf_base(const WfBufs& wb) { return kSegs * wb.seg_cap; }
__device__ __forceinline__ int32_t fresh_base(const WfBufs& wb) { return kSegs * wb.seg_cap + wb.capacity; }

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint32_t lane_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-aggregated appends of the lanes of a wave to N counters (call from
// converged code): `cls` = the lane's counter (-1: none). One ballot per
// counter; lane k < N adds class k's lane count to counter k, so the wave's
// appends are one atomic instruction (lanes of empty classes add nothing),
// and each lane gets the counter's old value from its class's lane plus its
// rank among its class's lanes. Returns the lane's slot (meaningful only for
// cls >= 0).
template <int N, typename Ptr>
__device__ __forceinline__ int32_t wave_append(int32_t cls, Ptr counter_of) {
  const int lane = lane_id();
  unsigned long long mine = 0ull;
  int32_t n_k = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const unsigned long long mk = __builtin_amdgcn_ballot_w64(cls == k);
    if (cls == k) mine = mk;
    if (lane == k) n_k = (int32_t)__popcll(mk);
  }
  int32_t base = 0;
  if (lane < N && n_k > 0) base = atomicAdd(counter_of(lane), n_k);
  base = __shfl(base, cls < 0 ? 0 : cls);
  return base + (int32_t)lane_rank(mine);
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
  bool fresh;                // a camera ray regenerated from its item (only its item word is stored)
};

// A ray that continues (wf_scatter appends it to its direction's segment of
// the next iteration's buffer; wf_drain stores it back in place).
struct Cont {
  pt_v3 o, d, thr;
  uint32_t item, ctr, meta;
  bool go;
};

// Streamed buffers (ray records, hit records, lists, staging) go through
// these helpers. The stage kernels re-read what the previous one wrote, and
// that reuse is worth more than streaming hints: A/B on MI355X
// (parity-identical), `nt` loads + stores / `nt` stores / `sc1` stores, C3
// -10 % / -5 % / -5 % (profiles/r02/ab/ab_nontemporal.log, profiles/r02/pmc_cache/).
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
__device__ __forceinline__ float2 h_load(const float2* p) {
  const pt_qf2 v = s_load((const pt_qf2*)p);
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ void h_store(float2* p, float2 v) { s_store((pt_qf2*)p, pt_qf2{v.x, v.y}); }

// A continuing ray's record at position p (all five streams).
__device__ __forceinline__ void store_ray(const RayBuf& B, int32_t p, const Cont& cn) {
  s_store((pt_qf4*)(B.a + p), pt_qf4{cn.o.x, cn.o.y, cn.o.z, cn.d.x});
  s_store((pt_qf2*)(B.d + p), pt_qf2{cn.d.y, cn.d.z});
  s_store((pt_qf4*)(B.c + p), pt_qf4{cn.thr.x, cn.thr.y, cn.thr.z, __uint_as_float(cn.meta)});
  s_store(B.ctr + p, cn.ctr);
  s_store(B.item + p, cn.item);
}

// Work items come in chunks of one 8x8 pixel square x csamp samples. Chunk c
// is square c % nsq of sample block c / nsq (so early chunks cover every
// square); item j of a chunk is pixel j % 64 of the square, sample j / 64 of
// the block. A wave's 64 fresh rays are consecutive items, so they come
// from one pixel square — the coherence the megakernel's waves get from
// their 8x8 squares. Items outside the frame or past the batch are skipped.
// it.p is the row-major pixel index (staging).
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

// The ray at position p for wf_scatter, with its decoded work item. A fresh
// camera ray (generated and traced in this iteration's wf_intersect, not
// stored) is regenerated from its item: the same get_ray draws
// (kernels.py:1219-1239, direction unnormalized, Q1), throughput 1, depth and
// wave 0.
__device__ __forceinline__ Ray load_ray(const DevFrame& fr, const WfBufs& wb, const RayBuf& X, int32_t p, Item& it) {
  Ray r;
  const uint32_t w = s_load(X.item + p);
  r.fresh = (w & kFresh) != 0u;
  r.item = w & ~kFresh;
  it = decode_item(fr, wb, r.item);
  if (r.fresh) {
    // (storing it in wf_intersect instead, 28 B, measured 1-2 % slower on C3 in round 4)
    Rng rng{path_key(fr, wb, it), 0u};
    get_ray(fr, it.px, it.py, rng, r.o, r.d);
    r.ctr = rng.n;
    r.thr = pt_v3f(1.0f, 1.0f, 1.0f);
    r.meta = 0u;
  } else {
    const float4 a = q_load(X.a + p), c = q_load(X.c + p);
    const float2 d = h_load(X.d + p);
    r.o = pt_v3f(a.x, a.y, a.z);
    r.d = pt_v3f(a.w, d.x, d.y);
    r.ctr = s_load(X.ctr + p);
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

// ------------------------------------------------------------ work pool
__device__ __forceinline__ int32_t shard_end(const WfBufs& wb, int32_t s) {
  int64_t e = (int64_t)(s + 1) * wb.shard_len;
  return e < wb.nitems ? (int32_t)e : wb.nitems;
}

// True when every pool shard is spent (wave-uniform; lane s < kShards reads
// shard s). Counters only grow, so a stale read can only say "not empty".
// wf_scatter looks once per iteration, after all of the iteration's claims;
// the next wf_intersect then claims in none of its waves or may claim in all.
__device__ __forceinline__ bool pool_dry(const WfBufs& wb) {
  const int lane = lane_id();
  bool left = false;
  if (lane < kShards)
    left = __hip_atomic_load(ctl_next(wb, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < shard_end(wb, lane);
  return pt_ballot(left) == 0ull;
}

// Work items for the lanes of a wave that want one (call from converged
// code): consecutive items of the wave's own shard, one atomic per wave and
// shard tried, then of the other shards while lanes are left; -1 for a lane
// that gets none (the pool is empty). A counter may run past its shard's end
// (by at most the lanes asking at once): it only grows.
__device__ __forceinline__ int32_t claim_items(const WfBufs& wb, int32_t shard, bool want) {
  const unsigned long long m = pt_ballot(want);
  if (m == 0ull) return -1;
  const int32_t n = (int32_t)__popcll(m), rank = (int32_t)lane_rank(m);
  int32_t item = -1, taken = 0;
  for (int32_t a = 0; a < kShards && taken < n; ++a) {
    const int32_t s = (shard + a) & (kShards - 1);
    const int32_t e = shard_end(wb, s);
    int32_t t = e;
    if (lane_id() == 0) {
      t = __hip_atomic_load(ctl_next(wb, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t < e) t = atomicAdd(ctl_next(wb, s), n - taken);
    }
    t = __shfl(t, 0);
    const int32_t got = t < e ? (e - t < n - taken ? e - t : n - taken) : 0;
    if (want && rank >= taken && rank < taken + got) item = t + (rank - taken);
    taken += got;
  }
  return item;
}

// Initial state of a batch (the host zeroed every counter): pool shard s
// starts at its first item.
__global__ __launch_bounds__(64) void wf_generate(WfBufs wb) {
  const int32_t s = (int32_t)threadIdx.x;
  if (s < kShards) *ctl_next(wb, s) = min(s * wb.shard_len, wb.nitems);
}

// ------------------------------------------------------------ segments
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t t = __shfl_up(v, (unsigned)o);
    if (lane >= o) v += t;
  }
  return v;
}

// The continuing rays of one parity, as a wave sees them: lane l < kSegs
// holds the entries of the lower shards' segments of its bin; lane b <
// kBins its bin's first work index and size. Work indices: the bins in
// order, each padded to whole waves, then the overflow region, padded, then
// the fresh rays. A segment's counter counts every append; its region holds
// seg_cap (the rest went to the overflow region).
struct SegTable {
  int32_t pre, bstart, btot;                    // per lane (see above)
  int32_t ovf_start, ovf_n, fresh_start, live;  // wave-uniform; live = continuing rays
};
__device__ __forceinline__ SegTable seg_table(const WfBufs& wb, int32_t par) {
  SegTable T;
  const int lane = lane_id();
  const int32_t c = lane < kSegs ? min(s_load(ctl_seg(wb, par, lane)), wb.seg_cap) : 0;
  const int32_t incl = wave_incl_scan(c);
  const int32_t first = lane & ~(kShards - 1);
  const int32_t below = __shfl(incl, first > 0 ? first - 1 : 0);
  T.pre = incl - c - (first > 0 ? below : 0);
  const int32_t bl = lane < kBins ? lane : 0;
  const int32_t hi = __shfl(incl, bl * kShards + kShards - 1);
  const int32_t lo = __shfl(incl, bl > 0 ? bl * kShards - 1 : 0);
  T.btot = lane < kBins ? hi - (bl > 0 ? lo : 0) : 0;
  const int32_t span = (T.btot + 63) & ~63;
  const int32_t sincl = wave_incl_scan(span);
  T.bstart = sincl - span;
  const int32_t spans = __shfl(sincl, 63);
  const int32_t ov = __builtin_amdgcn_readfirstlane(min(s_load(ctl_ovf(wb, par)), wb.capacity));
  // the wave-uniform fields in SGPRs (readfirstlane of converged values)
  T.ovf_start = __builtin_amdgcn_readfirstlane(spans);
  T.ovf_n = ov;
  T.fresh_start = __builtin_amdgcn_readfirstlane(spans + ((ov + 63) & ~63));
  T.live = __builtin_amdgcn_readfirstlane(__shfl(incl, 63) + ov);
  return T;
}

// Position of work index w0 + lane (w0 a wave's base, below fresh_start), or
// -1 for a padding lane. Call with every lane of the wave active: the bin's
// start, size and shard offsets are read from other lanes' registers
// (v_readlane), and a lane's register holds a defined value only while that
// lane is active. All the reads therefore come before any lane-dependent
// branch, and the padding test is a select. Round 6 root cause:
// round 5's form left the padding lanes first (`if (j >= btot) return -1`)
// and read the shard offsets of lanes b * 8 + k afterwards — in the last,
// partly filled wave of a bin those are padding lanes, inactive at the read.
// The shipped build kept the offsets in a register and read the right
// values; a build held to 5 waves/SIMD spilled them and reloaded them from
// scratch inside the branch, i.e. for the active lanes only, so some lanes
// read another value's bits as an offset and traced a ray twice or not at all.
__device__ __forceinline__ int32_t cont_position(const SegTable& T, const WfBufs& wb, int32_t w0) {
  const int lane = lane_id();
  if (w0 >= T.ovf_start) {  // wave-uniform
    const int32_t j = w0 - T.ovf_start + lane;
    return j < T.ovf_n ? ovf_base(wb) + j : -1;
  }
  const unsigned long long m = pt_ballot(lane < kBins && T.bstart <= w0 && w0 < T.bstart + T.btot);
  if (m == 0ull) return -1;  // (a wave base never falls in a bin's padding alone: bins are padded to < 64 more)
  const int32_t b = __ffsll((long long)m) - 1;  // wave-uniform: the bin this wave reads
  const int32_t bstart = __builtin_amdgcn_readlane(T.bstart, b), btot = __builtin_amdgcn_readlane(T.btot, b);
  int32_t pk[kShards];  // entries of the bin's lower shards, per shard (wave-uniform)
#pragma unroll
  for (int k = 1; k < kShards; ++k) pk[k] = __builtin_amdgcn_readlane(T.pre, b * kShards + k);
  const int32_t j = w0 - bstart + lane;
  int32_t s = 0, off = j;
#pragma unroll
  for (int k = 1; k < kShards; ++k) {
    if (j >= pk[k]) {
      s = k;
      off = j - pk[k];
    }
  }
  return j < btot ? (b * kShards + s) * wb.seg_cap + off : -1;
}

// Direction bin of a continuing ray: its octant.
__device__ __forceinline__ int32_t ray_bin(pt_v3 d) {
  return (d.x < 0.0f ? 1 : 0) | (d.y < 0.0f ? 2 : 0) | (d.z < 0.0f ? 4 : 0);
}

// Appends the wave's continuing rays to their segments of the next
// iteration's buffer (call from converged code): one atomic per wave and
// non-empty bin (one instruction, wave_append), then each ray's record to
// its position; ranks past a segment's region go to the overflow region
// (one more atomic).
__device__ __forceinline__ void append_cont(const WfBufs& wb, int32_t npar, int32_t shard, const Cont& cn) {
  const RayBuf& Y = wb.rb[npar];
  const int32_t bin = cn.go ? ray_bin(cn.d) : -1;
  const int32_t k = wave_append<kBins>(bin, [&](int32_t b) { return ctl_seg(wb, npar, b * kShards + shard); });
  const bool over = cn.go && k >= wb.seg_cap;
  const int32_t o = wave_append<1>(over ? 0 : -1, [&](int32_t) { return ctl_ovf(wb, npar); });
  if (cn.go) store_ray(Y, over ? ovf_base(wb) + o : (bin * kShards + shard) * wb.seg_cap + k, cn);
}

// A path that ends without a scatter (its traced segment has class
// kListEnded): a miss adds thr * background (shade_miss_rays, kernels.py:
// 1266-1280), an emissive hit thr * emit when the emit colour is non-zero
// (kernels.py:1365-1375). w = the ray's item word (a fresh camera ray's
// throughput is 1: no C record was stored for it), ref = the hit's leaf code,
// 0 for a miss. Its one colour goes to the staging slot.
__device__ __forceinline__ void end_unscattered(const DevScene& sc, const DevFrame& fr, const WfBufs& wb,
                                                const RayBuf& X, int32_t p, uint32_t w, int32_t ref) {
  pt_v3 thr = pt_v3f(1.0f, 1.0f, 1.0f);
  if (!(w & kFresh)) {
    const float4 c = q_load(X.c + p);
    thr = pt_v3f(c.x, c.y, c.z);
  }
  pt_v3 col = pt_mul(thr, pt_v3f(fr.bg[0], fr.bg[1], fr.bg[2]));
  if (ref != 0) {
    const float4 e = sc.mats[5 * mat_index(sc, ref) + 1];  // emit colour (Mat::m1)
    col = (e.x > 0.0f || e.y > 0.0f || e.z > 0.0f) ? pt_mul(thr, pt_v3f(e.x, e.y, e.z)) : pt_v3f(0.0f, 0.0f, 0.0f);
  }
  stage(fr, wb, w & ~kFresh, col);
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

// Appends position p to the list of class `list` (-1: none) of this
// iteration, one atomic per wave and non-empty list (one instruction,
// wave_append; call from converged code).
__device__ __forceinline__ void append_list(const WfBufs& wb, int32_t par, int32_t shard, int32_t list, int32_t p) {
  const int32_t k = wave_append<kLists>(list, [&](int32_t l) { return ctl_list(wb, par, l, shard); });
  if (list >= 0 && k < wb.medseg) s_store(list_slot(wb, list, shard, k), p);  // always < medseg: it bounds a shard's rays
}

// intersect_rays, kernels.py:1242-1263, plus the closest-hit classification:
// a miss (shade_miss_rays, kernels.py:1266-1280) or an emissive hit
// (kernels.py:1365-1375) ends its path here; every other traced ray is
// appended to the list of its hit's material class. The work: this
// iteration's continuing rays, segment by segment (each wave reads 64 rays of
// one direction bin, coalesced: item word + o, d = 28 B per ray), then the
// fresh camera rays that fill the pipe back up to `capacity` while the pool
// lasts. Writes the hit record (8 B) and one list entry (4 B) per ray; a path
// end reads thr (16 B) and writes its staging slot.
template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock, stress_waves(isect_min_waves<STACK, TRAV>())) void wf_intersect(DevScene sc, DevFrame fr, WfBufs wb, int32_t par,
                                                       unsigned long long* __restrict__ counters) {
  constexpr int LDS = isect_lds<STACK, TRAV>();
  __shared__ uint2 lds_stack[LDS * kWfBlock];
  const int tid = threadIdx.x;
  Stack st{lds_stack + tid, wb.spill, (uint32_t)(blockIdx.x * kWfBlock + tid) * 8u, gridDim.x * kWfBlock * 8u};
  const RayBuf& X = wb.rb[par];
  const int32_t shard = (int32_t)(blockIdx.x % kShards);
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  const SegTable T = seg_table(wb, par);
  // the pool was empty once the previous iteration's claims were done (the
  // previous wf_scatter looked): then this launch claims nothing, in every
  // wave, and traces exactly the continuing rays
  const bool dry = __builtin_amdgcn_readfirstlane(s_load(ctl_status(wb) + 2)) != 0;
  const int32_t nfresh = dry ? 0 : max(wb.capacity - T.live, 0);
  const int32_t nwork = T.fresh_start + nfresh;
  if (blockIdx.x == 0 && tid == 0) {  // for the host: the rays this launch traces when the pool was empty
    ctl_status(wb)[0] = T.live;
    ctl_status(wb)[1] = dry ? 1 : 0;
  }
  uint32_t n_live = 0, n_ended = 0;
  for (int32_t w0 = __builtin_amdgcn_readfirstlane((int32_t)(blockIdx.x * kWfBlock) + (tid & ~63)); w0 < nwork;
       w0 += stride) {  // (wave-uniform: an SGPR)
    int32_t p = -1;
    uint32_t item = 0u;
    pt_v3 o = pt_v3f(0.0f, 0.0f, 0.0f), d = o;
    if (w0 < T.fresh_start) {  // a continuing ray of a segment or of the overflow region
      p = cont_position(T, wb, w0);
      if (p >= 0) {
        item = s_load(X.item + p);
        const float4 a = q_load(X.a + p);
        const float2 dyz = h_load(X.d + p);
        o = pt_v3f(a.x, a.y, a.z);
        d = pt_v3f(a.w, dyz.x, dyz.y);
      }
    } else {  // generate_camera_rays (kernels.py:1219-1239) for the next work items
      const int32_t f = w0 - T.fresh_start + lane_id();
      const int32_t k = claim_items(wb, shard, f < nfresh);
      if (k >= 0) {
        const Item it = decode_item(fr, wb, (uint32_t)k);
        if (it.valid) {  // (padding items of squares past the frame / batch are skipped)
          Rng rng{path_key(fr, wb, it), 0u};
          get_ray(fr, it.px, it.py, rng, o, d);  // direction left unnormalized (Q1)
          p = fresh_base(wb) + f;
          item = (uint32_t)k | kFresh;
          s_store(X.item + p, item);
        }
      }
    }
    int32_t list = -1;
    if (p >= 0) {
      ++n_live;
      float t = 0.0f;
      int32_t ref = 0;
      const bool hit = traverse<STACK, kWfBlock, TRAV, LDS>(sc, o, d, kTMin, kTMax, st, t, ref);
      if (!hit) ref = 0;  // a miss: no leaf code
      list = hit ? leaf_class(ref) : kListEnded;
      if (list == kListEnded) {
        end_unscattered(sc, fr, wb, X, p, item, ref);
        ++n_ended;
        list = -1;
      } else {
        h_store(X.hit + p, make_float2(t, __int_as_float(ref)));
      }
    }
    append_list(wb, par, shard, list, p);
  }
  if (counters) {
    block_flush<1>({n_live}, lds_stack, counters + 0);
    block_flush<1>({n_ended}, lds_stack, counters + 2);
  }
}

// scatter epilogue of shade_and_scatter (kernels.py:1377-1399) plus the
// per-path wave budget of renderer.py:313: a continuing ray goes to cn (true
// returned). A path it ends is counted in ends[0] (Russian roulette) or
// ends[1] (depth or wave budget).
__device__ __forceinline__ bool scatter_epilogue(const DevFrame& fr, bool scattered, pt_v3 hp, pt_v3 sdir,
                                                 pt_v3 att, const Ray& cur, Rng& r, uint32_t (&ends)[2], Cont& cn) {
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
  cn.o = hp;
  cn.d = sdir;
  cn.thr = nthr;
  cn.item = cur.item;
  cn.ctr = r.n;
  cn.meta = (uint32_t)nd | ((uint32_t)(wave + 1) << 8);
  cn.go = true;
  return true;
}

// Per-lane tail of a path a scatter ended: stage its colour (0 unless it
// ended on an emissive boundary fallback; misses and emissive surface hits
// end in wf_intersect, end_unscattered).
__device__ __forceinline__ void finish_ended(const DevFrame& fr, const WfBufs& wb, const Ray& ray, pt_v3 emit) {
  stage(fr, wb, ray.item,
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

// The ray at position p of the Lambertian, glossy or dielectric list
// (`list`, wave-uniform): shade_and_scatter for a surface hit
// (kernels.py:1359-1399). A continuing ray goes to cn.
__device__ __forceinline__ void shade_entry(const DevScene& sc, const DevFrame& fr, const WfBufs& wb,
                                            const RayBuf& X, int32_t list, int32_t p, uint32_t& n_ended,
                                            uint32_t (&ends)[2], Cont& cn) {
  const float2 h = h_load(X.hit + p);
  const int32_t ref = __float_as_int(h.y);
  Item it;
  const Ray ray = load_ray(fr, wb, X, p, it);
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
  if (!scatter_epilogue(fr, sc_ok, hp, sdir, att, ray, r, ends, cn)) {
    finish_ended(fr, wb, ray, emitted(m));
    ++n_ended;
  }
}

// The ray at position p of the constant-medium list (exit traversal + free
// flight, apply_constant_medium kernels.py:365-450, and the volume branch of
// shade_and_scatter, kernels.py:1326-1357) or, is_noise, of the Perlin list.
// A continuing ray (a scatter, or a passthrough at the same depth) goes to cn.
template <int STACK, int TRAV>
__device__ __forceinline__ void medium_entry(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, Stack st,
                                             const RayBuf& X, int32_t p, bool is_noise, uint32_t& n_ended,
                                             uint32_t (&ends)[2], Cont& cn) {
  bool go = false;
  pt_v3 emit = pt_v3f(0.0f, 0.0f, 0.0f);
  const float2 h = h_load(X.hit + p);
  const int32_t ref = __float_as_int(h.y);
  Item it;
  const Ray ray = load_ray(fr, wb, X, p, it);
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
        cn.o = pt_add(ray.o, pt_scale(ray.d, t_exit + eps_t));
        cn.d = ray.d;
        cn.thr = ray.thr;
        cn.item = ray.item;
        cn.ctr = r.n;
        cn.meta = ray.meta + (1u << 8);
        cn.go = true;
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
  if (!passthrough) go = scatter_epilogue(fr, scattered, hp, sdir, att, ray, r, ends, cn);
  if (!go) {
    finish_ended(fr, wb, ray, emit);
    ++n_ended;
  }
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
// reference's order. The continuing rays go to their direction segments of
// the next iteration's buffer (append_cont).
#ifndef PTMI_WF_SCATTER_MIN_WAVES
// 4 waves/SIMD: <= 128 VGPRs. Round 3 measured 5 waves (96 VGPRs, 72 B/lane
// of scratch) +2.1 % on C3; since the continuing rays are appended by the
// wave (round 5) the 5-wave build spills 148 B/lane (24 scratch stores in the
// loop) and the 4-wave build 52 B: A/B on MI355X, parity-identical, 4 waves
// C3 +2.2 % (1914-1923 vs 1856-1899), mesh fog +3 % (profiles/r05/ab/ab_wf_sort.log).
// Kernels of more than 16 stack slots: their 20+ KB LDS stacks allow no more.
#define PTMI_WF_SCATTER_MIN_WAVES 4
#endif
// The medium waves' LDS stacks cap this kernel at 5 waves/SIMD. A/B on
// MI355X (round 4): split into a medium launch (5 waves) and a launch for the
// Perlin and surface lists without LDS stacks (5 / 6 waves), C3 -4 %
// (profiles/r04/ab/ab_r04i_split_knobs_ruv.log).
constexpr int32_t kScatterOrder[kLists] = {kListMedium, kListNoise, kListLambertian, kListGlossy, kListDielectric};

template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock, stress_waves(PTMI_WF_SCATTER_MIN_WAVES)) void wf_scatter(DevScene sc, DevFrame fr, WfBufs wb,
                                                    int32_t par, unsigned long long* __restrict__ counters) {
  __shared__ uint2 lds_stack[STACK * kWfBlock];
  Stack st{lds_stack + threadIdx.x};
  const RayBuf& X = wb.rb[par];
  const int32_t shard = (int32_t)(blockIdx.x % kShards);
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
  // this iteration's segments were read by its wf_intersect: they start empty
  // for the next wf_scatter's appends (which go to this parity)
  if (blockIdx.x == 0 && threadIdx.x < kSegs) *ctl_seg(wb, par, (int32_t)threadIdx.x) = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctl_ovf(wb, par) = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && counters && num[0] > 0)
    atomicAdd(counters + 1, (unsigned long long)num[0]);  // medium exit traversals
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // every claim of this iteration is done: is the pool empty?
    const bool d = pool_dry(wb);
    if (threadIdx.x == 0) ctl_status(wb)[2] = d ? 1 : 0;
  }
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  uint32_t n_ended = 0, ends[2] = {0u, 0u};
  for (int32_t base = __builtin_amdgcn_readfirstlane((int32_t)(blockIdx.x * kWfBlock) + (int32_t)(threadIdx.x & ~63u));
       base < n; base += stride) {  // (wave-uniform: an SGPR)
    // wave-uniform list of this wave's 64 entries
    int32_t j = base + lane_id(), l = 0;
#pragma unroll
    for (int k = 0; k + 1 < kLists; ++k)
      if (l == k && j >= span[k]) {
        j -= span[k];
        l = k + 1;
      }
    int32_t p = -1;
#pragma unroll
    for (int k = 0; k < kLists; ++k)
      if (l == k && j < num[k]) p = list_entry(wb, kScatterOrder[k], cnt[k], j);
    int32_t lid = kScatterOrder[0];  // this wave's list (wave-uniform select, no indexed table)
#pragma unroll
    for (int k = 1; k < kLists; ++k)
      if (l == k) lid = kScatterOrder[k];
    Cont cn;
    cn.go = false;
    if (p >= 0) {  // (p < 0: the list's padding)
      if (lid == kListMedium || lid == kListNoise)
        medium_entry<STACK, TRAV>(sc, fr, wb, st, X, p, lid == kListNoise, n_ended, ends, cn);
      else
        shade_entry(sc, fr, wb, X, lid, p, n_ended, ends, cn);
    }
    append_cont(wb, par ^ 1, shard, cn);
  }
  if (counters) block_flush<3>({n_ended, ends[0], ends[1]}, lds_stack, counters + 2);
}

#ifndef PTMI_WF_TRACE
#define PTMI_WF_TRACE 0  // diagnostic builds only: record every wf_drain segment (tools/wf_drain_trace.py)
#endif
#if PTMI_WF_TRACE
// One record per segment traced by wf_drain: item, meta and rng counter the
// segment starts with, its closest hit (t, ref), then the continuation
// (go, ctr, meta, thr.xyz) or, for an ended path, its staged colour.
constexpr uint32_t kTraceWords = 12, kTraceCap = 1u << 22;
__device__ uint32_t g_wf_trace_n;
__device__ uint32_t g_wf_trace[kTraceCap * kTraceWords];
#if PTMI_WF_TRACE == 1
__device__ __noinline__
#else
__device__ __forceinline__
#endif
void wf_trace(const DevFrame& fr, const WfBufs& wb, uint32_t item, uint32_t meta,
                                      uint32_t ctr, float t, int32_t ref, uint32_t go, const Cont& cn) {
  const uint32_t k = atomicAdd(&g_wf_trace_n, 1u);
  if (k >= kTraceCap) return;
  uint32_t* r = g_wf_trace + (size_t)k * kTraceWords;
  r[0] = item;
  r[1] = meta;
  r[2] = ctr;
  r[3] = __float_as_uint(t);
  r[4] = (uint32_t)ref;
  r[5] = go;
  if (go) {
    r[6] = cn.ctr;
    r[7] = cn.meta;
    r[8] = __float_as_uint(cn.thr.x);
    r[9] = __float_as_uint(cn.thr.y);
    r[10] = __float_as_uint(cn.thr.z);
  } else {
    const Item it = decode_item(fr, wb, item);
    const float* c = wb.staging + 3 * ((size_t)it.srel * (size_t)wb.npix + (size_t)it.p);
    r[6] = 0xffffffffu;
    r[7] = 0xffffffffu;
    r[8] = __float_as_uint(c[0]);
    r[9] = __float_as_uint(c[1]);
    r[10] = __float_as_uint(c[2]);
  }
  r[11] = 0x7ace0000u | (uint32_t)(threadIdx.x & 63);
}
#endif

// One segment of a tail path at position p: intersect_rays (kernels.py:
// 1242-1263), the classification of wf_intersect and the shading of
// wf_scatter (the same entry functions); the continuing ray is stored back in
// place. Returns whether the path goes on.
template <int STACK, int TRAV>
__device__ __forceinline__ bool drain_segment(const DevScene& sc, const DevFrame& fr, const WfBufs& wb, Stack st,
                                              const RayBuf& X, int32_t p, uint32_t& n_seg, uint32_t& n_med,
                                              uint32_t& n_ended, uint32_t (&ends)[2]) {
  const float4 a = q_load(X.a + p);
  const float2 dyz = h_load(X.d + p);
#if PTMI_WF_TRACE
  const uint32_t tr_item = s_load(X.item + p), tr_meta = __float_as_uint(q_load(X.c + p).w),
                 tr_ctr = s_load(X.ctr + p);
#endif
  float t = 0.0f;
  int32_t ref = 0;
  const bool hit = traverse<STACK, kWfBlock, TRAV>(sc, pt_v3f(a.x, a.y, a.z), pt_v3f(a.w, dyz.x, dyz.y), kTMin,
                                                   kTMax, st, t, ref);
  ++n_seg;
  if (!hit) ref = 0;
  h_store(X.hit + p, make_float2(t, __int_as_float(ref)));
  const int32_t list = hit ? leaf_class(ref) : kListEnded;
  Cont cn;
  cn.go = false;
  if (list == kListEnded) {
    end_unscattered(sc, fr, wb, X, p, s_load(X.item + p), ref);
    ++n_ended;
  } else if (list == kListMedium || list == kListNoise) {
    n_med += list == kListMedium ? 1u : 0u;
    medium_entry<STACK, TRAV>(sc, fr, wb, st, X, p, list == kListNoise, n_ended, ends, cn);
  } else {
    shade_entry(sc, fr, wb, X, list, p, n_ended, ends, cn);
  }
#if PTMI_WF_TRACE
  wf_trace(fr, wb, tr_item, tr_meta, tr_ctr, t, ref, cn.go ? 1u : 0u, cn);
#endif
  if (cn.go) store_ray(X, p, cn);
  return cn.go;  // false: the path ended (its colour is staged)
}

// The tail of a batch (wf_batch switches a pipe to it once the work pool is
// empty and the pipe traces fewer than capacity / drain_at rays per
// iteration): one launch finishes every path still in the pipe, each lane
// looping intersect -> classify -> shade over its own ray until the path
// ends — exactly the per-path steps of wf_intersect and wf_scatter (the same
// entry functions), with the continuing ray stored back in place, so every
// path, its draws, its wave budget (Q14) and the counters are unchanged.
// What changes is the schedule: instead of one intersect and one scatter
// launch per remaining wave (~7.5 us each even when nearly empty, and ~50 of
// them for the longest Russian-roulette survivors), the tail is one launch
// whose length is the longest remaining path. Launched on the pipe's stream
// after a wf_scatter, on the continuing rays of the next iteration's parity:
// the pool is empty, so no fresh ray is due.
#ifndef PTMI_WF_DRAIN_MIN_WAVES
#define PTMI_WF_DRAIN_MIN_WAVES 1
#endif
template <int STACK, int TRAV = PTMI_TRAV_STACK>
__global__ __launch_bounds__(kWfBlock, stress_waves(PTMI_WF_DRAIN_MIN_WAVES)) void wf_drain(DevScene sc, DevFrame fr, WfBufs wb, int32_t par,
                                                   unsigned long long* __restrict__ counters) {
  __shared__ uint2 lds_stack[STACK * kWfBlock];
  Stack st{lds_stack + threadIdx.x};
  const RayBuf& X = wb.rb[par];
  const SegTable T = seg_table(wb, par);
  uint32_t n_seg = 0, n_med = 0, n_ended = 0, ends[2] = {0u, 0u};
  // (the wave's work index is wave-uniform: an SGPR)
  const int32_t stride = (int32_t)(gridDim.x * kWfBlock);
  for (int32_t w0 = __builtin_amdgcn_readfirstlane((int32_t)(blockIdx.x * kWfBlock) + (int32_t)(threadIdx.x & ~63u));
       w0 < T.fresh_start; w0 += stride) {
    const int32_t p = cont_position(T, wb, w0);  // (every lane active: cross-lane reads inside)
    if (p < 0) continue;
    // each lane loops over its own path until it ends
    while (drain_segment<STACK, TRAV>(sc, fr, wb, st, X, p, n_seg, n_med, n_ended, ends)) {
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
// fork/join events of pipes 1.., the status readback events and their
// host-pinned slots [2][kPipes][2]. `mu` serialises ptmi_wf_render calls on
// the device (each call drives all pipes and reads their status back), so
// two host threads rendering on one device never share readback slots; calls
// on different devices run concurrently.
struct PipeStreams {
  std::mutex mu;
  hipStream_t s[kPipes] = {};
  hipEvent_t fork = nullptr, join[kPipes] = {};
  hipEvent_t rb[2][kPipes] = {};  // status readbacks of two consecutive chunks
  int32_t* pinned = nullptr;      // [2][kPipes][2]: rays traced by the chunk's last wf_intersect, pool empty
  bool ok = false;
};
constexpr int kMaxDevices = 64;
PipeStreams g_pipes[kMaxDevices];

// Called with ps->mu held.
hipError_t pipe_streams_init(PipeStreams* ps) {
  if (ps->ok) return hipSuccess;
  hipError_t e = hipSuccess;
  if (!ps->pinned) e = hipHostMalloc((void**)&ps->pinned, 2 * kPipes * 2 * sizeof(int32_t), hipHostMallocDefault);
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
// A pipe that traced fewer than capacity / drain_at rays after the pool ran
// dry finishes its paths in one wf_drain launch (0 = never: one intersect
// and one scatter launch per wave until the pipe is empty). The default;
// ptmi_wf_set_drain_at changes it at run time (tests drive the tail with 1:
// drain as soon as the pool is dry).
#define PTMI_WF_DRAIN_AT 16
#endif
#ifndef PTMI_WF_CAPACITY_LOG2
// rays per iteration (all pipes). A/B: 2^21 +3 % over 2^20 (C3, mesh fog);
// with the 8-wave wf_intersect (late round 5) 2^22 over 2^21: mesh fog +5 %
// (two runs), C3 +1.6 % / +-0 (C3 varies +-1.5 %); 2^23: mesh fog +9 %, C3
// -2 % (profiles/r05/ab/ab_wf_capacity_8waves.log)
#define PTMI_WF_CAPACITY_LOG2 22
#endif
constexpr int32_t kMaxCapacity = 1 << PTMI_WF_CAPACITY_LOG2;
std::atomic<int32_t> g_drain_at{PTMI_WF_DRAIN_AT};
constexpr int32_t kSlotQuantum = kShards * kWfBlock;

// per ray position and parity: a 16, c 16, d 8, hit 8, item 4, ctr 4 bytes
constexpr size_t kPosBytes = 56;
struct Layout {
  int32_t capacity, cp, seg_cap, npos, medseg;
  size_t rb, lists, staging, spill, ctl, total;
  size_t rb_pipe, lists_pipe;
};
constexpr size_t kSpillPipeBytes = (size_t)kSpillSlots * (PTMI_WF_MAX_BLOCKS / kPipes) * kWfBlock * 8;

Layout layout(int32_t npix, int32_t batch) {
  Layout L;
  int64_t items = (int64_t)npix * batch;
  // rays per iteration: 2^22 (or the batch's items if fewer), whatever the
  // frame size — the pool refills the buffers, so a 4K frame needs no more
  // (the ray buffers are 56 B x 12 positions per ray: 2.8 GB at 2^22)
  int64_t cap = kMaxCapacity;
  if (items < cap) cap = items;
  cap = (cap + kPipes * kSlotQuantum - 1) / (kPipes * kSlotQuantum) * (kPipes * kSlotQuantum);
  L.capacity = (int32_t)cap;  // all pipes
  L.cp = (int32_t)(cap / kPipes);
  int64_t sc = ((int64_t)L.cp / PTMI_WF_SEG_DIV + 63) / 64 * 64;
  L.seg_cap = (int32_t)(sc < 64 ? 64 : sc);
  L.npos = kSegs * L.seg_cap + 2 * L.cp;
  // a shard's blocks take every kShards-th 128-entry chunk of wf_intersect's
  // work (<= cp + the bins' and the overflow's padding): a list segment holds them all
  const int64_t work = (int64_t)L.cp + 64ll * (kBins + 1);
  const int64_t chunks = (work + kWfBlock - 1) / kWfBlock;
  L.medseg = (int32_t)((chunks + kShards - 1) / kShards * kWfBlock);
  L.rb_pipe = 2 * kPosBytes * (size_t)L.npos;
  L.lists_pipe = 4 * kShards * sizeof(int32_t) * (size_t)L.medseg;
  L.rb = 0;
  L.lists = L.rb + kPipes * L.rb_pipe;
  L.staging = (L.lists + kPipes * L.lists_pipe + 255) & ~(size_t)255;
  L.spill = (L.staging + 3 * sizeof(float) * (size_t)items + 255) & ~(size_t)255;
  L.ctl = L.spill + kPipes * kSpillPipeBytes;
  L.total = L.ctl + kCtlWords * sizeof(int32_t);
  return L;
}
}  // namespace

static_assert((PTMI_WF_MAX_BLOCKS / kPipes) % kShards == 0, "a pipe's grid must be a multiple of the shard count");

// One batch: generate on the caller's stream, fork the pipes, run each pipe's
// intersect -> scatter loop on its own stream until its rays have all ended
// and the pool is empty, join, resolve.
template <int STACK, int TRAV = PTMI_TRAV_STACK>
static hipError_t wf_batch(const DevScene& sc, const DevFrame& fr, const WfBufs* wbs, float* accum, int32_t batch,
                           unsigned long long* counters, hipStream_t stream, const PipeStreams& ps) {
  // a pipe's grid = a multiple of kShards, so block b's shard is b % kShards
  int64_t blocks = wbs[0].capacity / kWfBlock;
  if (blocks > PTMI_WF_MAX_BLOCKS / kPipes) blocks = PTMI_WF_MAX_BLOCKS / kPipes;
  const unsigned g = (unsigned)blocks;
  // the tail launch: one lane per continuing ray (<= capacity + the bins' padding)
  const unsigned gd = (unsigned)((wbs[0].capacity + 64 * (kBins + 1) + kWfBlock - 1) / kWfBlock);
  (void)hipMemsetAsync(wbs[0].next, 0, kCtlWords * sizeof(int32_t), stream);
  {
    const int pslot = prof_begin(kProfWfGenerate, stream);
    hipLaunchKernelGGL(wf_generate, dim3(1), dim3(64), 0, stream, wbs[0]);
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
  // live ray by one wave (or starts a new item), so this many iterations
  // always drain a pipe.
  const int64_t max_iters = (int64_t)wbs[0].nitems * (int64_t)(fr.max_depth > 0 ? fr.max_depth : 1) + 2;
  bool live[kPipes];
  for (int p = 0; p < kPipes; ++p) live[p] = true;
  int64_t it = 0;
  const int32_t chunk = PTMI_WF_RB_CHUNK;  // iterations between status readbacks
  const int64_t drain_at = g_drain_at.load(std::memory_order_relaxed);
  hipError_t err = hipSuccess;
  // The host reads chunk k's status only after chunk k + 1 is queued, so the
  // pipes never idle through the readback's host round trip. Iterations on a
  // drained pipe are no-ops (no ray left, no item to claim), so the one extra
  // chunk a pipe may run after draining changes nothing.
  bool inflight[2][kPipes] = {};
  int cur = 0;
  while (it < max_iters) {
    const int64_t n = max_iters - it < chunk ? max_iters - it : chunk;
    for (int64_t j = 0; j < n; ++j) {
      for (int p = 0; p < kPipes; ++p) {
        if (!live[p]) continue;
        const WfBufs& wb = wbs[p];
        const int32_t par = (int32_t)((it + j) & 1);  // which ray buffer and list counters this iteration uses
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
      err = hipMemcpyAsync(ps.pinned + (cur * kPipes + p) * 2, ctl_status(wbs[p]), 2 * sizeof(int32_t),
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
        const int32_t traced = ps.pinned[(prev * kPipes + p) * 2], dry = ps.pinned[(prev * kPipes + p) * 2 + 1];
        // the pool was empty before that iteration began, so it claimed no
        // item and traced only its continuing rays: none means the pipe is done
        if (dry && traced == 0) live[p] = false;
        if (live[p] && dry && drain_at > 0 && (int64_t)traced * drain_at < (int64_t)wbs[p].capacity) {
          // few paths left and no work to add: finish them in one launch,
          // queued behind the iterations in flight, on the rays the next
          // iteration would trace
          const int pd = prof_begin(kProfWfDrain, st[p]);
          hipLaunchKernelGGL((wf_drain<STACK, TRAV>), dim3(gd), dim3(kWfBlock), 0, st[p], sc, fr, wbs[p],
                             (int32_t)(it & 1), counters);
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

#if PTMI_WF_TRACE
}  // namespace ptmi
// Diagnostic builds: copy up to max_records wf_drain segment records to out
// (kTraceWords uint32 each) and return how many were recorded; reset clears.
extern "C" int64_t ptmi_wf_trace_read(uint32_t* out, int64_t max_records, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  uint32_t n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(ptmi::g_wf_trace_n), sizeof(n)) != hipSuccess) return -1;
  const int64_t k = (int64_t)(n < ptmi::kTraceCap ? n : ptmi::kTraceCap);
  const int64_t m = k < max_records ? k : max_records;
  if (m > 0 && out &&
      hipMemcpyFromSymbol(out, HIP_SYMBOL(ptmi::g_wf_trace), (size_t)m * ptmi::kTraceWords * sizeof(uint32_t)) !=
          hipSuccess)
    return -1;
  if (reset) {
    n = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(ptmi::g_wf_trace_n), &n, sizeof(n)) != hipSuccess) return -1;
  }
  return (int64_t)n;
}
namespace ptmi {
#endif

size_t wf_workspace_bytes(int32_t npix, int32_t batch) {
  if (npix <= 0 || batch <= 0) return 0;
  return layout(npix, batch).total;
}

hipError_t wf_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws, size_t ws_bytes,
                     float* accum, int32_t s_begin, int32_t s_count, unsigned long long* counters,
                     hipStream_t stream) {
  const int32_t npix = fr.w * fr.n_rows;
  // work items (sample, pixel) of a batch are ids below 2^31 (FastDiv's
  // range, and the kFresh bit), padded ids included: 64 per 8x8 pixel square,
  // and the batch's samples rounded up to whole chunks (wb.nitems below); the
  // pool counters may run past their shard's end by the lanes asking at once
  // (< 2^24 in all)
  const int64_t sq_items = 64ll * ((fr.w + 7) / 8) * ((fr.n_rows + 7) / 8);
  int32_t batch = s_count;
  const int64_t max_batch = sq_items > 0 ? (0x7fffffffll - (1ll << 24)) / sq_items - (PTMI_WF_CHUNK_SAMPLES - 1) : 0;
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
    const size_t np = (size_t)L.npos;
    WfBufs wbs[kPipes];
    for (int p = 0; p < kPipes; ++p) {
      WfBufs& wb = wbs[p];
      char* rbp = base + L.rb + p * L.rb_pipe;
      for (int q = 0; q < 2; ++q) {
        char* r = rbp + q * kPosBytes * np;
        wb.rb[q].a = (float4*)r;
        wb.rb[q].c = (float4*)(r + 16 * np);
        wb.rb[q].d = (float2*)(r + 32 * np);
        wb.rb[q].hit = (float2*)(r + 40 * np);
        wb.rb[q].item = (uint32_t*)(r + 48 * np);
        wb.rb[q].ctr = (uint32_t*)(r + 52 * np);
      }
      wb.lists = (int32_t*)(base + L.lists + p * L.lists_pipe);
      wb.staging = (float*)(base + L.staging);
      wb.next = (int32_t*)(base + L.ctl);
      wb.ctl = wb.next + (8 + p * kPipeLines) * kLine;
      wb.spill = base + L.spill + p * kSpillPipeBytes;
      wb.capacity = L.cp;
      wb.seg_cap = L.seg_cap;
      wb.medseg = L.medseg;
      wb.npix = npix;
      wb.sq_x = (fr.w + 7) / 8;
      wb.nsq = wb.sq_x * ((fr.n_rows + 7) / 8);
      wb.batch = nb;
      wb.csamp = nb < PTMI_WF_CHUNK_SAMPLES ? nb : PTMI_WF_CHUNK_SAMPLES;
      const int32_t nchunks = wb.nsq * ((nb + wb.csamp - 1) / wb.csamp);
      wb.nitems = nchunks * 64 * wb.csamp;
      wb.shard_len = (nchunks + kShards - 1) / kShards * 64 * wb.csamp;
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
