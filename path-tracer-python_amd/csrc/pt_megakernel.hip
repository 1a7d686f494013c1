// pt_megakernel.hip — depth-first integrator for gfx950.
//
// Replaces kernels.render_sample (kernels.py:1177-1202) + trace_ray
// (kernels.py:1025-1170). Design (MI355X-first, not a translation):
//   * one thread owns one pixel for a whole batch of samples and regenerates
//     the next camera path as soon as the previous one ends, so a wave keeps
//     all 64 lanes busy across path-length variance instead of idling until
//     its longest path of a sample finishes;
//   * every loop iteration runs ONE traversal for every active lane; the
//     constant-medium exit search (kernels.py:417) is not a nested second
//     traversal but its own iteration (mode MEDIUM_EXIT), so lanes doing it
//     share the traversal code with lanes tracing ordinary segments;
//   * direct mode: the accumulator is read once and written once per launch
//     (sample colours added in sample order in registers: same float
//     sequence as accum += color per sample);
//   * staged mode (the default for multi-sample calls): persistent waves
//     draw (8x8 tile, sample) units from sharded counters, so the launch
//     does not end in a long partially-filled last round of blocks; each
//     path writes its colour to staging[sample][pixel] and stage_resolve
//     adds them in sample order — the same float additions as direct mode;
//   * BVH: child-box BVH2 nodes (80 B, one node load tests both children),
//     traversal stack in LDS (slot-major, conflict-free), see pt_device.hpp.
// Perlin corner loop fully unrolled here (A/B on MI355X: +2.5 % megakernel,
// where it costs no occupancy); the wavefront shade kernel keeps it rolled.
#ifndef PTMI_PERLIN_UNROLL
#define PTMI_PERLIN_UNROLL 2
#endif
#include "pt_launch.hpp"
#include "pt_prof.hpp"

namespace ptmi {

enum : int32_t { kModeTrace = 0, kModeMediumExit = 1 };

struct PathState {
  pt_v3 o, dir, thr, color;
  Rng rng;
  int32_t depth;     // the reference's loop variable `depth` (kernels.py:1054)
  int32_t mode;
  float t_entry;     // medium boundary hit (mode MEDIUM_EXIT)
  int32_t ref_entry;
};

__device__ __forceinline__ void start_path(const DevFrame& fr, int32_t px, int32_t py, int32_t s,
                                           PathState& ps) {
  ps.rng.key = pt_path_key(fr.seed, (uint32_t)(py * fr.width + px), (uint32_t)s);
  ps.rng.n = 0;
  pt_v3 d;
  get_ray(fr, px, py, ps.rng, ps.o, d);
  ps.dir = pt_normalize(d);  // Q1: kernels.py:1042
  ps.thr = pt_v3f(1.0f, 1.0f, 1.0f);
  ps.color = pt_v3f(0.0f, 0.0f, 0.0f);
  ps.depth = 0;
  ps.mode = kModeTrace;
  ps.t_entry = 0.0f;
  ps.ref_entry = 0;
}

#ifndef PTMI_MK_SHADE_AT
// Shade once at most this many lanes are still mid-traversal. With leaf
// deferral (PTMI_MK_DEFER 12): 24 > 20 > 16 (C2 +1.7 % / +1 %; C4 +1.4 %);
// before it 12 ~ 16 > 10 > 8 >> 4 with the traversal priority, 8 > 16 > 24 > 0
// without (profiles/r03/ab/ab_leaf_defer.log, profiles/r01/ab_prio_shade_at.log).
#define PTMI_MK_SHADE_AT 24
#endif

#ifndef PTMI_MK_STEP_UNROLL
#define PTMI_MK_STEP_UNROLL 4  // A/B: 3 pops per header pass +1.9 % C2, +2.6 % C4 over 1 (round 1; 2: +1.5 %, 4: +1.6 %); round 4, with the 4-load node visits: 4 over 3 C2 +0.8 %, C5 +0.5 %, C4 +0.2 % (profiles/r04/ab/ab_r04su_step_unroll.log)
#endif

#ifndef PTMI_MK_PRIO_TRAV
// Wave priority (s_setprio) in the traversal loop and in shading: a wave in its
// latency-bound traversal steps wins VALU issue over one in shading, so its
// next node load goes out sooner (A/B with SHADE_AT 12: C2 +1.3 %, C4 +4 %,
// C5 +1.4 %; the reverse order -1 %; profiles/r01/ab_prio_shade_at.log).
// -1 = no s_setprio.
#define PTMI_MK_PRIO_TRAV 2
#endif
#ifndef PTMI_MK_PRIO_SHADE
#define PTMI_MK_PRIO_SHADE 1
#endif
#ifndef PTMI_MK_PRIO_DRAIN
// Traversal priority of a persistent wave whose units have run out: its
// drain, the longest of its remaining paths, runs with ~21 % of its lanes
// live and issues every instruction for them (probe, tools/drain_probe.py:
// 12 % of the waves' cycles in an 8-GPU tile shard's 5 M-sample call, 1.7 %
// in a whole-frame 64-spp call). Below shading and every fuller wave's
// traversal, it takes the issue cycles they leave. A/B on MI355X
// (parity-identical; traversal 2 / shading 1 / drain 0 against 1 / 0 / 1):
// C2 +2 %, C4 +2 %, whole frame at 64 spp per call +2.9 %, an 8-rank tile
// shard +2.7 %; drain 0 with traversal 1 / shading 0: +1.7 %, C4 -0.6 %
// (profiles/r05/ab/ab_mk_prio_drain.log). Handing the drained waves' paths
// to a second launch instead (full waves, the rest of the chip free) lost 2
// to 8 %: that launch waits behind the next overlapped call's persistent
// waves (profiles/r05/ab/ab_mk_handover.log). -1: PTMI_MK_PRIO_TRAV.
#define PTMI_MK_PRIO_DRAIN 0
#endif
// (A/B, round 5, not kept: a draining wave's shading at its own priority,
// and full waves' traversal above the others', profiles/r05/ab/.)
// A/B, not kept (profiles/): Perlin-textured hits held until 4 or 8 of a wave
// are ready, -1 to -1.5 % (r01/ab_mk_hold_noise.log); non-temporal staging
// stores, +-0.3 % (r02/ab/ab_nontemporal.log); one random_unit_vector site per
// shading round (the wavefront's wf_scatter keeps it), C2 -1.1 %
// (r02/ab/ab_one_scatter.log); the unit fetch's shard loop kept rolled,
// -0.6 to -1.1 % (r02/ab/ab_mk_fetch_rolled.log).
// Staged mode keeps the path's staging slot, computed when its item is bound,
// in a register instead of decoding the item again when the path ends (A/B:
// C2 +0.8 %, C4 +1 %; profiles/r02/ab/ab_one_scatter.log). Lanes continuing
// a path and lanes starting one (refill) mark need_seg and begin together
// after the refill: one trav_begin call site per pass of the outer loop
// instead of two divergent copies (3 divisions + the root slab) in one
// shading round (C2 +1.6 %, C4 +2.3 %; profiles/r02/ab/ab_mk_one_begin.log).
#ifndef PTMI_MK_DEFER
// Leaf deferral (trav_step's DEFER, pt_device.hpp) at this many lanes: C2
// +7.5 %, C5 +6.3 %, C4 +8 % with the shading threshold at 24 (0 = off).
#define PTMI_MK_DEFER 12
#endif
// A/B, not kept (round 4): shading-round deferral by material kind (a lane
// whose segment needs an expensive kind of shading waits until 4 / 8 / 12 /
// 16 lanes need the same kind): C2 -0.5 %, C4 -1 %
// (profiles/r04/ab/ab_r04i_split_knobs_ruv.log, ab_wf_layout_drain_mk_shade_defer.log).
// One random_unit_vector call site per shading round (scatter_begin /
// scatter_end, pt_device.hpp) for the medium scatter, metal fuzz and
// isotropic, instead of three divergent copies of the rejection loop: the
// loop then runs once, to the wave's longest lane. A/B on MI355X (round 4,
// parity-identical): C4 +2.1 %, C2 +-0.3 % (profiles/r04/ab/ab_r04i_split_knobs_ruv.log;
// round 2 measured C2 -1.1 % with the code of the time).
// ... and that site in wave-uniform code, the wave sharing the loop
// (random_unit_vector_wave, pt_device.hpp).
// Turbulence of a shading round's Perlin-textured hits by the whole wave
// (perlin_turb3_wave, pt_device.hpp). Ablation on MI355X (round 4, textures
// replaced by constants, not parity): without the Perlin evaluation C2 +5 %,
// C5 +4.8 %; without the image lookup +1.2 % (profiles/r04/ab/ab_r04l_texture_ablation.log).
#ifndef PTMI_MK_MIN_WAVES
#define PTMI_MK_MIN_WAVES 4  // 4 waves/SIMD: <= 128 VGPRs, no spills (gfx950 hipcc 7.2)
#endif
// Staged kernels for leaf depth 16-18 (17-19 slots, e.g. C4's torus BVH) get
// exactly the slots they need instead of the 20-slot kernel, and the 5-wave
// VGPR budget: 17 slots leave LDS for 18 one-wave blocks per CU instead of 16.
// A/B on MI355X, C4 (leaf depth 16), parity-identical: 1357 -> 1414 Msamples/s
// (+4.2 %; profiles/r02/ab/ab_exact_stack.log).
#ifndef PTMI_MK_MIN_WAVES_16
// 16-slot kernels (leaf depth <= 15, e.g. vol2): 16 * 8 B * 64 lanes * 20
// waves fill the 160 KiB LDS, and without SLP vectorization (Makefile) the
// kernel fits 96 VGPRs with no spills, so 5 waves/SIMD (A/B on MI355X,
// parity-identical: C2 +0.5 % over the 4-wave 20-slot kernel;
// profiles/r02/ab/ab_no_slp.log). With SLP on it spilled 148 B/lane: -20 %.
#define PTMI_MK_MIN_WAVES_16 5
#endif

// One-wave blocks, each an 8x8 pixel tile (A/B on MI355X: +7 % C2 / +12 % C4
// over 4-wave 16x16 blocks: a finished wave frees its slot at once).
constexpr int kMkBlock = 64;

// Staged mode, persistent waves: the grid is one round of the chip's wave
// slots and every wave draws 64-item units (one 8x8 tile x one sample) from a
// device counter and refills its lanes across units — no wave ends while work
// is left, and there is no partly empty last round. Units are tile-major (all
// samples of a tile are consecutive), and a fetch takes up to
// PTMI_MK_CHUNK_SAMPLES units while plenty are left, fewer in the tail, so a
// wave changes tile rarely (lanes of two tiles in one wave fetch more distinct
// cache lines per load) and the last fetches are small.
#ifndef PTMI_MK_CHUNK_SAMPLES
#define PTMI_MK_CHUNK_SAMPLES 32  // A/B (C2, C4): 32/4 ~ 16/4 ~ 64/4 > 16/2, 16/8, 8/4 >> 64/2
#endif
#ifndef PTMI_MK_TAIL_DIV_SMALL
#define PTMI_MK_TAIL_DIV_SMALL 2  // ... for batches of fewer than PTMI_MK_SMALL_BATCH samples
#endif
#ifndef PTMI_MK_SMALL_BATCH
#define PTMI_MK_SMALL_BATCH 8000000
#endif
#ifndef PTMI_MK_SMALL_WPC
// Persistent waves per CU for a batch of fewer than PTMI_MK_SMALL_GRID_BATCH
// samples (the occupancy allows 20 for vol2): the next overlapped call's waves
// share the chip while this one drains. A/B on MI355X, an 8-rank tile shard's
// 64-spp calls against 20 waves per CU: 10 +1.1 %, 12 +0.6 %, 14 +0.5 %, 16
// -0.6 %, 8 -4 %, 6 -29 % (profiles/r06/ab/mk_small_grid.log; round 5:
// profiles/r05/ab/ab_mk_persist_wpc.log).
#define PTMI_MK_SMALL_WPC 10
#endif
#ifndef PTMI_MK_SMALL_GRID_BATCH
// Batches (samples) below which PTMI_MK_SMALL_WPC applies: 16 M covers the
// 4-rank tile shard (10.2 M samples per 64-spp call: +0.7 % over the full
// grid) and leaves 2-rank shards (20.5 M) and whole frames on the full grid
// (profiles/r06/ab/mk_small_grid.log).
#define PTMI_MK_SMALL_GRID_BATCH 16000000
#endif
#ifndef PTMI_MK_TAIL_DIV
#define PTMI_MK_TAIL_DIV 4  // a fetch takes at most (units left) / (TAIL_DIV * waves) units
                            // (re-tuned: 2 is +3 % on C2 but -8 % on C4's long fog paths;
                            // profiles/r01/ab_fetch_sizing.log)
#endif

// Unit counters: the units are split into PTMI_MK_SHARDS contiguous shards,
// each with its own counter on its own 256-B line, and wave w pulls from shard
// w % PTMI_MK_SHARDS first (one shard per XCD under round-robin placement),
// then steals from the others. One device-scope counter saturates near 88
// returning atomics per us (MI355X_MICROARCH.md, "dequeue"), and a launch
// makes ~10^5 fetches, most of them small ones in its tail, where every wave
// is waiting for its next unit.
#ifndef PTMI_MK_SHARDS
#define PTMI_MK_SHARDS 8
#endif
// Shard s holds tiles s, s + S, s + 2S, ... (interleaved across the image, so
// every shard costs about the same; 0: contiguous unit ranges, whose shards
// drain at different times). A/B on MI355X, C2, 64-spp calls (overlapped):
// one counter 2448 (2479), 8 contiguous shards 2320 (2546), 8 interleaved
// 2560 (2597), 4 interleaved 2552 (2590) Msamples/s; 16-spp calls 1954 ->
// 2324 (profiles/r02/ab/ab_mk_shards.log).
constexpr int kMkShards = PTMI_MK_SHARDS;
constexpr int kMkCtlLine = 64;  // int32 words per 256-B counter line

struct MkWork {
  int32_t* ctl;      // kMkShards counters, one per 256-B line: units taken from each shard (zeroed before the launch)
  int32_t shard_len; // units per shard (the last one may be short)
  int32_t csamp;     // most units per fetch
  int32_t tiles_x;   // 64-pixel tiles per row
  int32_t tw_log2;   // tile width log2: 3 for 8x8 tiles, 4 for 16x4, 5 for 32x2, 6 for 64x1
  int32_t nb;        // samples of the batch (units per tile)
  FastDiv by_nb, by_tiles_x, by_len;
  int32_t nunits;    // units of the batch (multiple of csamp)
  int32_t tail_div;  // TAIL_DIV * waves of the grid
};
constexpr int kMkTile = 8;

// Tile height (log2) of the staged megakernel's 64-pixel tiles. A frame's
// local rows are its row bands packed together, so an 8x8 tile over 4-row
// bands (bench.py --gpus 8 at 800 rows) would cover two runs of 4 image rows
// 32 rows apart; a tile as tall as the band's largest power-of-two divisor
// (16x4, 32x2, 64x1) stays inside one band. Which lane renders which pixel
// changes nothing in the image (staging[sample][pixel], ordered resolve).
static int mk_tile_rows_log2(const DevFrame& fr) {
  if (fr.band_stride <= 1) return 3;
  const int32_t th = fr.band_rows & -fr.band_rows;
  return th >= 8 ? 3 : th >= 4 ? 2 : th >= 2 ? 1 : 0;
}
static int64_t mk_tiles(const DevFrame& fr, int32_t* tx_out = nullptr) {
  const int hl = mk_tile_rows_log2(fr), tw = 64 >> hl, th = 1 << hl;
  const int64_t tx = (fr.w + tw - 1) / tw, ty = (fr.n_rows + th - 1) / th;
  if (tx_out) *tx_out = (int32_t)tx;
  return tx * ty;
}

template <int STACK, bool STAGED, int TRAV = PTMI_TRAV_STACK>
// waves/SIMD the LDS stack allows: 160 KiB / (STACK * 8 B * 256) blocks per CU
// (16 -> 5, 20 -> 4, 24 -> 3, 32 -> 2), and the VGPR budget of that many
// waves (96 at 5, 128 at 4).
// TRAV = PTMI_TRAV_STACKLESS (STACK 1: no stack) walks the reference's
// stackless traversal instead (TravSL, pt_device.hpp).
__global__ __launch_bounds__(kMkBlock, stress_waves(STACK < 20 ? PTMI_MK_MIN_WAVES_16 : STACK <= 20 ? PTMI_MK_MIN_WAVES : 1)) void mk_render_kernel(
    DevScene sc, DevFrame fr, float* __restrict__ accum, int32_t s_begin, int32_t s_count, int32_t chunk,
    float* __restrict__ staging, unsigned long long* __restrict__ counters, MkWork wk) {
  constexpr bool kPersist = STAGED;  // staged launches are persistent
  const float4* nodes = sc.nodes;
  {  // node base pinned in an SGPR pair for the whole kernel: under SGPR
     // pressure the compiler otherwise re-loads it from the kernarg segment on
     // every traversal step (s_load + lgkmcnt wait on the pop's critical path)
    const uint64_t nb = (uint64_t)nodes;
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)nb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(nb >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    nodes = (const float4*)(((uint64_t)hi << 32) | lo);
  }
  __shared__ uint2 lds_stack[STACK * kMkBlock];
  const int tid = threadIdx.x;
  Stack st{lds_stack + tid};

  // each wave renders an 8x8 pixel square (square footprints keep a wave's
  // camera rays coherent in the BVH)
  const int lane = tid & 63;
  const int32_t sq_x = fr.x0 + (int32_t)blockIdx.x * kMkTile;  // the wave's square
  const int32_t sq_y = (int32_t)blockIdx.y * kMkTile;          // (local rows)
  const size_t npix = (size_t)fr.w * (size_t)fr.n_rows;
  const pt_v3 bg = pt_v3f(fr.bg[0], fr.bg[1], fr.bg[2]);
  uint32_t n_seg = 0, n_med = 0, n_paths = 0;  // per-thread counts of one launch
  uint32_t n_rr = 0, n_cap = 0;                 // paths ended by Russian roulette / by the depth cap
  PathState ps;

  // Work of the wave. Direct mode: lane L owns pixel L of the square for all
  // samples of the call (its accumulator lives in registers). Staged mode:
  // the wave's (sample, pixel) items are handed out to lanes as their paths
  // end (ballot + mbcnt), so all 64 lanes stay busy until the wave's last few
  // paths; any lane may render any item, because colours go to
  // staging[sample][pixel].
  const int32_t s0 = s_begin, ns = s_count;
  const uint32_t total = 64u * (uint32_t)ns;
  uint32_t next = 64u;  // wave-uniform: next unassigned item
  uint32_t item = (uint32_t)lane;
  uint32_t wend = 0u;   // persistent: end of the wave's current units (items)
  bool drained = false; // persistent: the batch's units are all handed out
  int32_t px = 0, py = -1, lr = 0, s = s0;
  uint32_t slot = 0u;  // staging slot of the bound item
  float* ap = nullptr;
  pt_v3 acc = pt_v3f(0.0f, 0.0f, 0.0f);
  bool live = false;
  // item -> tile origin (x, local row) and sample; persistent items are
  // unit-major: unit u = chunk u / csamp (tile chunk % ntiles, sample block
  // chunk / ntiles), sample u % csamp of the block
  struct Loc {
    int32_t x, row, s;  // tile origin (image x, local row), sample
  };
  auto locate = [&](uint32_t k) -> Loc {
    if (kPersist) {
      // shard-contiguous unit numbering: shard s holds tiles s, s + S, s + 2S, ...
      const uint32_t v = k >> 6, sh = fdiv(v, wk.by_len), j = v - sh * (uint32_t)wk.shard_len;
      const uint32_t tq = fdiv(j, wk.by_nb), t = tq * (uint32_t)kMkShards + sh, ty = fdiv(t, wk.by_tiles_x);
      return Loc{fr.x0 + ((int32_t)(t - ty * (uint32_t)wk.tiles_x) << wk.tw_log2), (int32_t)ty << (6 - wk.tw_log2),
                 s_begin + (int32_t)(j - tq * (uint32_t)wk.nb)};
    }
    return Loc{sq_x, sq_y, s0 + (int32_t)(k >> 6)};
  };
  auto bind = [&](uint32_t k) -> bool {  // item -> pixel/sample; false if outside the frame / batch
    const int32_t p = (int32_t)(k & 63u);
    const Loc l = locate(k);
    s = l.s;
    const int twl = kPersist ? wk.tw_log2 : 3;
    px = l.x + (p & ((1 << twl) - 1));
    lr = l.row + (p >> twl);
    py = (lr < fr.n_rows && px < fr.x0 + fr.w && s < s_begin + s_count) ? frame_row(fr, lr) : -1;
    if (STAGED) slot = (uint32_t)(s - s_begin) * (uint32_t)npix + (uint32_t)lr * (uint32_t)fr.w + (uint32_t)(px - fr.x0);
    return py >= 0;
  };
  if (kPersist) {  // first units of the wave
    next = 0u;
    item = 0xffffffffu;
  }
  if (!kPersist && item < total && bind(item)) {
    if (!STAGED) {
      ap = accum + 3 * ((size_t)py * (size_t)fr.width + (size_t)px);
      acc = pt_v3f(ap[0], ap[1], ap[2]);
    }
    start_path(fr, px, py, s, ps);
    live = true;
  }
  __syncthreads();

  // Traversal of the current segment: begun when the segment starts and then
  // advanced one pop at a time. The wave keeps stepping traversals while more
  // than PTMI_MK_SHADE_AT lanes are still mid-traversal; then the lanes whose
  // traversal has finished shade (and begin their next segment or take a new
  // item) while the stragglers wait with their traversal state kept — instead
  // of the whole wave idling until its longest traversal ends (node steps ran
  // at ~35 % SIMD efficiency that way). 0 = wait for every lane.
  typename TravOf<TRAV>::T tr;
  tr.init(st);
  bool trav = false;  // a segment is in flight (traversal running or result pending)
  bool need_seg = false;  // begin a segment after this pass's refill
  auto begin_segment = [&]() {
    const bool em = ps.mode == kModeMediumExit;
    trav_begin<STACK, kMkBlock>(sc, tr, st, ps.dir, ps.o, em ? ps.t_entry + 0.0001f : kTMin, kTMax);  // :418/:1057
    if (em) ++n_med; else ++n_seg;
    trav = true;
  };
  if (live) begin_segment();

#if PTMI_PROBE == 4
  // shading-round probe (diagnostic build, tools/probe.py --sections): wave
  // cycles per section of the outer loop
  uint64_t p4[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t p4_t = __builtin_amdgcn_s_memtime();
#define PT_P4(k)                                        \
  {                                                     \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    p4[k] += t_ - p4_t;                                 \
    p4_t = t_;                                          \
  }
#else
#define PT_P4(k)
#endif
#if PTMI_PROBE == 3
  // drain probe (diagnostic build, tools/drain_probe.py): a persistent wave's
  // cycles, its cycles after the batch's units ran out for it, and live-lane x
  // cycles in them
  const uint64_t dr_t0 = __builtin_amdgcn_s_memtime();
  uint64_t dr_tdry = 0, dr_prev = 0, dr_lanecyc = 0;
  bool dr_dry = false;
#endif
#if PTMI_PROBE == 2
  // wave-level probe (diagnostic build): shader cycles in the traversal-step
  // loop and in shading/refill; wave steps and the branches they ran
  uint64_t pr_trav = 0, pr_shade = 0, pr_steps = 0, pr_sph = 0, pr_oth = 0, pr_node = 0, pr_both = 0, pr_busy = 0;
  uint64_t pr_t = __builtin_amdgcn_s_memtime();
#endif
  for (;;) {
#if PTMI_MK_PRIO_TRAV >= 0
#if PTMI_MK_PRIO_DRAIN >= 0
    if (kPersist && drained && next >= wend)  // a draining wave: its few live lanes yield issue to full waves
      __builtin_amdgcn_s_setprio(PTMI_MK_PRIO_DRAIN);
    else
#endif
      __builtin_amdgcn_s_setprio(PTMI_MK_PRIO_TRAV);
#endif
    for (;;) {  // traversal steps
      // a lane's stack is empty unless its segment is mid-traversal (busy => trav)
      const unsigned long long mbusy = pt_ballot(tr.busy());
      // 32-bit halves: a 64-bit popcount is compared with a VALU v_cmp_u64
      const uint32_t nbusy = __builtin_popcount((uint32_t)mbusy) + __builtin_popcount((uint32_t)(mbusy >> 32));
      if (nbusy == 0) break;
      if (nbusy <= (uint32_t)PTMI_MK_SHADE_AT && pt_ballot(trav && !tr.busy()) != 0ull) break;
#if PTMI_PROBE == 2
      tr.probe = 0;
#endif
      // PTMI_MK_STEP_UNROLL pops per pass of the loop header (its busy count
      // and shading test sit on every wave's serial chain)
#pragma unroll
      for (int u = 0; u < PTMI_MK_STEP_UNROLL; ++u)
        // the first pop's busy lanes are the header's mask, not a second
        // compare (A/B: +0.8 %, profiles/r05/ab/ab_step_flat.log)
        if (u == 0 ? __builtin_amdgcn_inverse_ballot_w64(mbusy) : tr.busy())
          trav_step<STACK, kMkBlock, PTMI_MK_DEFER>(sc, nodes, tr, st, ps.o, ps.dir);
#if PTMI_PROBE == 2
      ++pr_steps;
      pr_sph += pt_ballot(tr.probe & 1) ? 1 : 0;
      pr_oth += pt_ballot(tr.probe & 2) ? 1 : 0;
      pr_node += pt_ballot(tr.probe & 4) ? 1 : 0;
      pr_both += (pt_ballot(tr.probe & 1) && pt_ballot(tr.probe & 2)) ? 1 : 0;
      pr_busy += nbusy;
#endif
    }
#if PTMI_PROBE == 2
    {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      pr_trav += t - pr_t;
      pr_t = t;
    }
#endif
#if PTMI_MK_PRIO_TRAV >= 0
    __builtin_amdgcn_s_setprio(PTMI_MK_PRIO_SHADE);
#endif
    PT_P4(0)  // traversal steps
    const bool shade_now = trav && !tr.busy();
    // Perlin-textured surface hits of this round: their turbulence by the
    // whole wave (perlin_turb3_wave), before the divergent shading below
    const bool pn = shade_now && ps.mode != kModeMediumExit && tr.any() && leaf_class(tr.best) == PTMI_CLASS_NOISE;
    float pturb = 0.0f;
    if (pt_ballot(pn) != 0ull) pturb = perlin_turb3_wave(sc, pn, pt_add(ps.o, pt_scale(ps.dir, tr.closest)), lane);
    // Shading, in two halves around the round's one random_unit_vector site
    // (medium scatter, metal fuzz, isotropic), which runs in wave-uniform code
    // so that the wave can share its rejection loop (random_unit_vector_wave).
    bool done = false, scattered = false, passthrough = false, to_medium = false;
    pt_v3 hp = pt_v3f(0.0f, 0.0f, 0.0f), sdir = hp, att = hp, n = hp;
    int32_t ruv = kRuvNone, sref = 0;
    float4 m0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // the metal's albedo and fuzz (scatter_end)
    PT_P4(1)  // wave turbulence
    if (shade_now) {  // segment traced: shade it
      trav = false;
      const bool exit_mode = ps.mode == kModeMediumExit;
      const bool hit = tr.any();
      const float t = tr.closest;
      const int32_t ref = tr.best;
      int32_t g = -1;
      if (!exit_mode) {
        if (!hit) {
          ps.color = pt_add(ps.color, pt_mul(ps.thr, bg));  // kernels.py:1164-1168
          done = true;
        } else {
          g = mat_index(sc, ref);
          if (leaf_class(ref) == PTMI_CLASS_MEDIUM) {  // medium boundary (class in the leaf code): exit search next
            ps.mode = kModeMediumExit;
            ps.t_entry = t;
            ps.ref_entry = ref;
            to_medium = true;
          }
        }
      } else {
        g = mat_index(sc, ps.ref_entry);
      }
      if (g >= 0 && !to_medium) {
        const Mat m = load_mat(sc, g);
        bool surface = !exit_mode;
        sref = ref;
        float st = t;
        if (exit_mode) {
          ps.mode = kModeTrace;
          float t_exit;
          pt_v3 mp;
          // apply_constant_medium, kernels.py:421-448 (density m3.w)
          if (medium_step(hit, t, ps.t_entry, m.m3.w, ps.o, ps.dir, ps.rng, mp, t_exit)) {
            hp = mp;  // kernels.py:1082-1097
            ruv = kRuvMedium;
            att = pt_v3f(m.m4.x, m.m4.y, m.m4.z);
            scattered = true;
          } else if (t_exit > 0.0f) {  // kernels.py:1100-1110
            passthrough = true;
            float rl = sqrtf(pt_dot(ps.dir, ps.dir));
            float eps_t = 0.001f / rl;
            ps.o = pt_add(ps.o, pt_scale(ps.dir, t_exit + eps_t));
          } else {  // fallback: shade the boundary as a surface, kernels.py:1111-1119
            surface = true;
            sref = ps.ref_entry;
            st = ps.t_entry;
          }
        }
        if (surface) {  // kernels.py:1120-1128
          hp = pt_add(ps.o, pt_scale(ps.dir, st));
          n = hit_normal(sc, sref, hp, ps.dir);
          ps.color = pt_add(ps.color, pt_mul(ps.thr, emitted(m)));  // kernels.py:1123-1124
          ruv = scatter_begin(sc, sref, m, ps.dir, hp, n, ps.rng, sdir, att, scattered, pn && !exit_mode, pturb);
          m0 = m.m0;
        }
      }
    }
    PT_P4(2)  // material, medium step, surface scatter (first half)
    // one random_unit_vector site per round: medium, metal fuzz, isotropic
    if (pt_ballot(ruv != kRuvNone) != 0ull) {
      const RuvOut ro = random_unit_vector_wave(ps.rng.key, ps.rng.n, ruv != kRuvNone, lane);
      ps.rng.n = ro.n;
      if (ruv == kRuvMedium) {
        sdir = ro.v;
      } else if (ruv != kRuvNone) {
        Mat mm{};
        mm.m0 = m0;
        scattered = scatter_end(sc, ruv, sref, mm, hp, n, ro.v, sdir, att);
      }
    }
    PT_P4(3)  // unit vector (wave) and scatter_end
    if (shade_now) {
      if (!done && !to_medium) {
        if (scattered) {  // kernels.py:1131-1157
          ps.o = hp;
          ps.dir = sdir;
          ps.thr = pt_mul(ps.thr, att);
          if (ps.depth + 1 >= fr.max_depth) {
            done = true;
            ++n_cap;
          } else {
            if (ps.depth + 1 >= kRRMinDepth) {
              float sp = pt_minf(pt_maxf(pt_maxf(ps.thr.x, ps.thr.y), ps.thr.z), kRRMaxProb);
              if (ps.rng.next() > sp) {
                done = true;
                ++n_rr;
              } else {
                ps.thr = pt_divs(ps.thr, sp);
              }
            }
            if (!done) ++ps.depth;
          }
        } else if (passthrough) {
          ++ps.depth;
          if (ps.depth >= fr.max_depth) {
            done = true;
            ++n_cap;
          }
        } else {
          done = true;
        }
      }
      if (done) {
        ++n_paths;
        if (STAGED) {  // staging[s][p]; stage_resolve adds them in sample order
          float* o = staging + 3 * (size_t)slot;
          o[0] = ps.color.x;
          o[1] = ps.color.y;
          o[2] = ps.color.z;
          live = false;
        } else {  // render_sample: accum += color (kernels.py:1187), next sample of the same pixel
          acc = pt_add(acc, ps.color);
          ++s;
          live = s < s0 + ns;
          if (live) {
            start_path(fr, px, py, s, ps);
            need_seg = true;
          }
        }
      } else {
        need_seg = true;  // next segment of this path (or its medium exit search)
      }
    }
    PT_P4(4)  // epilogue: RR, staging
    if (kPersist) {  // hand the wave's next items to the lanes without a path, fetching units as needed
      const unsigned long long want = __ballot(!live);
      if (want && !(drained && next >= wend)) {
        const uint32_t n = (uint32_t)__popcll(want);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
        const uint32_t avail = wend - next;
        uint32_t my = rank < avail ? next + rank : 0xffffffffu;
        if (n > avail && !drained) {  // one fetch covers it: a unit is 64 items
          int32_t u0 = 0;
          if (lane == 0) {
            u0 = -1;
            for (int a = 0; a < kMkShards; ++a) {  // home shard first, then steal
              const int32_t sh = (int32_t)((blockIdx.x + (unsigned)a) % (unsigned)kMkShards);
              const int32_t lo = sh * wk.shard_len, hi = min(lo + wk.shard_len, wk.nunits);
              int32_t* c = wk.ctl + sh * kMkCtlLine;
              const int32_t cur = lo + __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (cur >= hi) continue;
              const int32_t take = max(1, min(wk.csamp, (hi - cur) / wk.tail_div));
              const int32_t t = lo + atomicAdd(c, take);
              if (t < hi) {
                u0 = t;
                wend = 64u * (uint32_t)min(t + take, hi);  // lane 0's copy, broadcast below
                break;
              }
            }
          }
          u0 = __shfl(u0, 0);
          wend = __shfl(wend, 0);
          if (u0 >= 0) {
            const uint32_t cb = 64u * (uint32_t)u0;
            if (rank >= avail) my = cb + (rank - avail);
            next = cb + (n - avail);
          } else {
            drained = true;
            next = wend;
          }
        } else {
          next = n > avail ? wend : next + n;
        }
        if (!live && my != 0xffffffffu) {
          item = my;
          if (bind(item)) {
            start_path(fr, px, py, s, ps);
            live = true;
            need_seg = true;
          }
        }
      }
      PT_P4(5)  // refill: unit fetch, bind, camera ray
      if (need_seg) {
        need_seg = false;
        begin_segment();
      }
      PT_P4(6)  // segment begin (inverse direction, root slab)
#if PTMI_PROBE == 2
      {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        pr_shade += t - pr_t;
        pr_t = t;
      }
#endif
#if PTMI_PROBE == 3
      if (drained && next >= wend) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (!dr_dry) {
          dr_dry = true;
          dr_tdry = t;
        } else {
          dr_lanecyc += (t - dr_prev) * (uint64_t)__popcll(__ballot(live || trav));
        }
        dr_prev = t;
      }
#endif
      if (__ballot(live) == 0ull && drained && next >= wend) break;
    } else {
      if (need_seg) {
        need_seg = false;
        begin_segment();
      }
      if (__ballot(live) == 0ull) break;
    }
  }
#if PTMI_PROBE == 4
  if (kPersist && lane == 0)
    for (int k = 0; k < 7; ++k) atomicAdd(&g_probe[k], p4[k]);
#endif
#undef PT_P4
#if PTMI_PROBE == 3
  if (kPersist && lane == 0) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    atomicAdd(&g_probe[0], t - dr_t0);
    atomicAdd(&g_probe[1], dr_dry ? t - dr_tdry : 0ull);
    atomicAdd(&g_probe[2], dr_lanecyc);
    atomicAdd(&g_probe[3], 1ull);
  }
#endif
#if PTMI_PROBE == 2
  if (lane == 0) {
    atomicAdd(&g_probe[8], pr_trav);
    atomicAdd(&g_probe[9], pr_shade);
    atomicAdd(&g_probe[10], pr_steps);
    atomicAdd(&g_probe[11], pr_sph);
    atomicAdd(&g_probe[12], pr_oth);
    atomicAdd(&g_probe[13], pr_node);
    atomicAdd(&g_probe[14], pr_both);
    atomicAdd(&g_probe[15], pr_busy);
  }
#endif
  if (!STAGED && ap) {
    ap[0] = acc.x;
    ap[1] = acc.y;
    ap[2] = acc.z;
  }
  if (counters) {  // block sums in the (now idle) stack LDS: no extra LDS, 5 blocks/CU fit
    __syncthreads();
    unsigned long long* red = reinterpret_cast<unsigned long long*>(lds_stack);
    if (tid < kNumCounters) red[tid] = 0ull;
    __syncthreads();
    atomicAdd(&red[0], (unsigned long long)n_seg);
    atomicAdd(&red[1], (unsigned long long)n_med);
    atomicAdd(&red[2], (unsigned long long)n_paths);
    atomicAdd(&red[3], (unsigned long long)n_rr);
    atomicAdd(&red[4], (unsigned long long)n_cap);
    __syncthreads();
    if (tid < kNumCounters) atomicAdd(counters + tid, red[tid]);
  }
}

// accum[pixel] += staging[s][p] for s = 0..batch-1 in order (render_sample's
// per-sample accumulation, kernels.py:1187 / renderer.py:405).
__global__ __launch_bounds__(kBlock) void stage_resolve(DevFrame fr, const float* __restrict__ staging, int32_t npix,
                                                        int32_t batch, float* __restrict__ accum) {
  for (int32_t p = (int32_t)(blockIdx.x * kBlock + threadIdx.x); p < npix; p += (int32_t)(gridDim.x * kBlock)) {
    int32_t lr = p / fr.w;
    int32_t px = fr.x0 + (p - lr * fr.w);
    int32_t py = frame_row(fr, lr);
    float* ap = accum + 3 * ((size_t)py * (size_t)fr.width + (size_t)px);
    float a0 = ap[0], a1 = ap[1], a2 = ap[2];
    const float* sp = staging + 3 * (size_t)p;
    for (int32_t s = 0; s < batch; ++s) {
      const float* c = sp + 3 * (size_t)s * (size_t)npix;
      a0 += c[0];
      a1 += c[1];
      a2 += c[2];
    }
    ap[0] = a0;
    ap[1] = a1;
    ap[2] = a2;
  }
}

hipError_t launch_stage_resolve(const DevFrame& fr, const float* staging, int32_t npix, int32_t batch,
                                float* accum, int prof_kind, hipStream_t stream) {
  unsigned g = (unsigned)((npix + kBlock - 1) / kBlock);
  if (g > 2048) g = 2048;
  const int pslot = prof_begin(prof_kind, stream);
  hipLaunchKernelGGL(stage_resolve, dim3(g), dim3(kBlock), 0, stream, fr, staging, npix, batch, accum);
  prof_end(pslot, stream);
  return hipGetLastError();
}

template <int STACK, int TRAV = PTMI_TRAV_STACK>
static hipError_t launch_mk(const DevScene& sc, const DevFrame& fr, float* accum, int32_t s_begin,
                            int32_t s_count, unsigned long long* counters, hipStream_t stream) {
  dim3 grid((unsigned)((fr.w + kMkTile - 1) / kMkTile), (unsigned)((fr.n_rows + kMkTile - 1) / kMkTile));
  const int pslot = prof_begin(kProfMk, stream);
  hipLaunchKernelGGL((mk_render_kernel<STACK, false, TRAV>), grid, dim3(kMkBlock), 0, stream, sc, fr, accum, s_begin,
                     s_count, s_count, (float*)nullptr, counters, MkWork{});
  prof_end(pslot, stream);
  return hipGetLastError();
}

hipError_t mk_render(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, float* accum,
                     int32_t s_begin, int32_t s_count, unsigned long long* counters, hipStream_t stream) {
  if (fr.traversal == PTMI_TRAV_STACKLESS)
    return launch_mk<1, PTMI_TRAV_STACKLESS>(sc, fr, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= 16) return launch_mk<16>(sc, fr, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= 20) return launch_mk<20>(sc, fr, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= 24) return launch_mk<24>(sc, fr, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= 32) return launch_mk<32>(sc, fr, accum, s_begin, s_count, counters, stream);
  if (stack_needed <= kRefStackSlots - 1) return launch_mk<64>(sc, fr, accum, s_begin, s_count, counters, stream);
  // leaf depth > 62: the reference's 64-entry stack drops pushes (TravRS)
  return launch_mk<kRefStackSlots, kTravRefStack>(sc, fr, accum, s_begin, s_count, counters, stream);
}

// ---------------------------------------------------------------- staged
#ifndef PTMI_MK_STAGED_MIN_STACK
#define PTMI_MK_STAGED_MIN_STACK 16  // staged: STACK 16 scenes use the 16-slot kernel at 5 waves/SIMD (PTMI_MK_MIN_WAVES_16)
#endif

static size_t mk_staging_bytes(int32_t npix, int32_t batch) {
  return (3 * sizeof(float) * (size_t)npix * (size_t)batch + 255) & ~(size_t)255;
}

size_t mk_workspace_bytes(int32_t npix, int32_t batch) {  // staging + the shards' 256-B counter lines
  if (npix <= 0 || batch <= 0) return 0;
  return mk_staging_bytes(npix, batch) + 256 * kMkShards;
}

// The megakernel of one staged batch: every (sample, pixel) colour of the
// batch into staging[sample][pixel]; the accumulator is not touched (the
// resolve is launch_stage_resolve, on the caller's schedule).
template <int STACK, int TRAV = PTMI_TRAV_STACK>
static hipError_t launch_mk_trace(const DevScene& sc, const DevFrame& fr, float* staging, int32_t s_begin,
                                  int32_t nb, unsigned long long* counters, hipStream_t stream) {
  float* accum = nullptr;  // staged kernels write staging only
  int32_t tx = 0;
  const int64_t tiles = mk_tiles(fr, &tx);
  int dev = 0, ncu = 0, per_cu = 0;
  hipError_t e0 = hipGetDevice(&dev);
  if (e0 == hipSuccess) e0 = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e0 == hipSuccess)
    e0 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mk_render_kernel<STACK, true, TRAV>, kMkBlock, 0);
  if (e0 != hipSuccess) return e0;
  MkWork wk;
  wk.ctl = (int32_t*)((char*)staging + mk_staging_bytes(fr.w * fr.n_rows, nb));
  wk.csamp = PTMI_MK_CHUNK_SAMPLES;
  wk.tiles_x = tx;
  wk.tw_log2 = 6 - mk_tile_rows_log2(fr);
  wk.nb = nb;
  if (tiles * nb * 64 >= (1ll << 32)) return hipErrorInvalidValue;  // item ids are 32-bit
  // shard s: tiles s, s + S, ... (interleaved across the image, so every shard
  // costs about the same); virtual units past the last tile decode to rows
  // outside the frame and are skipped
  wk.shard_len = (int32_t)((tiles + kMkShards - 1) / kMkShards) * nb;
  wk.nunits = wk.shard_len * kMkShards;
  if ((int64_t)wk.nunits * 64 >= (1ll << 32)) return hipErrorInvalidValue;
  wk.by_len = fast_div((uint32_t)wk.shard_len);
  wk.by_nb = fast_div((uint32_t)nb);
  wk.by_tiles_x = fast_div((uint32_t)wk.tiles_x);
  // Small batches (an 8-rank tile shard) run on a smaller persistent grid, so
  // the next overlapped call's waves share the chip while this one drains.
  if ((int64_t)fr.w * fr.n_rows * nb < PTMI_MK_SMALL_GRID_BATCH && per_cu > PTMI_MK_SMALL_WPC) per_cu = PTMI_MK_SMALL_WPC;
  int64_t waves = (int64_t)(per_cu > 0 ? per_cu : 1) * (ncu > 0 ? ncu : 1);
  const int64_t chunks = wk.nunits;
  if (waves > chunks) waves = chunks;
  // per shard: the waves pulling from it. Small batches (a multi-GPU tile
  // shard: 5 M samples per call for vol2 at 8 GPUs) are all tail: halving the
  // divisor there takes larger fetches, so a wave changes tile less often
  // (A/B, 8-rank rehearsal: +2 % per GPU; profiles/r03/ab/ab_mk_small_calls.log).
  const int64_t tail = (int64_t)fr.w * fr.n_rows * nb < PTMI_MK_SMALL_BATCH ? PTMI_MK_TAIL_DIV_SMALL : PTMI_MK_TAIL_DIV;
  const int64_t tdiv = tail * waves / kMkShards;
  wk.tail_div = (int32_t)(tdiv > 1 ? tdiv : 1);
  (void)hipMemsetAsync(wk.ctl, 0, 256 * kMkShards, stream);
  const int pslot = prof_begin(kProfMk, stream);
  hipLaunchKernelGGL((mk_render_kernel<STACK, true, TRAV>), dim3((unsigned)waves), dim3(kMkBlock), 0, stream,
                     sc, fr, accum, s_begin, nb, nb, staging, counters, wk);
  prof_end(pslot, stream);
  return hipGetLastError();
}

hipError_t mk_trace_staged(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws,
                           int32_t s_begin, int32_t nb, unsigned long long* counters, hipStream_t stream) {
  float* st = (float*)ws;
  if (fr.traversal == PTMI_TRAV_STACKLESS)
    return launch_mk_trace<1, PTMI_TRAV_STACKLESS>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed <= PTMI_MK_STAGED_MIN_STACK) return launch_mk_trace<16>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed == 17) return launch_mk_trace<17>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed == 18) return launch_mk_trace<18>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed == 19) return launch_mk_trace<19>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed <= 20) return launch_mk_trace<20>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed <= 24) return launch_mk_trace<24>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed <= 32) return launch_mk_trace<32>(sc, fr, st, s_begin, nb, counters, stream);
  if (stack_needed <= kRefStackSlots - 1) return launch_mk_trace<64>(sc, fr, st, s_begin, nb, counters, stream);
  // leaf depth > 62: the reference's 64-entry stack drops pushes (TravRS)
  return launch_mk_trace<kRefStackSlots, kTravRefStack>(sc, fr, st, s_begin, nb, counters, stream);
}

int64_t mk_max_batch(const DevFrame& fr) {
  // item ids (tile, sample, pixel of the 64-pixel tile) are 32-bit: tiles * batch * 64 < 2^32
  const int64_t tiles = mk_tiles(fr);
  const int64_t padded = (tiles + kMkShards - 1) / kMkShards * kMkShards;  // interleaved shards' virtual units
  return tiles > 0 ? ((1ll << 32) - 1) / (padded * 64) : 0;
}

hipError_t mk_render_staged(const DevScene& sc, const DevFrame& fr, int32_t stack_needed, void* ws,
                            size_t ws_bytes, float* accum, int32_t s_begin, int32_t s_count,
                            unsigned long long* counters, hipStream_t stream) {
  if (s_count < 2)  // one sample: direct accumulation, no staging
    return mk_render(sc, fr, stack_needed, accum, s_begin, s_count, counters, stream);
  const int32_t npix = fr.w * fr.n_rows;
  int32_t batch = s_count;
  const int64_t max_batch = mk_max_batch(fr);
  if (max_batch < 1) return hipErrorInvalidValue;
  if (batch > max_batch) batch = (int32_t)max_batch;
  while (batch > 1 && mk_workspace_bytes(npix, batch) > ws_bytes) batch = (batch + 1) / 2;
  if (mk_workspace_bytes(npix, batch) > ws_bytes) return hipErrorInvalidValue;
  for (int32_t b0 = 0; b0 < s_count; b0 += batch) {
    const int32_t nb = s_count - b0 < batch ? s_count - b0 : batch;
    hipError_t e = mk_trace_staged(sc, fr, stack_needed, ws, s_begin + b0, nb, counters, stream);
    if (e == hipSuccess) e = launch_stage_resolve(fr, (const float*)ws, npix, nb, accum, kProfMkResolve, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ptmi

#if PTMI_PROBE
extern "C" int ptmi_probe_read(unsigned long long* out, int reset) {
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(out, HIP_SYMBOL(ptmi::g_probe), 16 * sizeof(unsigned long long));
  if (reset) {
    unsigned long long z[16] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(ptmi::g_probe), z, sizeof(z));
  }
  return 0;
}
#endif
