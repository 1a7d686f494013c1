// pt_device.hpp — gfx950 device-side building blocks of the integrator:
// packed scene access, primitive intersection, the child-box BVH2 traversal
// with an LDS stack, textures, materials and the medium step.
//
// Semantics follow src/render_server/taichi_renderer/kernels.py (cited per
// function); arithmetic and random draws follow include/ptmi_math.h and
// include/ptmi_rng.h so results are bit-identical to the CPU oracle.
// Compile with -ffp-contract=off (see Makefile).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ptmi.h"
#include "../../include/ptmi_math.h"
#include "../../include/ptmi_rng.h"

namespace ptmi {

constexpr float kTMin = 0.001f;     // kernels.py:1057, 1254
constexpr float kTMax = 1e10f;
constexpr int kRRMinDepth = 5;      // kernels.py:1050
constexpr float kRRMaxProb = 0.95f; // kernels.py:1051
constexpr int kNumCounters = PTMI_NUM_COUNTERS;  // include/ptmi.h


// n / d by one 64-bit multiply and shift: m = floor(2^(32+l) / d) + 1 with
// 2^l >= d (so m <= 2^33) gives floor(n / d) exactly for every n < 2^32 in
// exact arithmetic; the 64-bit product n * m does not wrap while n < 2^31
// (any n < 2^32 when d is a power of two, m = 2^32 + 1). Callers keep n below
// 2^31: the megakernel divides unit ids (item >> 6), the wavefront padded work
// item ids, bounded in wf_render.
struct FastDiv {
  uint64_t m;
  uint32_t sh, d;
};
static inline FastDiv fast_div(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  return FastDiv{((1ull << (32 + l)) / d) + 1ull, 32u + l, d};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (uint32_t)(((uint64_t)n * f.m) >> f.sh); }
constexpr int kBlock = 256;

// Register-budget stress build (libptmi_stress.so, tests/test_gpu_stress_build.py):
// PTMI_STRESS_WAVES = N raises every render kernel's minimum waves per SIMD to
// N, i.e. caps its VGPRs so that it spills. A legal register budget must not
// change a result; the stress build renders the parity cases against the
// oracle, so code that depends on what an inactive lane's register holds
// (round 6, cont_position in pt_wavefront.hip) fails there. 0: off.
#ifndef PTMI_STRESS_WAVES
#define PTMI_STRESS_WAVES 0
#endif
constexpr int stress_waves(int w) { return PTMI_STRESS_WAVES > w ? PTMI_STRESS_WAVES : w; }

enum : int32_t { kSphere = 0, kTriangle = 1, kQuad = 2 };

struct DevScene {
  const float4* __restrict__ nodes;
  int32_t n_inner;
  int32_t root_ref;
  float root_min[3], root_max[3];
  const float4* __restrict__ spheres;
  const float4* __restrict__ quads;
  const float4* __restrict__ tris;
  const float4* __restrict__ mats;
  int32_t mat_base[3];  // indexed by prim type: sphere 0, triangle ns+nq, quad ns
  const uint32_t* __restrict__ texels;
  int32_t num_images;
  int32_t img_offset[PTMI_MAX_IMAGES], img_w[PTMI_MAX_IMAGES], img_h[PTMI_MAX_IMAGES];
  const float4* __restrict__ perlin_vec;
  const int32_t* __restrict__ perlin_perm;
  const float4* __restrict__ ref_nodes;  // reference-layout nodes (stackless traversal), 3 float4 each
  int32_t n_nodes;                       // all BVH nodes
};

struct DevFrame {
  float center[3], pixel00[3], delta_u[3], delta_v[3], defocus_u[3], defocus_v[3];
  float defocus_angle;
  float bg[3];
  int32_t max_depth;
  uint32_t seed;
  int32_t width, height;
  int32_t x0, y0, w, h;
  int32_t band_rows, band_stride, band_offset;
  int32_t n_rows;  // rows of the window this frame owns (after banding)
  int32_t traversal;  // PTMI_TRAV_*
};

__device__ __forceinline__ int32_t leaf_type(int32_t ref) { return (ref >> 28) & 3; }
__device__ __forceinline__ int32_t leaf_index(int32_t ref) { return ref & 0x01ffffff; }
// material class of a leaf (PTMI_CLASS_*, include/ptmi.h), packed by the host
__device__ __forceinline__ int32_t leaf_class(int32_t ref) { return (ref >> 25) & 7; }

// Local row (0..n_rows-1) -> image row, or -1.
__device__ __forceinline__ int32_t frame_row(const DevFrame& fr, int32_t lr) {
  int32_t band = lr / fr.band_rows;
  int32_t within = lr - band * fr.band_rows;
  int32_t row = fr.y0 + (band * fr.band_stride + fr.band_offset) * fr.band_rows + within;
  return (row < fr.y0 + fr.h) ? row : -1;
}

// ---------------------------------------------------------------- RNG
struct Rng {
  uint32_t key, n;
  __device__ __forceinline__ float next() { return pt_rand(key, n++); }
};

__device__ __forceinline__ pt_v3 random_in_unit_disk(Rng& r) {  // kernels.py:17-25
  for (;;) {
    float x = r.next() * 2.0f - 1.0f;
    float y = r.next() * 2.0f - 1.0f;
    pt_v3 p = pt_v3f(x, y, 0.0f);
    if (pt_dot(p, p) < 1.0f) return p;
  }
}

__device__ __forceinline__ pt_v3 random_unit_vector(Rng& r) {  // kernels.py:29-38
  for (;;) {
    float x = r.next() * 2.0f - 1.0f;
    float y = r.next() * 2.0f - 1.0f;
    float z = r.next() * 2.0f - 1.0f;
    pt_v3 p = pt_v3f(x, y, z);
    float l2 = pt_dot(p, p);
    if (l2 < 1.0f && l2 > 1e-20f) return pt_normalize(p);
  }
}

// random_unit_vector for the lanes of a wave that need one (need; call from
// wave-uniform code), the other lanes testing their candidates: the
// rejection loop's candidates are independent counter-based draws (candidate
// j of a lane at counter n is the three draws n + 3j, n + 3j + 1, n + 3j + 2),
// so with k lanes pending each gets C = 64 / k (at most 16) lanes, lane j of
// its group tests candidate j, and the lane takes its first accepted one and
// advances its counter past it: the same draws, the same first accepted
// candidate and the same normalisation as its own loop, bit-identical. An
// ablation with the loop replaced by one candidate (not parity) put the loop
// at 2.3 % of C2 and 4.9 % of C4 (profiles/r04/ab/ab_r04q_ruv_ablation.log): it
// runs to the wave's unluckiest lane (acceptance pi/6 per candidate). More
// than 32 lanes pending: each lane runs its own loop. A/B on MI355X (round 4,
// parity-identical) against the divergent site: C4 +1.4 %, C2 +0.2 %, C5
// +0.1 % (the split of the shading code around the uniform site alone: C4
// -1.3 %; profiles/r04/ab/ab_r04r_wave_ruv.log).
// Inlined: A/B within noise of a call (C4 +1.4 vs +1.3 %, C5 +0.1 vs -0.2 %).
struct RuvOut {
  pt_v3 v;
  uint32_t n;  // the lane's counter after its draws
};
__device__ __forceinline__ RuvOut random_unit_vector_wave(uint32_t key, uint32_t ctr, bool need, int lane) {
  unsigned long long pend = __builtin_amdgcn_ballot_w64(need);
  const uint32_t k0 = (uint32_t)__popcll(pend);
  if (k0 > 32u) {  // too many for a group each: the plain loop
    Rng r{key, ctr};
    pt_v3 v = pt_v3f(0.0f, 0.0f, 0.0f);
    if (need) v = random_unit_vector(r);
    return RuvOut{v, r.n};
  }
  pt_v3 p = pt_v3f(0.0f, 0.0f, 0.0f);
  uint32_t n0 = ctr;
  while (pend != 0ull) {
    const uint32_t k = (uint32_t)__popcll(pend);
    const uint32_t lg = k <= 1u ? 0u : 32u - (uint32_t)__builtin_clz(k - 1u);  // ceil(log2 k)
    const uint32_t lc = lg >= 2u ? 6u - lg : 4u;                                 // log2 C, C <= 16
    const bool pending = (pend >> lane) & 1ull;
    const uint32_t lo = (uint32_t)pend, hi = (uint32_t)(pend >> 32);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
    const uint32_t nrank = __builtin_amdgcn_mbcnt_hi(~hi, __builtin_amdgcn_mbcnt_lo(~lo, 0u));
    // a permutation of the lanes: pending lanes to [0, k) in lane order, the rest after
    const int dst = (int)(pending ? rank : k + nrank);
    const int owner_of = __builtin_amdgcn_ds_permute(dst << 2, lane);  // lane r < k: the r-th pending lane
    const int g = lane >> lc, j = lane & ((1 << lc) - 1);
    const bool valid = (uint32_t)g < k;
    const int owner = __builtin_amdgcn_ds_bpermute((valid ? g : 0) << 2, owner_of);
    const uint32_t okey = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)key);
    const uint32_t on = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)n0) + 3u * (uint32_t)j;
    const float x = pt_rand(okey, on) * 2.0f - 1.0f;
    const float y = pt_rand(okey, on + 1u) * 2.0f - 1.0f;
    const float z = pt_rand(okey, on + 2u) * 2.0f - 1.0f;
    const float l2 = pt_dot(pt_v3f(x, y, z), pt_v3f(x, y, z));
    const unsigned long long acc = __builtin_amdgcn_ballot_w64(valid && l2 < 1.0f && l2 > 1e-20f);
    // a pending lane: its group's first accepted candidate, if any
    const uint32_t base = pending ? rank << lc : 0u;  // < 64: k groups of C lanes
    const unsigned long long gbits = (acc >> base) & ((1ull << (1u << lc)) - 1ull);
    const uint32_t jf = gbits != 0ull ? (uint32_t)__builtin_ctzll(gbits) : 0u;
    const int src = (int)(base + jf);
    const float ax = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(x)));
    const float ay = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(y)));
    const float az = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(z)));
    bool still = false;
    if (pending) {
      if (gbits != 0ull) {
        p = pt_v3f(ax, ay, az);
        n0 += 3u * (jf + 1u);
      } else {
        n0 += 3u << lc;
        still = true;
      }
    }
    pend = __builtin_amdgcn_ballot_w64(still);
  }
  return RuvOut{need ? pt_normalize(p) : p, n0};
}

__device__ __forceinline__ pt_v3 random_cosine_direction(pt_v3 n, Rng& r) {  // kernels.py:42-71
  float r1 = r.next();
  float r2 = r.next();
  float z = sqrtf(1.0f - r2);
  float phi = PT_2PI_F * r1;
  float st = sqrtf(r2);
  float sp, cp;
  pt_sincosf(phi, &sp, &cp);
  float x = cp * st, y = sp * st;
  pt_v3 w = pt_normalize(n);
  pt_v3 a = (fabsf(w.x) < 0.9f) ? pt_v3f(1.0f, 0.0f, 0.0f)
            : (fabsf(w.y) < 0.9f) ? pt_v3f(0.0f, 1.0f, 0.0f) : pt_v3f(0.0f, 0.0f, 1.0f);
  pt_v3 v = pt_normalize(pt_cross(a, w));
  pt_v3 u = pt_cross(v, w);
  return pt_normalize(pt_add(pt_add(pt_scale(u, x), pt_scale(v, y)), pt_scale(w, z)));
}

// ---------------------------------------------------------------- camera
// kernels.py:177-201 (get_ray). Returns the unnormalized direction.
__device__ __forceinline__ void get_ray(const DevFrame& fr, int32_t px, int32_t py, Rng& r, pt_v3& o,
                                        pt_v3& d) {
  float ox = r.next() - 0.5f;
  float oy = r.next() - 0.5f;
  pt_v3 p00 = pt_v3f(fr.pixel00[0], fr.pixel00[1], fr.pixel00[2]);
  pt_v3 du = pt_v3f(fr.delta_u[0], fr.delta_u[1], fr.delta_u[2]);
  pt_v3 dv = pt_v3f(fr.delta_v[0], fr.delta_v[1], fr.delta_v[2]);
  pt_v3 ps = pt_add(pt_add(p00, pt_scale(du, (float)px + ox)), pt_scale(dv, (float)py + oy));
  pt_v3 c = pt_v3f(fr.center[0], fr.center[1], fr.center[2]);
  o = c;
  if (fr.defocus_angle > 0.0f) {
    pt_v3 p = random_in_unit_disk(r);
    pt_v3 fu = pt_v3f(fr.defocus_u[0], fr.defocus_u[1], fr.defocus_u[2]);
    pt_v3 fv = pt_v3f(fr.defocus_v[0], fr.defocus_v[1], fr.defocus_v[2]);
    o = pt_add(pt_add(c, pt_scale(fu, p.x)), pt_scale(fv, p.y));
  }
  d = pt_sub(ps, o);
}

// ---------------------------------------------------------------- primitives
// Leaf primitives are loaded whole (one round trip) before their test (A/B on
// MI355X: +1.4 % C2, +4 % C4, +2.6 % wavefront). A/B, not kept: the leaf tests
// as one predicate instead of nested early-outs, -1 % mk, -2 % wf
// (profiles/r01/ab_leaf_flat.log).
// a && b && c && d of per-lane compares as lane masks (v_cmp into SGPR pairs,
// s_and): the compiler otherwise materialises each compare with v_cndmask and
// combines them with 16-bit VALU bit ops (~16 VALU per quad test on gfx950)
__device__ __forceinline__ bool pt_all4(bool a, bool b, bool c, bool d) {
  return __builtin_amdgcn_inverse_ballot_w64(__builtin_amdgcn_ballot_w64(a) & __builtin_amdgcn_ballot_w64(b) &
                                             __builtin_amdgcn_ballot_w64(c) & __builtin_amdgcn_ballot_w64(d));
}

__device__ __forceinline__ bool pt_all2(bool a, bool b) {
  return __builtin_amdgcn_inverse_ballot_w64(__builtin_amdgcn_ballot_w64(a) & __builtin_amdgcn_ballot_w64(b));
}

// Each returns the candidate t (hit only if returned true); hit point and
// normal are recomputed at shading time from (o, d, t) with the same
// operation order the reference uses inside the hit functions.

// Sphere roots (h -+ sqrt(disc)) / a through a per-ray reciprocal of a
// (pt_div_by, include/ptmi_math.h): A/B on MI355X, parity-identical: C2 +0.9 %, C5 +0.6 %, C3
// +0.3 % (profiles/r02/ab/ab_sphere_markstein.log)
// EXCL: the caller updates the closest hit only when t < tmax (tmax being
// the current closest t), so the final range test takes t < tmax itself and
// the caller drops its compare: the same updates, one compare fewer.
template <bool EXCL = false>
__device__ __forceinline__ bool hit_sphere_t(const float4 s, pt_v3 o, pt_v3 d, float tmin, float tmax,
                                             float& t) {  // kernels.py:209-248
  pt_v3 c = pt_v3f(s.x, s.y, s.z);
  pt_v3 oc = pt_sub(c, o);
  float a = pt_dot(d, d);
  const float ra = pt_recip_for_div(a);  // loop-invariant in a traversal: hoisted per segment
#define PT_SPH_DIV(x) pt_div_by((x), a, ra)
  float h = pt_dot(d, oc);
  float cc = pt_dot(oc, oc) - s.w * s.w;
  float disc = h * h - a * cc;
  if (disc >= 0.0f) {
    float sq = sqrtf(disc);
    float root = PT_SPH_DIV(h - sq);
    if (root < tmin || root > tmax) root = PT_SPH_DIV(h + sq);
    if (pt_all2(root >= tmin, EXCL ? root < tmax : root <= tmax)) { t = root; return true; }
  }
  return false;
#undef PT_SPH_DIV
}

template <bool EXCL = false>
__device__ __forceinline__ bool hit_quad_v(const float4 a, const float4 b, const float4 c, const float4 e, pt_v3 o,
                                           pt_v3 d, float tmin, float tmax, float& t) {  // kernels.py:311-362
  pt_v3 n = pt_v3f(a.x, a.y, a.z);
  float denom = pt_dot(n, d);
  if (fabsf(denom) >= 1e-8f) {
    float tt = (a.w - pt_dot(n, o)) / denom;
    if (pt_all2(tt >= tmin, EXCL ? tt < tmax : tt <= tmax)) {
      pt_v3 Q = pt_v3f(b.x, b.y, b.z), u = pt_v3f(b.w, c.x, c.y), v = pt_v3f(c.z, c.w, e.x);
      pt_v3 w = pt_v3f(e.y, e.z, e.w);
      pt_v3 ip = pt_add(o, pt_scale(d, tt));
      pt_v3 pv = pt_sub(ip, Q);
      float alpha = pt_dot(w, pt_cross(pv, v));
      float beta = pt_dot(w, pt_cross(u, pv));
      if (pt_all4(alpha >= 0.0f, alpha <= 1.0f, beta >= 0.0f, beta <= 1.0f)) { t = tt; return true; }
    }
  }
  return false;
}

template <bool EXCL = false>
__device__ __forceinline__ bool hit_quad_t(const float4* __restrict__ q, pt_v3 o, pt_v3 d, float tmin,
                                           float tmax, float& t) {
  // all 64 B in one round trip (the compiler otherwise sinks the loads into
  // the branches: three dependent L2 round trips per quad test)
  typedef float pt_f4 __attribute__((ext_vector_type(4)));
  pt_f4 A = ((const pt_f4*)q)[0], B = ((const pt_f4*)q)[1], C = ((const pt_f4*)q)[2], E = ((const pt_f4*)q)[3];
  asm volatile("" : "+v"(A), "+v"(B), "+v"(C), "+v"(E));
  return hit_quad_v<EXCL>(make_float4(A.x, A.y, A.z, A.w), make_float4(B.x, B.y, B.z, B.w),
                    make_float4(C.x, C.y, C.z, C.w), make_float4(E.x, E.y, E.z, E.w), o, d, tmin, tmax, t);
}

template <bool EXCL = false>
__device__ __forceinline__ bool hit_tri_v(const float4 a, const float4 b, const float4 c, pt_v3 o, pt_v3 d,
                                          float tmin, float tmax, float& t) {  // kernels.py:252-307
  pt_v3 v0 = pt_v3f(a.x, a.y, a.z), e1 = pt_v3f(a.w, b.x, b.y), e2 = pt_v3f(b.z, b.w, c.x);
  pt_v3 hv = pt_cross(d, e2);
  float det = pt_dot(e1, hv);
  if (fabsf(det) >= 1e-8f) {
    float inv = 1.0f / det;
    pt_v3 s = pt_sub(o, v0);
    float u = inv * pt_dot(s, hv);
    if (pt_all2(u >= 0.0f, u <= 1.0f)) {
      pt_v3 q = pt_cross(s, e1);
      float v = inv * pt_dot(d, q);
      if (pt_all2(v >= 0.0f, u + v <= 1.0f)) {
        float tt = inv * pt_dot(e2, q);
        if (pt_all2(tt >= tmin, EXCL ? tt < tmax : tt <= tmax)) { t = tt; return true; }
      }
    }
  }
  return false;
}

// (A/B, round 5, not kept: a dword load of e2.z instead of the third 16 B,
// C4 +0.2 %, noise.)
template <bool EXCL = false>
__device__ __forceinline__ bool hit_tri_t(const float4* __restrict__ tr, pt_v3 o, pt_v3 d, float tmin,
                                          float tmax, float& t) {
  typedef float pt_f4 __attribute__((ext_vector_type(4)));
  pt_f4 A = ((const pt_f4*)tr)[0], B = ((const pt_f4*)tr)[1];
  pt_f4 C = ((const pt_f4*)tr)[2];
  asm volatile("" : "+v"(A), "+v"(B), "+v"(C));
  return hit_tri_v<EXCL>(make_float4(A.x, A.y, A.z, A.w), make_float4(B.x, B.y, B.z, B.w),
                         make_float4(C.x, C.y, C.z, C.w), o, d, tmin, tmax, t);
}

__device__ __forceinline__ bool hit_leaf(const DevScene& sc, int32_t ref, pt_v3 o, pt_v3 d, float tmin,
                                         float tmax, float& t) {
  int32_t ty = leaf_type(ref), ix = leaf_index(ref);
  if (ty == kSphere) return hit_sphere_t(sc.spheres[ix], o, d, tmin, tmax, t);
  if (ty == kQuad) return hit_quad_t(sc.quads + 4 * ix, o, d, tmin, tmax, t);
  return hit_tri_t(sc.tris + 3 * ix, o, d, tmin, tmax, t);
}

// Surface normal of a hit, kernels.py:246, 300-305, 355-360.
__device__ __forceinline__ pt_v3 hit_normal(const DevScene& sc, int32_t ref, pt_v3 hp, pt_v3 d) {
  int32_t ty = leaf_type(ref), ix = leaf_index(ref);
  if (ty == kSphere) {
    float4 s = sc.spheres[ix];
    return pt_divs(pt_sub(hp, pt_v3f(s.x, s.y, s.z)), s.w);
  }
  if (ty == kQuad) {
    float4 a = sc.quads[4 * ix];
    pt_v3 n = pt_v3f(a.x, a.y, a.z);
    return (pt_dot(n, d) < 0.0f) ? n : pt_neg(n);
  }
  float4 c = sc.tris[3 * ix + 2];
  pt_v3 n = pt_v3f(c.y, c.z, c.w);
  return (pt_dot(d, n) > 0.0f) ? pt_neg(n) : n;
}

// ---------------------------------------------------------------- traversal
// Closest hit over the child-box BVH2 with the reference's visiting order
// (traverse_bvh_legacy, kernels.py:625-742): far child pushed first by the
// projected distance of the children's box centres, a popped node culled
// when its box misses [t_min, closest_t], closest hit updated only when
// t < closest_t. Each stack entry carries the child's slab entry distance E
// (computed once when the parent is expanded); the reference's pop-time
// test max(E, t_min) <= min(X, closest_t) is split exactly into X >= E (at
// push) and E <= closest_t (at pop). Stack: STACK 8-byte {ref, E} slots per
// thread in LDS, slot-major, so a wave's ds_read_b64/ds_write_b64 hit
// distinct banks.
//
// Node layout (include/ptmi.h): the two children's box coordinates are
// interleaved per component — {lo.x L,R | lo.y L,R}{lo.z L,R | hi.x L,R}
// {hi.y L,R | hi.z L,R}{ref L, ref R, -, -} — so both children's slabs and
// centre distances are computed as pairs (pt_f2) of scalar f32 ops.
//
// A/B history on MI355X (all parity-identical): near-child shortcut with a
// nested pop loop -17 %; top of stack in registers +0-2 % (mk) / -3 % (wf);
// while-while -15 %; persistent lanes refilled per ray (wf) -7 %; skipping
// culled pops in an inner loop -11 %; scalar-cache fetch of wave-uniform
// nodes -1.7 % (the SGPR->VGPR moves cost more VALU than the texture path
// saves); testing a leaf pushed on top in the expanding step itself -3 % mk
// (profiles/r01/ab_leaf_top.log); near-child node prefetch across unrolled
// pops -11 to -13 % (profiles/r02/ab/ab_trav_prefetch.log). Kept: child
// pairs (scalar since round 2), precomputed centres, branch-free pushes.

// The node step's child pairs are two scalar f32 ops, not one v_pk_*_f32: a
// packed f32 op costs a wave about the issue time of the two scalar ops it
// replaces (MI355X_MICROARCH.md constants, 'vector-instruction ISSUE cost' and
// the packed-f32 filler row), and the pairs need operand shuffles. A/B on
// MI355X, parity-identical, after -fno-slp-vectorize: C2 +5.5 %, C3 and C4
// within noise (profiles/r02/ab/ab_trav_scalar.log).
struct pt_f2 {
  float x, y;
};
__device__ __forceinline__ pt_f2 operator+(pt_f2 a, pt_f2 b) { return pt_f2{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ pt_f2 operator-(pt_f2 a, pt_f2 b) { return pt_f2{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ pt_f2 operator*(pt_f2 a, pt_f2 b) { return pt_f2{a.x * b.x, a.y * b.y}; }

// A thread's traversal stack: slot k at slot0[k * SB] (SB = threads per
// block) in LDS for k < LDS (a kernel template argument); a kernel whose LDS
// holds fewer slots than the stack needs (LDS < STACK: wf_intersect, where
// LDS sets the occupancy) keeps the deeper slots in global memory, slot k at
// byte spill_off + (k - LDS) * spill_stride of spill (slot-major over the
// grid's threads, so a wave's accesses are coalesced). Deep entries are rare:
// the pops and pushes of the top LDS slots take the LDS path.
struct Stack {
  uint2* slot0;              // &lds[tid]
  char* spill = nullptr;     // global spill slots (LDS < STACK only)
  uint32_t spill_off = 0;    // this thread's byte offset in a spill slot row
  uint32_t spill_stride = 0; // bytes between a thread's consecutive spill slots
};

// LDS accesses by 32-bit byte address (a stack pointer kept as the address of
// its slot: one v_add per pop or push, no index scaling).
typedef uint32_t pt_u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) pt_u2v pt_lds_u2v;
typedef __attribute__((address_space(3))) uint32_t pt_lds_u32;
__device__ __forceinline__ uint32_t lds_addr(uint2* p) { return (uint32_t)(uintptr_t)(pt_lds_u2v*)p; }
__device__ __forceinline__ pt_u2v lds_load2(uint32_t a) { return *(pt_lds_u2v*)(uintptr_t)a; }
__device__ __forceinline__ void lds_store2(uint32_t a, uint32_t x, uint32_t y) {
  pt_lds_u32* q = (pt_lds_u32*)(uintptr_t)a;
  q[0] = x;
  q[1] = y;
}

// Stack slot access by LDS-style address a = slot0 + k * kSlot, for a stack
// of LDS slots in LDS and the rest spilled (LDS < STACK); lim = the address
// of slot LDS. With LDS == STACK these are the plain LDS accesses.
typedef __attribute__((address_space(1))) pt_u2v pt_glb_u2v;
template <int STACK, int LDS, int SB>
__device__ __forceinline__ pt_u2v stack_load(const Stack& st, uint32_t lim, uint32_t a) {
  if constexpr (LDS >= STACK) {
    return lds_load2(a);
  } else {
    if (a < lim) return lds_load2(a);
    constexpr int kShift = __builtin_ctz(SB * 8);
    const uint32_t off = st.spill_off + ((a - lim) >> kShift) * st.spill_stride;
    return *(const pt_glb_u2v*)((const __attribute__((address_space(1))) char*)st.spill + off);
  }
}
template <int STACK, int LDS, int SB>
__device__ __forceinline__ void stack_store(const Stack& st, uint32_t lim, uint32_t a, uint32_t x, uint32_t y) {
  if constexpr (LDS >= STACK) {
    lds_store2(a, x, y);
  } else {
    if (a < lim) {
      lds_store2(a, x, y);
    } else {
      constexpr int kShift = __builtin_ctz(SB * 8);
      const uint32_t off = st.spill_off + ((a - lim) >> kShift) * st.spill_stride;
      *(pt_glb_u2v*)((__attribute__((address_space(1))) char*)st.spill + off) = pt_u2v{x, y};
    }
  }
}

// Lane mask of a predicate (v_cmp straight into an SGPR pair; __ballot's int
// argument costs a v_cndmask + v_cmp per call).
__device__ __forceinline__ unsigned long long pt_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ void slab(pt_v3 o, pt_v3 inv, float mnx, float mny, float mnz, float mxx, float mxy,
                                     float mxz, float tmin, float& E, float& X) {
  float t0x = (mnx - o.x) * inv.x, t1x = (mxx - o.x) * inv.x;
  float t0y = (mny - o.y) * inv.y, t1y = (mxy - o.y) * inv.y;
  float t0z = (mnz - o.z) * inv.z, t1z = (mxz - o.z) * inv.z;
  E = pt_maxf(pt_maxf(pt_minf(t0x, t1x), pt_minf(t0y, t1y)), pt_maxf(pt_minf(t0z, t1z), tmin));
  X = pt_minf(pt_minf(pt_maxf(t0x, t1x), pt_maxf(t0y, t1y)), pt_maxf(t0z, t1z));
}

__device__ __forceinline__ pt_f2 pt_f2s(float v) { return pt_f2{v, v}; }

#ifndef PTMI_PROBE
#define PTMI_PROBE 0
#endif
#if PTMI_PROBE
__device__ unsigned long long g_probe[16];
#endif

// Node stride (include/ptmi.h, ptmi_node_bytes()). The traversal reads the
// first 64 B (boxes, refs, z centres) and computes the x / y centres; the
// last 16 B hold them precomputed and are not read. A/B on MI355X (round 4,
// parity-identical): a 64-B stride without them, C2 -1.2 %, C4 -1.1 %, C5
// -0.7 %, C3 +-0 (profiles/r04/ab/ab_r04z_node64.log), so the stride stays 80.
constexpr uint32_t kNodeBytes = 80;

// In-flight traversal of one ray: begin (root test, push root) and one pop
// of the loop per step, so a kernel can interleave steps of different rays'
// traversals with other work; traverse() runs begin + steps to completion.
struct Trav {
  pt_v3 inv;
  float tmin, closest;
  int32_t best;  // leaf code of the closest hit; 0 = none (leaf codes are negative)
  uint32_t sp;   // LDS byte address of the next free stack slot
  uint32_t sp0;  // LDS byte address of slot 0: the stack is empty when sp == sp0
#if PTMI_PROBE == 2
  uint32_t probe;  // branches this lane took in the current step: 1 sphere, 2 quad/tri, 4 node
#endif
  __device__ __forceinline__ bool any() const { return best != 0; }
  __device__ __forceinline__ bool busy() const { return sp != sp0; }
  __device__ __forceinline__ void init(Stack st) { sp = sp0 = lds_addr(st.slot0); }
};

template <int STACK, int SB = kBlock>
__device__ __forceinline__ void trav_begin(const DevScene& sc, Trav& tr, Stack st, pt_v3 d, pt_v3 o, float tmin,
                                           float tmax) {
  tr.inv = pt_v3f(fabsf(d.x) > 1e-8f ? 1.0f / d.x : 1e8f, fabsf(d.y) > 1e-8f ? 1.0f / d.y : 1e8f,
                  fabsf(d.z) > 1e-8f ? 1.0f / d.z : 1e8f);  // kernels.py:642-646 (Q15)
  tr.tmin = tmin;
  tr.closest = tmax;
  tr.best = 0;
  tr.init(st);
  if (sc.n_inner == 0 && sc.root_ref >= 0) return;  // empty scene
  float E, X;
  slab(o, tr.inv, sc.root_min[0], sc.root_min[1], sc.root_min[2], sc.root_max[0], sc.root_max[1], sc.root_max[2],
       tmin, E, X);
  if (pt_minf(X, tr.closest) >= E) {
    lds_store2(tr.sp, (uint32_t)sc.root_ref, __float_as_uint(E));
    tr.sp += SB * 8;
  }
}

// One step of the traversal loop (one pop); precondition tr.busy().
// A/B on MI355X (parity-identical): deferring a popped leaf's test to the next
// step -5 % mk / -3.5 % wf; testing a just-pushed leaf in the expanding step
// -3 % mk (profiles/r01/ab_leaf_top.log). Sphere roots through a per-ray
// reciprocal of dot(d, d) (Markstein's fma sequence, bit-exact) and sqrt
// without the tiny/inf fix-ups: 14-20 VALU fewer per sphere test, and no
// faster (-0.5 %; profiles/r01/ab_fast_div_sqrt.log). One 80-B fetch per
// popped entry, node or primitive, issued before the node/leaf branch (one
// L2 wait per mixed step instead of two): -4.6 % mk, -14 % wf
// (profiles/r01/ab_unified_fetch.log); each lane's own entry load (node,
// sphere, quad or triangle) issued before any test, one wait per step, -4 %
// mk / -1 % wf (profiles/r01/ab_early_fetch.log). Node stride 128 B (one node
// per line) -5 %; 64-B nodes with x/y centres computed +0.4 % (noise), kept at
// 80 B (profiles/r01/ab_node_layout.log). Two-level 256-B node packets (a
// node's children and grandchildren, the near child expanded in the same
// step) -20 to -43 % (profiles/r02/ab/ab_trav2_packets.log).
//
// DEFER > 0 (leaf deferral): a lane whose top entry is a live leaf test
// (sphere, quad or triangle) keeps it (no pop) while fewer than DEFER lanes of
// the wave have a leaf test on top and some other lane has other work (a node
// step), so the leaf branches later run for more lanes at once. Each lane
// still pops its own entries in its own order: results are unchanged (GPU
// parity and counters green). The megakernel uses it (PTMI_MK_DEFER); A/B on
// MI355X against no deferral, with its shading threshold: every leaf at 12
// lanes, shading at <= 24 busy lanes: C2 +7.5 %, C5 +6.3 %, C4 +8 %; at 16 /
// 20 lanes +7 / +6 % (C2); quads and triangles only: C4 +6 %, C2 -3 %;
// spheres only at 4 / 8: C2 +0.5 %; triangles only -7 to -23 % (C4)
// (profiles/r03/ab/ab_leaf_defer.log; round 2's per-class forms,
// profiles/r02/ab/ab_leaf_defer.log).
template <int STACK, int SB = kBlock, int DEFER = 0, int LDS = STACK>
__device__ __forceinline__ void trav_step(const DevScene& sc, const float4* node_base, Trav& tr, Stack st, pt_v3 o,
                                          pt_v3 d) {
  // global address space: global_load, not flat_load (a laundered generic
  // pointer would otherwise lose it); clang vector type, no C++ copy ctor
  typedef float pt_f4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) pt_f4 gf4;
  gf4* nodes = (gf4*)node_base;
  constexpr uint32_t kSlot = SB * 8;  // bytes between a lane's consecutive slots
  const uint32_t lim = tr.sp0 + (uint32_t)LDS * kSlot;  // address of the first spilled slot (LDS < STACK)
  tr.sp -= kSlot;
  const pt_u2v ent = stack_load<STACK, LDS, SB>(st, lim, tr.sp);
  const int32_t ref = (int32_t)ent.x;
  // The pop's tests as lane masks, each computed once (round 5): leaf? and
  // live? (E <= closest), and with DEFER the deferred lanes; the cull, the
  // leaf / node branch and the deferral read the masks instead of re-issuing
  // compares, the non-deferred live lanes branch once, a deferred lane
  // restores its pointer by one select in a scalar branch taken only when some
  // lane defers. In the leaf branch the three primitive tests are independent
  // branches on the type's lane masks, each leaving its candidate t (one
  // register across them), and one compare after them updates the closest
  // hit (the tests take t < closest themselves, hit_*_t<true>). A/B on MI355X
  // (parity-identical, each against the step before it; profiles/r05/ab/):
  // deferral ballot from masks (no && materialised with v_cndmask + v_cmp)
  // C2 +1.0 %, C4 +0.6 %, C5 +0.9 % (ab_mk_defer_masks.log); the masks shared
  // by the cull and the branch C2 +1.8 %, C4 +1.4 %, C5 +1.8 %, mesh fog
  // wavefront +0.8 % (ab_step_masks.log); the closest-hit update inside each
  // type's branch with t < closest in the test +0.4 / +1.3 / +0.5 %, C3 +1 %
  // (ab_leaf_update.log); the deferred lanes as a mask and one branch level
  // fewer +1.0 / +1.4 / +1.0 % (ab_step_flat.log); independent type branches
  // with a candidate t +0.45 / +0.45 / +0.5 %, C3 +0.5 % (ab_leaf_tc.log).
  const unsigned long long m_leaf = pt_ballot(ref < 0), m_live = pt_ballot(__uint_as_float(ent.y) <= tr.closest);
  // leaf test (kernels.py:671-697) and node expansion (kernels.py:698-740),
  // for the lanes of each kind
  auto leaf_step = [&]() {
#if PTMI_PROBE == 2
    tr.probe |= leaf_type(ref) == kSphere ? 1 : 2;
#endif
    float t;
    const int32_t ty = leaf_type(ref), ix = leaf_index(ref);
    float tc = tr.closest;
    const unsigned long long m_s = pt_ballot(ty == kSphere), m_q = pt_ballot(ty == kQuad);
    if (__builtin_amdgcn_inverse_ballot_w64(m_s)) {
      if (hit_sphere_t<true>(sc.spheres[ix], o, d, tr.tmin, tr.closest, t)) tc = t;
    }
    if (__builtin_amdgcn_inverse_ballot_w64(m_q)) {
      if (hit_quad_t<true>(sc.quads + 4 * ix, o, d, tr.tmin, tr.closest, t)) tc = t;
    }
    if (__builtin_amdgcn_inverse_ballot_w64(~(m_s | m_q))) {
      if (hit_tri_t<true>(sc.tris + 3 * ix, o, d, tr.tmin, tr.closest, t)) tc = t;
    }
    if (tc < tr.closest) {
      tr.closest = tc;
      tr.best = ref;
    }
  };
  auto node_step = [&]() {
#if PTMI_PROBE == 2
    tr.probe |= 4;
#endif
#if PTMI_PROBE == 1
    {  // debug probe: node visits and wave-uniform node visits (lane counts)
      const int32_t ru = __builtin_amdgcn_readfirstlane(ref);
      const bool uni = __ballot(ref != ru) == 0ull;
      atomicAdd(&g_probe[0], 1ull);
      if (uni) atomicAdd(&g_probe[1], 1ull);
      const unsigned long long act = __ballot(true);
      if (__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u)) == 0) {
        atomicAdd(&g_probe[2], 1ull);  // wave-level node steps
        atomicAdd(&g_probe[3], (unsigned long long)__popcll(act));  // active lanes in them
      }
    }
#endif
    // internal: kernels.py:698-740, both children at once
    const pt_f2 ox = pt_f2s(o.x), oy = pt_f2s(o.y), oz = pt_f2s(o.z);
    const pt_f2 ix = pt_f2s(tr.inv.x), iy = pt_f2s(tr.inv.y), iz = pt_f2s(tr.inv.z);
    const pt_f2 dx = pt_f2s(d.x), dy = pt_f2s(d.y), dz = pt_f2s(d.z);
    const float tmin = tr.tmin;
    gf4* nd = (gf4*)((const __attribute__((address_space(1))) char*)nodes + (uint32_t)ref);  // the node at byte offset ref
    const pt_f4 A = nd[0], B = nd[1], C = nd[2], R = nd[3];
    const pt_f2 lox = {A.x, A.y}, loy = {A.z, A.w}, loz = {B.x, B.y};
    const pt_f2 hix = {B.z, B.w}, hiy = {C.x, C.y}, hiz = {C.z, C.w};
    const pt_f2 t0x = (lox - ox) * ix, t1x = (hix - ox) * ix;
    const pt_f2 t0y = (loy - oy) * iy, t1y = (hiy - oy) * iy;
    const pt_f2 t0z = (loz - oz) * iz, t1z = (hiz - oz) * iz;
    const float E0 = pt_maxf(pt_maxf(pt_minf(t0x.x, t1x.x), pt_minf(t0y.x, t1y.x)), pt_maxf(pt_minf(t0z.x, t1z.x), tmin));
    const float X0 = pt_minf(pt_minf(pt_maxf(t0x.x, t1x.x), pt_maxf(t0y.x, t1y.x)), pt_maxf(t0z.x, t1z.x));
    const float E1 = pt_maxf(pt_maxf(pt_minf(t0x.y, t1x.y), pt_minf(t0y.y, t1y.y)), pt_maxf(pt_minf(t0z.y, t1z.y), tmin));
    const float X1 = pt_minf(pt_minf(pt_maxf(t0x.y, t1x.y), pt_maxf(t0y.y, t1y.y)), pt_maxf(t0z.y, t1z.y));
    // projected centre distances dot(centre - o, d), (x + y) + z order (kernels.py:707-713)
    // x / y centres from the boxes just loaded, (min + max) * 0.5 as the
    // reference computes them (bit-identical); the z centres come with the
    // refs. A/B on MI355X (round 4, parity-identical), against loading all
    // three (a fifth 16-B load per node): C3 +2.4 %, C2 +0.9 %, C5 +0.9 %, C4
    // +-0 (profiles/r04/ab/ab_r04x_node_centres.log; the megakernel's
    // texture-address unit is 70 % busy, profiles/r04/pmc_ta/); the refs alone
    // as an 8-B load with the z centres computed too: C2 -4 %, C3 -2 %
    // (ab_r04y_node_refs_only.log).
    const pt_f2 cx = (lox + hix) * pt_f2s(0.5f), cy = (loy + hiy) * pt_f2s(0.5f), cz = {R.z, R.w};
    const pt_f2 dist = ((cx - ox) * dx + (cy - oy) * dy) + (cz - oz) * dz;
    const bool ln = dist.x < dist.y;  // child 0 is the near one; the far child is pushed first
    const bool h0 = X0 >= E0, h1 = X1 >= E1;
    // Far first, then near, each kept only if its box is hit: the far child
    // lands at sp and the near one at sp + slot when the far one is hit, else
    // the near one at sp and the (dropped) far one at sp + slot, above the
    // top. Child 0 takes the upper slot when (near and the far child 1 is hit)
    // or (far and missed). Writing each child's {ref, E} straight to its slot
    // needs no value selects. No bound check: an internal node at depth d has
    // at most d pending entries, so sp + 2 slots <= max_leaf_depth + 1 <= STACK
    // (enforced at dispatch) and the reference's overflow drop never triggers.
    // up0 = ln ? h1 : !h0, as and/or of the compares' lane masks (SALU; a bool
    // select would be materialised with four v_cndmask)
    const unsigned long long mln = pt_ballot(ln), mh0 = pt_ballot(h0), mh1 = pt_ballot(h1);
    const bool up0 = __builtin_amdgcn_inverse_ballot_w64((mln & mh1) | (~mln & ~mh0));
    const uint32_t lo = tr.sp, hi = tr.sp + kSlot;
    stack_store<STACK, LDS, SB>(st, lim, up0 ? hi : lo, __float_as_uint(R.x), __float_as_uint(E0));
    stack_store<STACK, LDS, SB>(st, lim, up0 ? lo : hi, __float_as_uint(R.y), __float_as_uint(E1));
    tr.sp += (h0 ? kSlot : 0u) + (h1 ? kSlot : 0u);
  };
  // With deferral the node lanes go first: their loads go out before the
  // deferral's scalar chain, which concerns leaf lanes only. A/B on MI355X
  // (parity-identical), with the chain itself shortened (1 <= nd < DEFER as
  // one unsigned compare, no early-out branch): C2 +1.3 %, C4 +1.2 %, C5
  // +1.2 % (node lanes first alone +0.7 / +0.7 / +0.7 %, the chain alone
  // +0.5 / +0.3 / +0.2 %); node lanes first in the wavefront's traversals
  // (no deferral): C3 -1.1 %, mesh fog +0.6 % (profiles/r05/ab/ab_node_first.log).
  if constexpr (DEFER > 0) {
    if (__builtin_amdgcn_inverse_ballot_w64(m_live & ~m_leaf)) node_step();
  }
  unsigned long long m_def = 0ull;  // deferred lanes
  if constexpr (DEFER > 0) {
    const unsigned long long md = m_leaf & m_live;
    const uint32_t nd = __builtin_popcount((uint32_t)md) + __builtin_popcount((uint32_t)(md >> 32));
    m_def = (nd - 1u < (uint32_t)(DEFER - 1) && md != pt_ballot(true)) ? md : 0ull;  // 1 <= nd < DEFER
    if (m_def != 0ull) tr.sp += __builtin_amdgcn_inverse_ballot_w64(m_def) ? kSlot : 0u;  // kept on top
  }
  const unsigned long long m_go = m_live & ~m_def;  // lanes that test their popped entry in this step
#if PTMI_PROBE == 1
  if (!__builtin_amdgcn_inverse_ballot_w64(m_def)) {
    atomicAdd(&g_probe[4], 1ull);                                                        // pops
    if (!__builtin_amdgcn_inverse_ballot_w64(m_live)) atomicAdd(&g_probe[5], 1ull);      // culled pops
    else if (ref < 0) atomicAdd(&g_probe[6 + (leaf_type(ref) == kSphere ? 0 : 1)], 1ull);  // leaf tests
  }
#endif
  if constexpr (DEFER > 0) {
    if (__builtin_amdgcn_inverse_ballot_w64(m_go & m_leaf)) leaf_step();
  } else {
    if (!__builtin_amdgcn_inverse_ballot_w64(m_go)) return;
    if (__builtin_amdgcn_inverse_ballot_w64(m_leaf)) {
      leaf_step();
      return;
    }
    node_step();
  }
}

// ---------------------------------------------------------------- stackless traversal
// traverse_bvh_stackless (kernels.py:453-597): the reference's alternative
// traversal, selected by its module constant USE_STACKLESS_TRAVERSAL
// (kernels.py:746; the frame's PTMI_TRAV_STACKLESS here). It walks the
// reference's own preorder nodes (ref_nodes, include/ptmi.h) left child
// first with parent pointers and no stack, one iteration of the reference's
// loop per step, at most 2 * num_bvh_nodes iterations (:487-491): a node's box
// is tested against [t_min, closest_t] when the walk enters it (:523), a
// leaf's primitive right after (:536-571), and the walk climbs back with the
// `came from` state (:497-520; the reference compares the parent's left child
// with the node, `side` in ref_nodes is that comparison precomputed). No LDS.
struct TravSL {
  pt_v3 inv;
  float tmin, closest;
  int32_t best;  // leaf code of the closest hit; 0 = none
  int32_t node;  // current node index; -1 = the walk has left the root
  int32_t came;  // -1 entering node, 0 back from its left child, 1 back from its right child
  int32_t it, max_it;
#if PTMI_PROBE == 2
  uint32_t probe;
#endif
  __device__ __forceinline__ bool any() const { return best != 0; }
  __device__ __forceinline__ bool busy() const { return node >= 0 && it < max_it; }
  __device__ __forceinline__ void init(Stack) {
    node = -1;
    it = max_it = 0;
    best = 0;
  }
};

template <int STACK, int SB = kBlock>
__device__ __forceinline__ void trav_begin(const DevScene& sc, TravSL& tr, Stack, pt_v3 d, pt_v3 o, float tmin,
                                           float tmax) {
  (void)o;
  tr.inv = pt_v3f(fabsf(d.x) > 1e-8f ? 1.0f / d.x : 1e8f, fabsf(d.y) > 1e-8f ? 1.0f / d.y : 1e8f,
                  fabsf(d.z) > 1e-8f ? 1.0f / d.z : 1e8f);  // kernels.py:478-482 (Q15)
  tr.tmin = tmin;
  tr.closest = tmax;
  tr.best = 0;
  tr.node = 0;
  tr.came = -1;
  tr.it = 0;
  tr.max_it = 2 * sc.n_nodes;
}

// One iteration of the reference's while loop (kernels.py:493-595).
template <int STACK, int SB = kBlock, int DEFER = 0, int LDS = STACK>
__device__ __forceinline__ void trav_step(const DevScene& sc, const float4*, TravSL& tr, Stack, pt_v3 o, pt_v3 d) {
  ++tr.it;
  const float4* nd = sc.ref_nodes + 3 * tr.node;
  const float4 s0 = nd[0], s1 = nd[1], s2 = nd[2];
  const int32_t left = __float_as_int(s0.w), right = __float_as_int(s1.w);
  bool up = false;
  if (tr.came == 0) {  // back from the left child: the right one next, else climb (:497-510)
    if (right >= 0) {
      tr.node = right;
      tr.came = -1;
      return;
    }
    up = true;
  } else if (tr.came == 1) {  // back from the right child: climb (:511-520)
    up = true;
  } else {
    // hit_aabb_optimized (kernels.py:601-621) against [t_min, closest_t]
    const float t0x = (s0.x - o.x) * tr.inv.x, t1x = (s1.x - o.x) * tr.inv.x;
    const float t0y = (s0.y - o.y) * tr.inv.y, t1y = (s1.y - o.y) * tr.inv.y;
    const float t0z = (s0.z - o.z) * tr.inv.z, t1z = (s1.z - o.z) * tr.inv.z;
    const float lo = pt_maxf(pt_maxf(pt_minf(t0x, t1x), pt_minf(t0y, t1y)), pt_maxf(pt_minf(t0z, t1z), tr.tmin));
    const float hi = pt_minf(pt_minf(pt_maxf(t0x, t1x), pt_maxf(t0y, t1y)), pt_minf(pt_maxf(t0z, t1z), tr.closest));
    const int32_t code = __float_as_int(s2.y);
    if (!(hi >= lo)) {
      up = true;  // :523-533
    } else if (code != 0) {  // leaf: test its primitive, then climb (:536-571)
#if PTMI_PROBE == 2
      tr.probe |= leaf_type(code) == kSphere ? 1 : 2;
#endif
      float t;
      if (hit_leaf(sc, code, o, d, tr.tmin, tr.closest, t) && t < tr.closest) {
        tr.closest = t;
        tr.best = code;
      }
      up = true;
    } else if (left >= 0) {  // internal: left child first (:572-595)
      tr.node = left;
      tr.came = -1;
    } else if (right >= 0) {
      tr.node = right;
      tr.came = -1;
    } else {
      up = true;
    }
  }
  if (up) {  // parent >= 0: came = which child this node is; else done
    const int32_t p = __float_as_int(s2.x);
    tr.came = __float_as_int(s2.z);
    tr.node = p;  // -1 at the root
  }
}

// ---------------------------------------------------------------- reference stack (deep BVHs)
// traverse_bvh_legacy (kernels.py:625-742) exactly as the reference runs it,
// for BVHs whose leaf depth exceeds 62: a 64-entry stack of node indices; the
// box of a popped node is tested against [t_min, closest_t] (:667); an
// internal node pushes both children unconditionally, the far one first by
// projected child-centre distance (:705-732; a missing child is skipped,
// :733-740), and a push is dropped once the stack holds 64 entries (the
// `if stack_ptr < 64` guards, :719-740). Trav (children culled at push, one
// slot per hit child) gives the same hits while no push is dropped, which
// leaf depth <= 62 guarantees; past that, the reference's dropped pushes are
// part of its result, so the dispatch runs this walk (kTravRefStack, STACK
// 64) on the reference's own nodes (ref_nodes) instead. Slot .x = node index.
constexpr int kTravRefStack = 2;  // internal: chosen by the dispatch (leaf depth > 62), not a frame setting
constexpr int kRefStackSlots = 64;  // kernels.py:649
struct TravRS {
  pt_v3 inv;
  float tmin, closest;
  int32_t best;  // leaf code of the closest hit; 0 = none
  uint32_t sp, sp0;
#if PTMI_PROBE == 2
  uint32_t probe;
#endif
  __device__ __forceinline__ bool any() const { return best != 0; }
  __device__ __forceinline__ bool busy() const { return sp != sp0; }
  __device__ __forceinline__ void init(Stack st) { sp = sp0 = lds_addr(st.slot0); }
};

template <int STACK, int SB = kBlock>
__device__ __forceinline__ void trav_begin(const DevScene& sc, TravRS& tr, Stack st, pt_v3 d, pt_v3 o, float tmin,
                                           float tmax) {
  static_assert(STACK >= kRefStackSlots, "the reference stack has 64 entries");
  (void)o;
  tr.inv = pt_v3f(fabsf(d.x) > 1e-8f ? 1.0f / d.x : 1e8f, fabsf(d.y) > 1e-8f ? 1.0f / d.y : 1e8f,
                  fabsf(d.z) > 1e-8f ? 1.0f / d.z : 1e8f);  // kernels.py:642-646 (Q15)
  tr.tmin = tmin;
  tr.closest = tmax;
  tr.best = 0;
  tr.init(st);
  if (sc.n_nodes > 0) {  // the root (:649-652); with no nodes the reference pops and skips it
    lds_store2(tr.sp, 0u, 0u);
    tr.sp += SB * 8;
  }
}

// One iteration of the reference's while loop (kernels.py:654-740).
template <int STACK, int SB = kBlock, int DEFER = 0, int LDS = STACK>
__device__ __forceinline__ void trav_step(const DevScene& sc, const float4*, TravRS& tr, Stack, pt_v3 o, pt_v3 d) {
  constexpr uint32_t kSlot = SB * 8;
  tr.sp -= kSlot;
  const int32_t ni = (int32_t)lds_load2(tr.sp).x;
  if (ni < 0 || ni >= sc.n_nodes) return;  // :660-661
  const float4* nd = sc.ref_nodes + 3 * ni;
  const float4 s0 = nd[0], s1 = nd[1], s2 = nd[2];
  const float t0x = (s0.x - o.x) * tr.inv.x, t1x = (s1.x - o.x) * tr.inv.x;  // hit_aabb_optimized :601-621
  const float t0y = (s0.y - o.y) * tr.inv.y, t1y = (s1.y - o.y) * tr.inv.y;
  const float t0z = (s0.z - o.z) * tr.inv.z, t1z = (s1.z - o.z) * tr.inv.z;
  const float lo = pt_maxf(pt_maxf(pt_minf(t0x, t1x), pt_minf(t0y, t1y)), pt_maxf(pt_minf(t0z, t1z), tr.tmin));
  const float hi = pt_minf(pt_minf(pt_maxf(t0x, t1x), pt_maxf(t0y, t1y)), pt_minf(pt_maxf(t0z, t1z), tr.closest));
  if (!(hi >= lo)) return;  // :667-668
  const int32_t code = __float_as_int(s2.y);
  if (code != 0) {  // leaf :671-697
#if PTMI_PROBE == 2
    tr.probe |= leaf_type(code) == kSphere ? 1 : 2;
#endif
    float t;
    if (hit_leaf(sc, code, o, d, tr.tmin, tr.closest, t) && t < tr.closest) {
      tr.closest = t;
      tr.best = code;
    }
    return;
  }
#if PTMI_PROBE == 2
  tr.probe |= 4;
#endif
  const int32_t left = __float_as_int(s0.w), right = __float_as_int(s1.w);
  const uint32_t cap = tr.sp0 + (uint32_t)kRefStackSlots * kSlot;  // `stack_ptr < 64`
  int32_t first = right, second = left;  // one child only: right, then left (:733-740)
  if (left >= 0 && right >= 0) {         // far child first (:705-732)
    const float4* ln = sc.ref_nodes + 3 * left;
    const float4* rn = sc.ref_nodes + 3 * right;
    const float4 l0 = ln[0], l1 = ln[1], r0 = rn[0], r1 = rn[1];
    const pt_v3 lc = pt_v3f((l0.x + l1.x) * 0.5f, (l0.y + l1.y) * 0.5f, (l0.z + l1.z) * 0.5f);
    const pt_v3 rc = pt_v3f((r0.x + r1.x) * 0.5f, (r0.y + r1.y) * 0.5f, (r0.z + r1.z) * 0.5f);
    if (!(pt_dot(pt_sub(lc, o), d) < pt_dot(pt_sub(rc, o), d))) {
      first = left;
      second = right;
    }
  }
  if (first >= 0 && tr.sp < cap) {
    lds_store2(tr.sp, (uint32_t)first, 0u);
    tr.sp += kSlot;
  }
  if (second >= 0 && tr.sp < cap) {
    lds_store2(tr.sp, (uint32_t)second, 0u);
    tr.sp += kSlot;
  }
}

// Traversal state type by frame.traversal (PTMI_TRAV_*), or kTravRefStack.
template <int TRAV>
struct TravOf {
  typedef Trav T;
};
template <>
struct TravOf<PTMI_TRAV_STACKLESS> {
  typedef TravSL T;
};
template <>
struct TravOf<kTravRefStack> {
  typedef TravRS T;
};

#ifndef PTMI_TRAV_UNROLL
#define PTMI_TRAV_UNROLL 3  // pops per loop test in traverse() (wavefront kernels; A/B: 3 +0.5 % C3 / mesh fog, 2 +0.3 %)
#endif
// No leaf deferral here: in the wavefront's one-ray-per-lane traversals it
// lost 3-12 % (DEFER 8 / 12 / 20, C3 and mesh fog; profiles/r03/ab/ab_leaf_defer.log).
template <int STACK, int SB = kBlock, int TRAV = PTMI_TRAV_STACK, int LDS = STACK>
__device__ __forceinline__ bool traverse(const DevScene& sc, pt_v3 o, pt_v3 d, float tmin, float tmax, Stack st,
                                         float& t_out, int32_t& ref_out) {
  typename TravOf<TRAV>::T tr;
  trav_begin<STACK, SB>(sc, tr, st, d, o, tmin, tmax);  // the root: slot 0, in LDS
  while (tr.busy()) {
#pragma unroll
    for (int u = 0; u < PTMI_TRAV_UNROLL; ++u)
      if (u == 0 || tr.busy()) trav_step<STACK, SB, 0, LDS>(sc, sc.nodes, tr, st, o, d);
  }
  t_out = tr.closest;
  ref_out = tr.best;
  return tr.any();
}

// ---------------------------------------------------------------- textures
struct Mat {
  float4 m0, m1, m2, m3, m4;
  __device__ __forceinline__ uint32_t flags() const { return __float_as_uint(m4.w); }
  __device__ __forceinline__ int32_t mat_type() const { return (int32_t)(flags() & 0xfu); }
  __device__ __forceinline__ int32_t tex_type() const { return (int32_t)((flags() >> 4) & 0xfu); }
  __device__ __forceinline__ bool is_medium() const { return (flags() >> 8) & 1u; }
  __device__ __forceinline__ int32_t image() const { return (int32_t)(flags() >> 16) - 1; }
};

__device__ __forceinline__ int32_t mat_index(const DevScene& sc, int32_t ref) {
  return sc.mat_base[leaf_type(ref)] + leaf_index(ref);
}
__device__ __forceinline__ uint32_t mat_flags(const DevScene& sc, int32_t g) {
  return __float_as_uint(sc.mats[5 * g + 4].w);
}

#ifndef PTMI_PERLIN_UNROLL
#define PTMI_PERLIN_UNROLL 1
#endif
__device__ __forceinline__ float perlin_noise(const DevScene& sc, pt_v3 p) {  // kernels.py:110-151
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int32_t i = pt_f2i(fx), j = pt_f2i(fy), k = pt_f2i(fz);
  float uu = u * u * (3.0f - 2.0f * u);
  float vv = v * v * (3.0f - 2.0f * v);
  float ww = w * w * (3.0f - 2.0f * w);
  const int32_t* px = sc.perlin_perm;
  const int32_t* py = sc.perlin_perm + 256;
  const int32_t* pz = sc.perlin_perm + 512;
  float accum = 0.0f;
  // outer corner loop rolled by default (-8 VGPRs; +2 % wavefront on MI355X)
#pragma unroll PTMI_PERLIN_UNROLL
  for (int di = 0; di < 2; ++di)
#pragma unroll
    for (int dj = 0; dj < 2; ++dj)
#pragma unroll
      for (int dk = 0; dk < 2; ++dk) {
        int32_t idx = px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255];
        float4 g = sc.perlin_vec[idx];
        pt_v3 wt = pt_v3f(u - (float)di, v - (float)dj, w - (float)dk);
        float fxw = di ? uu : (1.0f - uu);
        float fyw = dj ? vv : (1.0f - vv);
        float fzw = dk ? ww : (1.0f - ww);
        accum += fxw * fyw * fzw * pt_dot(pt_v3f(g.x, g.y, g.z), wt);
      }
  return accum;
}

__device__ __forceinline__ float perlin_turb3(const DevScene& sc, pt_v3 p) {  // kernels.py:155-169
  float accum = 0.0f, weight = 1.0f;
  pt_v3 tp = p;
#pragma unroll 1
  for (int oc = 0; oc < 3; ++oc) {
    accum += weight * perlin_noise(sc, tp);
    weight *= 0.5f;
    tp = pt_scale(tp, 2.0f);
  }
  return fabsf(accum);
}

// perlin_turb3 for the lanes of a wave that need it (need, at their p), the
// whole wave working on two of them at a time: lane c of each half computes
// term c of 24 — octave c >> 3, corner c & 7 — with perlin_noise's f32
// expressions (the octave point p * 2^oc is perlin_turb3's repeated doubling,
// exact), then every lane sums the two lanes' terms in perlin_noise's corner
// order and perlin_turb3's octave order, the same operations in the same
// sequence, so the result is bit-identical. A shading round with a few
// Perlin-textured hits otherwise runs the whole 3-octave evaluation (six
// dependent table loads, ~400 VALU) for one or two lanes; here a pair costs
// two table round trips and ~150 VALU. Call from wave-uniform control flow.
// A call, not inlined: A/B on MI355X (round 4, parity-identical) against the
// inlined form, C2 +1.4 %, C5 +1.3 %, C4 +1.2 % — inlined, its temporaries
// raise the register pressure of the whole persistent loop (scratch 36 ->
// 112 B/lane); as a call, the kernel keeps its 96 VGPRs and no scratch
// (profiles/r04/ab/ab_r04m_wave_turb.log).
__device__ __attribute__((noinline)) float perlin_turb3_wave(const DevScene& sc, bool need, pt_v3 p, int lane) {
  unsigned long long pend = pt_ballot(need);
  float res = 0.0f;
  const int c = lane & 31;
  const int oc = c >> 3, di = (c >> 2) & 1, dj = (c >> 1) & 1, dk = c & 1;
  const float oscale = oc == 0 ? 1.0f : (oc == 1 ? 2.0f : 4.0f);
  const int32_t* px = sc.perlin_perm;
  const int32_t* py = sc.perlin_perm + 256;
  const int32_t* pz = sc.perlin_perm + 512;
  while (pend != 0ull) {
    const int l0 = (int)__builtin_ctzll(pend);
    pend &= pend - 1ull;
    const int l1 = pend != 0ull ? (int)__builtin_ctzll(pend) : l0;
    if (pend != 0ull) pend &= pend - 1ull;
    const bool hi = lane >= 32;
    const float qx0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.x), l0));
    const float qy0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.y), l0));
    const float qz0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.z), l0));
    const float qx1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.x), l1));
    const float qy1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.y), l1));
    const float qz1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.z), l1));
    const pt_v3 tp = pt_scale(pt_v3f(hi ? qx1 : qx0, hi ? qy1 : qy0, hi ? qz1 : qz0), oscale);
    const float fx = floorf(tp.x), fy = floorf(tp.y), fz = floorf(tp.z);
    const float u = tp.x - fx, v = tp.y - fy, w = tp.z - fz;
    const int32_t i = pt_f2i(fx), j = pt_f2i(fy), k = pt_f2i(fz);
    const float uu = u * u * (3.0f - 2.0f * u);
    const float vv = v * v * (3.0f - 2.0f * v);
    const float ww = w * w * (3.0f - 2.0f * w);
    const int32_t idx = px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255];
    const float4 g = sc.perlin_vec[idx];
    const pt_v3 wt = pt_v3f(u - (float)di, v - (float)dj, w - (float)dk);
    const float fxw = di ? uu : (1.0f - uu);
    const float fyw = dj ? vv : (1.0f - vv);
    const float fzw = dk ? ww : (1.0f - ww);
    const float term = fxw * fyw * fzw * pt_dot(pt_v3f(g.x, g.y, g.z), wt);
    // corner sums as a left fold along each 8-lane octave group: after step
    // s, lane c holds (((0 + t[c-s]) + t[c-s+1]) ... + t[c]) (DPP row_shr:1
    // moves lane c-1's partial to lane c; groups do not cross 16-lane rows),
    // so lane 8 * oc + 7 ends with perlin_noise's accumulation
    float acc = 0.0f + term;
#pragma unroll
    for (int q = 1; q < 8; ++q)
      acc = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc), 0x111, 0xf, 0xf, false)) + term;
    const int ai = __float_as_int(acc);
    float t0 = 0.0f, t1 = 0.0f, wgt = 1.0f;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      t0 += wgt * __int_as_float(__builtin_amdgcn_readlane(ai, 8 * o + 7));
      t1 += wgt * __int_as_float(__builtin_amdgcn_readlane(ai, 32 + 8 * o + 7));
      wgt *= 0.5f;
    }
    if (lane == l0) res = fabsf(t0);
    if (lane == l1) res = fabsf(t1);
  }
  return res;
}

// image_texture (kernels.py:976-1008; get_sphere_uv :79-102): the Earth-map
// lookup of a sphere hit (magenta for other primitives).
// (A/B, not kept: as a call, not inlined, the megakernel spills 416 B/lane:
// a call from the divergent shading code saves the whole live state.)
__device__ __forceinline__ pt_v3 image_texture(const DevScene& sc, int32_t ref, const Mat& m, pt_v3 hp) {
  if (leaf_type(ref) != kSphere) return pt_v3f(1.0f, 0.0f, 1.0f);
  int32_t img = m.image();
  float4 s = sc.spheres[leaf_index(ref)];
  pt_v3 n = pt_normalize(pt_sub(hp, pt_v3f(s.x, s.y, s.z)));  // get_sphere_uv, kernels.py:79-102
  float phi = pt_acosf(-n.y);
  float theta = pt_atan2f(-n.z, n.x) + PT_PI_F;
  float u = theta / PT_2PI_F;
  float v = phi / PT_PI_F;
  if (img < 0 || img >= sc.num_images) return pt_v3f(1.0f, 1.0f, 1.0f);
  int32_t W = sc.img_w[img], H = sc.img_h[img];
  u = pt_maxf(0.0f, pt_minf(1.0f, u));
  v = 1.0f - pt_maxf(0.0f, pt_minf(1.0f, v));
  int32_t ii = pt_f2i(u * (float)W);
  int32_t jj = pt_f2i(v * (float)H);
  ii = ii < 0 ? 0 : (ii > W - 1 ? W - 1 : ii);
  jj = jj < 0 ? 0 : (jj > H - 1 ? H - 1 : jj);
  uint32_t px = sc.texels[sc.img_offset[img] + jj * W + ii];
  return pt_v3f((float)(px & 0xffu) / 255.0f, (float)((px >> 8) & 0xffu) / 255.0f,
                (float)((px >> 16) & 0xffu) / 255.0f);
}

// has_turb: turb is perlin_turb3(sc, hp), already evaluated (perlin_turb3_wave)
__device__ __forceinline__ pt_v3 eval_texture(const DevScene& sc, int32_t ref, const Mat& m, pt_v3 hp,
                                             bool has_turb = false, float turb = 0.0f) {
  // kernels.py:925-1017
  int32_t tex = m.tex_type();
  pt_v3 c1 = pt_v3f(m.m2.x, m.m2.y, m.m2.z);
  if (tex == 0) return c1;
  float scale = m.m2.w;
  if (tex == 1) {
    float inv_scale = 1.0f / scale;
    int32_t xi = pt_f2i(floorf(inv_scale * hp.x));
    int32_t yi = pt_f2i(floorf(inv_scale * hp.y));
    int32_t zi = pt_f2i(floorf(inv_scale * hp.z));
    int32_t s = (int32_t)((uint32_t)xi + (uint32_t)yi + (uint32_t)zi);
    return (s % 2 == 0) ? c1 : pt_v3f(m.m3.x, m.m3.y, m.m3.z);
  }
  if (tex == 2) return image_texture(sc, ref, m, hp);
  if (tex == 3) {
    float nv = pt_sinf(scale * hp.z + 10.0f * (has_turb ? turb : perlin_turb3(sc, hp)));
    return pt_scale(pt_scale(c1, 0.5f), 1.0f + nv);
  }
  return pt_v3f(1.0f, 1.0f, 1.0f);
}

// ---------------------------------------------------------------- materials
__device__ __forceinline__ pt_v3 reflect3(pt_v3 v, pt_v3 n) {  // kernels.py:767-769
  return pt_sub(v, pt_scale(n, 2.0f * pt_dot(v, n)));
}
__device__ __forceinline__ pt_v3 refract3(pt_v3 uv, pt_v3 n, float eta) {  // kernels.py:773-778
  float ct = pt_minf(-pt_dot(uv, n), 1.0f);
  pt_v3 perp = pt_scale(pt_add(uv, pt_scale(n, ct)), eta);
  pt_v3 par = pt_scale(n, -sqrtf(fabsf(1.0f - pt_dot(perp, perp))));
  return pt_add(perp, par);
}
__device__ __forceinline__ float reflectance(float c, float ri) {  // kernels.py:782-786
  float r0 = (1.0f - ri) / (1.0f + ri);
  r0 = r0 * r0;
  return r0 + (1.0f - r0) * pt_pow5f(1.0f - c);
}

// Dielectric scatter direction, kernels.py:876-903 (attenuation 1).
__device__ __forceinline__ pt_v3 scatter_dielectric(const Mat& m, pt_v3 dir, pt_v3 n, Rng& r) {
  float ir = m.m1.w;
  bool front = pt_dot(dir, n) < 0.0f;
  pt_v3 nf = front ? n : pt_neg(n);
  float ratio = front ? (1.0f / ir) : ir;
  pt_v3 ud = pt_normalize(dir);
  float ct = pt_minf(-pt_dot(ud, nf), 1.0f);
  float st = sqrtf(1.0f - ct * ct);
  bool cannot = ratio * st > 1.0f;
  float u = r.next();  // unconditional draw
  return (cannot || reflectance(ct, ratio) > u) ? reflect3(ud, nf) : refract3(ud, nf, ratio);
}

// scatter(), kernels.py:818-917. Returns scattered; writes direction and
// attenuation. Material record already loaded.
__device__ __forceinline__ bool scatter(const DevScene& sc, int32_t ref, const Mat& m, pt_v3 dir, pt_v3 hp,
                                     pt_v3 n, Rng& r, pt_v3& sdir, pt_v3& att) {
  int32_t mt = m.mat_type();
  sdir = pt_v3f(0.0f, 0.0f, 0.0f);
  att = pt_v3f(1.0f, 1.0f, 1.0f);
  if (mt == 0) {
    att = eval_texture(sc, ref, m, hp);
    sdir = random_cosine_direction(n, r);
    return true;
  }
  if (mt == 1) {
    pt_v3 refl = reflect3(pt_normalize(dir), n);
    sdir = pt_add(refl, pt_scale(random_unit_vector(r), m.m0.w));
    if (pt_dot(sdir, n) > 0.0f) {
      att = pt_v3f(m.m0.x, m.m0.y, m.m0.z);
      return true;
    }
    return false;
  }
  if (mt == 2) {
    sdir = scatter_dielectric(m, dir, n, r);
    return true;
  }
  if (mt == 4) {
    sdir = random_unit_vector(r);
    att = eval_texture(sc, ref, m, hp);
    return true;
  }
  return false;  // emissive (3) and unknown types
}

// scatter() in two parts around its random unit vector (metal fuzz and
// isotropic, kernels.py:865-871, 911-915), so that a kernel shading several
// lanes can draw the unit vectors of every lane that needs one (these and the
// constant-medium scatter, kernels.py:1082-1097) at one call site: the
// rejection loop then runs once, to the wave's longest lane, instead of once
// per divergent branch. Each lane's draws keep their order: nothing these
// materials do before the unit vector draws, and the isotropic texture
// (evaluated before it, at the Lambertian's texture site) draws nothing.
// scatter_begin returns the pending kind; scatter_end finishes it.
enum : int32_t { kRuvNone = 0, kRuvMetal = 1, kRuvIso = 2, kRuvMedium = 3 };

__device__ __forceinline__ int32_t scatter_begin(const DevScene& sc, int32_t ref, const Mat& m, pt_v3 dir,
                                                 pt_v3 hp, pt_v3 n, Rng& r, pt_v3& sdir, pt_v3& att,
                                                 bool& scattered, bool has_turb = false, float turb = 0.0f) {
  int32_t mt = m.mat_type();
  sdir = pt_v3f(0.0f, 0.0f, 0.0f);
  att = pt_v3f(1.0f, 1.0f, 1.0f);
  scattered = false;
  if (mt == 0 || mt == 4) att = eval_texture(sc, ref, m, hp, has_turb, turb);  // one texture site (draws nothing)
  if (mt == 0) {
    sdir = random_cosine_direction(n, r);
    scattered = true;
    return kRuvNone;
  }
  if (mt == 1) {
    sdir = reflect3(pt_normalize(dir), n);  // the reflection; the fuzz is added in scatter_end
    return kRuvMetal;
  }
  if (mt == 2) {
    sdir = scatter_dielectric(m, dir, n, r);
    scattered = true;
    return kRuvNone;
  }
  if (mt == 4) return kRuvIso;
  return kRuvNone;  // emissive (3) and unknown types
}

// v: the lane's random_unit_vector draw. Returns scattered.
__device__ __forceinline__ bool scatter_end(const DevScene& sc, int32_t kind, int32_t ref, const Mat& m, pt_v3 hp,
                                            pt_v3 n, pt_v3 v, pt_v3& sdir, pt_v3& att) {
  if (kind == kRuvMetal) {
    sdir = pt_add(sdir, pt_scale(v, m.m0.w));
    if (pt_dot(sdir, n) > 0.0f) {
      att = pt_v3f(m.m0.x, m.m0.y, m.m0.z);
      return true;
    }
    return false;
  }
  sdir = v;  // kRuvIso (att: its texture, from scatter_begin)
  return true;
}

__device__ __forceinline__ Mat load_mat(const DevScene& sc, int32_t g) {
  const float4* p = sc.mats + 5 * g;
  Mat m;
  m.m0 = p[0]; m.m1 = p[1]; m.m2 = p[2]; m.m3 = p[3]; m.m4 = p[4];
  return m;
}

__device__ __forceinline__ pt_v3 emitted(const Mat& m) {  // kernels.py:790-814
  return (m.mat_type() == 3) ? pt_v3f(m.m1.x, m.m1.y, m.m1.z) : pt_v3f(0.0f, 0.0f, 0.0f);
}

// Second half of apply_constant_medium (kernels.py:421-448) once the exit
// traversal from t_entry + 1e-4 has been done. Returns is_medium_hit and the
// scatter point; t_exit = 0 when no exit was found.
__device__ __forceinline__ bool medium_step(bool hit_exit, float t_exit_hit, float t_entry, float density,
                                            pt_v3 o, pt_v3 d, Rng& r, pt_v3& p, float& t_exit) {
  t_exit = 0.0f;
  if (!hit_exit) return false;
  t_exit = t_exit_hit;
  float t1 = pt_maxf(t_entry, kTMin);
  float t2 = pt_minf(t_exit, kTMax);
  if (t1 < t2) {
    if (t1 < 0.0f) t1 = 0.0f;
    float rl = sqrtf(pt_dot(d, d));
    float inside = (t2 - t1) * rl;
    float hd = -pt_logf(pt_maxf(r.next(), 1e-10f)) / density;
    if (hd < inside) {
      float ts = t1 + hd / rl;
      p = pt_add(o, pt_scale(d, ts));
      return true;
    }
  }
  return false;
}

}  // namespace ptmi
