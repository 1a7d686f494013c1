/*
 * ptmi.h — C-ABI of libptmi.so, the MI355X (gfx950) path-tracing integrator.
 *
 * This is the drop-in boundary for the reference's hot loop: the Taichi
 * kernels the reference launches directly from its host class
 * (src/render_server/taichi_renderer/renderer.py) — there is no FFI in the
 * reference, so each entry point below names the reference launch/host site it
 * replaces. Plain C types only: device pointers are raw pointers owned by the
 * caller (the Python host allocates them as torch tensors); the library never
 * allocates device memory inside a render call (it owns a small pinned
 * readback area and, per device, the wavefront's 3 extra streams and their
 * events, created on first use). All functions return 0 on success and a
 * negative PTMI_E* code on error; ptmi_last_error() gives a message.
 */
#ifndef PTMI_H
#define PTMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTMI_ABI_VERSION 7
#define PTMI_MAX_IMAGES 16

enum {
    PTMI_OK = 0,
    PTMI_EINVAL = -1,      /* bad argument / shape */
    PTMI_ECAPACITY = -2,   /* scene exceeds a structural limit (e.g. BVH depth) */
    PTMI_EHIP = -3,        /* HIP runtime error */
    PTMI_ENODEV = -4,      /* no gfx950 device */
};

/* Device scene, packed by the host from the reference's compiled arrays
 * (scene_compiler.py:931 compile_scene + bvh_compiler.py:132 compile_bvh;
 * replaces the field uploads of renderer.py:102-228 / fields.py:25-153).
 * Layouts (all little-endian, 16-byte aligned):
 *   nodes   : n_inner x 20 f32 (80 B) — internal BVH2 node holding BOTH
 *             children's boxes, interleaved per component so the two
 *             children form packed-f32 pairs: {min.x c0,c1, min.y c0,c1 |
 *             min.z c0,c1, max.x c0,c1 | max.y c0,c1, max.z c0,c1 |
 *             ref0, ref1 (i32 bits), centre.z c0,c1 | centre.x c0,c1,
 *             centre.y c0,c1}; centre = (min + max) * 0.5f in f32 (the
 *             kernels read the first 64 B and compute centre.x / .y from
 *             the boxes, the same operations; the last 16 B stay packed).
 *             ref >= 0: internal node, as its BYTE offset in nodes
 *             (index x 80: the traversal adds it to the node base with
 *             no index scaling); ref < 0: leaf code
 *             0x80000000 | type << 28 | class << 25 | prim index (type: 0
 *             sphere, 1 triangle, 2 quad — scene_compiler.py:10-12; class:
 *             the primitive's PTMI_CLASS_* from its material flags, used by
 *             the wavefront to sort hits by material without a load;
 *             prim index < 2^25 per type). ABI v6.
 *   spheres : ns x 4 f32 {cx, cy, cz, r}                (fields.py:25)
 *   quads   : nq x 16 f32 {n.xyz, D | Q.xyz, u.x | u.yz, v.xy | v.z, w.xyz}
 *   tris    : nt x 12 f32 {v0.xyz, e1.x | e1.yz, e2.xy | e2.z, n.xyz}
 *   mats    : (ns+nq+nt) x 20 f32, spheres then quads then triangles:
 *             {albedo.xyz, fuzz | emit.xyz, ir | color1.xyz, tex_scale |
 *              color2.xyz, density | medium_albedo.xyz, flags(u32 bits)}
 *             flags = mat_type | tex_type << 4 | is_medium << 8 |
 *                     (image_index + 1) << 16
 *   texels  : RGBA8 texels of all image textures, image k at img_offset[k]
 *   perlin_vec  : 256 x 4 f32 (randvec, w unused)
 *   perlin_perm : 3 x 256 i32 (perm_x, perm_y, perm_z)
 *   ref_nodes   : num_bvh_nodes x 12 f32 (48 B), the reference's own
 *             flattened nodes in its preorder (sah_bvh_builder.py:338-418,
 *             fields.py:52-63) for the stackless traversal
 *             (PTMI_TRAV_STACKLESS): {min.xyz, left | max.xyz, right |
 *             parent, leaf code (0 = internal), side, 0} (i32 bits), side = 0
 *             when the node is its parent's left child, else 1. Used by the
 *             stackless traversal and by BVHs of leaf depth > 62 (the
 *             reference's 64-entry stack walk); may be NULL otherwise.
 */
typedef struct ptmi_scene_view {
    const float *nodes;
    int32_t n_inner;
    int32_t root_ref;          /* ref of the root (0 if internal) */
    float root_min[3], root_max[3];
    int32_t max_leaf_depth;    /* root = 0; sizes the traversal stack. Past 62 the
                                  kernels run the reference's own 64-entry stack
                                  walk on ref_nodes (kernels.py:625-742, pushes
                                  beyond 64 entries dropped), so ref_nodes must be
                                  set (PTMI_EINVAL otherwise) */
    const float *spheres;
    const float *quads;
    const float *tris;
    const float *mats;
    int32_t num_spheres, num_quads, num_triangles;
    const uint32_t *texels;
    int32_t num_images;
    int32_t img_offset[PTMI_MAX_IMAGES], img_w[PTMI_MAX_IMAGES], img_h[PTMI_MAX_IMAGES];
    const float *perlin_vec;
    const int32_t *perlin_perm;
    const float *ref_nodes;
    int32_t num_bvh_nodes;     /* all nodes: 2 x primitives - 1 (0 for an empty world) */
} ptmi_scene_view;

/* Camera upload values (renderer.py:230-247 / fields.py:159-165). */
typedef struct ptmi_camera {
    float center[3], pixel00[3], delta_u[3], delta_v[3], defocus_u[3], defocus_v[3];
    float defocus_angle;
} ptmi_camera;

/* BVH traversal (traverse_bvh, kernels.py:749-759, switched by the module
 * constant USE_STACKLESS_TRAVERSAL, kernels.py:746): the reference's default
 * stack traversal with front-to-back child order (traverse_bvh_legacy,
 * kernels.py:625-742), or its parent-pointer stackless traversal, left child
 * first (traverse_bvh_stackless, kernels.py:453-597; needs ref_nodes). */
enum { PTMI_TRAV_STACK = 0, PTMI_TRAV_STACKLESS = 1 };

/* One render request: camera + render state (fields.py:171-172) + the pixel
 * set this call owns. The pixel set is the window [x0,x0+w) x [y0,y0+h)
 * restricted to rows whose band ((row - y0) / band_rows) satisfies
 * band % band_stride == band_offset (band_stride = 1: every row). Multi-GPU
 * tile sharding uses band_stride = world size, band_offset = rank. */
typedef struct ptmi_frame {
    ptmi_camera cam;
    float bg[3];
    int32_t max_depth;
    uint32_t seed;
    int32_t width, height;
    int32_t x0, y0, w, h;
    int32_t band_rows, band_stride, band_offset;
    int32_t traversal;         /* PTMI_TRAV_* */
} ptmi_frame;

/* Device counters (u64): [0] ray segments traced from the depth loop / waves,
 * [1] medium-exit traversals (kernels.py:417), [2] completed paths,
 * [3] paths ended by Russian roulette (kernels.py:1145-1157, the reference's
 * rr_paths_killed, fields.py:295), [4] paths ended by the depth / wave budget
 * (kernels.py:1139-1141, 1383; renderer.py:313: its max_depth_terminations,
 * fields.py:287), [5] the part of [0] the wavefront traced in its one-launch
 * tail (wf_drain; 0 for the megakernel), so per-kernel rates can attribute
 * segments to the launch that traced them. Accumulated with atomics; pass
 * NULL to skip. [3] and [4] since ABI v6, [5] since ABI v7 (the buffer must
 * hold PTMI_NUM_COUNTERS entries). */
#define PTMI_NUM_COUNTERS 6
#define PTMI_COUNTER_TAIL_SEGMENTS 5

/* Material class in a leaf code (bits 25-27), from the material flags:
 * constant-medium boundary; Perlin-textured Lambertian or isotropic; else by
 * material type: Lambertian 0, dielectric 2, emissive 3, glossy otherwise
 * (metal 1, isotropic 4, unknown types). */
#define PTMI_CLASS_LAMBERTIAN 0
#define PTMI_CLASS_GLOSSY 1
#define PTMI_CLASS_DIELECTRIC 2
#define PTMI_CLASS_MEDIUM 3
#define PTMI_CLASS_NOISE 4
#define PTMI_CLASS_EMISSIVE 5

int ptmi_version(void);
const char *ptmi_last_error(void);

/* Byte stride of the library's BVH node array (the `nodes` layout above):
 * 80, one child record per internal node. Internal refs are node index x
 * this stride. */
int ptmi_node_bytes(void);

/* Checks a scene view's counts, alignment and structural limits on the host. */
int ptmi_scene_check(const ptmi_scene_view *scene);

/* Megakernel: replaces kernels.render_sample() (kernels.py:1177-1202) as
 * launched by TaichiRenderer.render() (renderer.py:405-409) and
 * InteractiveViewer (interactive_viewer.py:389): accumulates samples
 * [sample_begin, sample_begin + sample_count) of every pixel of the frame's
 * pixel set into accum (height x width x 3 f32, row-major), adding each
 * sample's colour in sample order. One launch covers many samples (each
 * thread regenerates its pixel's next path as the previous one ends). */
int ptmi_mk_render(const ptmi_scene_view *scene, const ptmi_frame *frame, float *accum,
                   int32_t sample_begin, int32_t sample_count, uint64_t *counters, void *stream);

/* Megakernel with persistent waves: one round of the chip's wave slots, each
 * wave drawing (8x8 tile, sample) units from a device counter in `workspace`
 * until the batch is done, so a launch has no partly occupied last round.
 * Each path's colour goes to a staging slot [sample][pixel] of `workspace`
 * and a resolve kernel adds them into accum in sample order: same results,
 * bit for bit, as ptmi_mk_render. A batch holds fewer than 2^32 (8x8 tile,
 * sample, pixel) item ids: larger calls run as several batches.
 * workspace: device memory (16-byte aligned)
 * of at least ptmi_mk_workspace_bytes(frame, 1) bytes;
 * ptmi_mk_workspace_bytes(frame, B) = 12 * pixels * B (rounded up to 256) +
 * 2048 (8 work-counter lines) lets one batch hold B samples. Asynchronous, graph-capturable. */
size_t ptmi_mk_workspace_bytes(const ptmi_frame *frame, int32_t batch_samples);
int ptmi_mk_render_ws(const ptmi_scene_view *scene, const ptmi_frame *frame, void *workspace,
                      size_t workspace_bytes, float *accum, int32_t sample_begin, int32_t sample_count,
                      uint64_t *counters, void *stream);

/* The two halves of ptmi_mk_render_ws for one batch, for callers that
 * schedule them on different streams: ptmi_mk_trace_ws runs the megakernel
 * for samples [sample_begin, sample_begin + sample_count) of every pixel of
 * the frame into the workspace's staging slots (the accumulator is not
 * touched; the whole call must fit one batch: workspace_bytes >=
 * ptmi_mk_workspace_bytes(frame, sample_count)); ptmi_mk_resolve_ws then
 * adds those sample_count staged colours into accum in sample order. Trace
 * then resolve gives, bit for bit, what ptmi_mk_render_ws gives. With two
 * workspaces a caller can start the next batch's trace while the previous
 * one drains (its last long paths leave most of the chip idle; ~1.5 ms per
 * launch on vol2_final_scene) and keep the resolves in order on one stream. */
int ptmi_mk_trace_ws(const ptmi_scene_view *scene, const ptmi_frame *frame, void *workspace,
                     size_t workspace_bytes, int32_t sample_begin, int32_t sample_count, uint64_t *counters,
                     void *stream);
/* Largest sample_count one ptmi_mk_trace_ws batch of this frame accepts (its
 * (8x8 tile, sample, pixel) item ids must stay below 2^32); 0 on a bad frame.
 * ABI v6. */
int64_t ptmi_mk_max_batch(const ptmi_frame *frame);
int ptmi_mk_resolve_ws(const ptmi_frame *frame, const void *workspace, size_t workspace_bytes, float *accum,
                       int32_t sample_count, void *stream);

/* Wavefront: replaces generate_camera_rays / intersect_rays /
 * shade_miss_rays / reset_next_ray_count / shade_and_scatter /
 * swap_ray_buffers (kernels.py:1219-1418) as driven by
 * TaichiRenderer.render_wavefront() (renderer.py:305-334), with the same
 * accumulation semantics as ptmi_mk_render. workspace: device memory
 * (16-byte aligned) of at least ptmi_wf_workspace_bytes(frame, 1) bytes;
 * ptmi_wf_workspace_bytes(frame, B) bytes let one batch hold B samples of
 * every pixel (ray queues + a per-(sample, pixel) staging slot). Larger
 * sample counts run in batches. The queue runs as 4 independent pipes: pipe 0
 * on `stream`, pipes 1-3 on library-owned streams forked from `stream` and
 * joined back into it with events, so the work is ordered after earlier and
 * before later work on `stream` like one launch. Synchronises the pipes once
 * every few queue iterations to read their live-ray counts (not
 * graph-capturable). Thread-safe: the library's per-device streams, events
 * and pinned readback slots are created under a per-device lock, and calls on
 * one device are serialised by that lock (calls on different devices run
 * concurrently). Launches go to the current HIP device, which must be the
 * device holding the pointers. Batches are capped at 2^31 - 1 (sample,
 * pixel) work items, padded to whole 8x8 squares and chunks, whatever the
 * workspace size (the item word's top bit flags a fresh camera ray). */
size_t ptmi_wf_workspace_bytes(const ptmi_frame *frame, int32_t batch_samples);
int ptmi_wf_render(const ptmi_scene_view *scene, const ptmi_frame *frame, void *workspace,
                   size_t workspace_bytes, float *accum, int32_t sample_begin, int32_t sample_count,
                   uint64_t *counters, void *stream);
/* Schedule knob of ptmi_wf_render's tail (no effect on results): once the
 * work pool is dry and a pipe traces fewer than capacity / divisor rays per
 * iteration, one launch finishes the paths still in its ray buffer (its
 * continuing rays), instead of one intersect and one scatter launch per
 * remaining wave. 0 = no tail launch; default 16. Process-wide, read at the
 * start of each batch. Returns the previous divisor, or PTMI_EINVAL for a
 * negative one. ABI v7. */
int ptmi_wf_set_drain_at(int32_t divisor);

/* Clears the accumulator's pixel set: kernels.clear_accum_buffer()
 * (kernels.py:1205-1209) / fields.clear_accumulation_buffer (fields.py:280). */
int ptmi_clear(const ptmi_frame *frame, float *accum, void *stream);

/* Tone map: LivePreview.buffer_to_image (preview.py:117-132):
 * u8 = clip(sqrt(max(0, accum * (1/max(1,spp)))) * 255.999, 0, 255). */
int ptmi_tonemap(const float *accum, uint8_t *out, int32_t width, int32_t height, int32_t spp,
                 void *stream);

/* Host-side binned-SAH BVH build (sah_bvh_builder.py:167-418 via
 * build_sah_bvh_from_primitives :445-485), f32 arithmetic identical to the
 * reference under NumPy >= 2 (NEP 50). Inputs (f32): spheres ns x 4
 * {c.xyz, r}; quads nq x 9 {Q, u, v}; tris nt x 9 {v0, v1, v2}. Outputs are the
 * 7 flattened arrays, capacity 2*(ns+nq+nt)-1 nodes; *n_nodes receives the
 * count. */
int ptmi_bvh_build_sah(const float *spheres, int32_t ns, const float *quads, int32_t nq,
                       const float *tris, int32_t nt, float *bbox_min, float *bbox_max,
                       int32_t *left, int32_t *right, int32_t *parent, int32_t *prim_type,
                       int32_t *prim_idx, int32_t *n_nodes);

/* Per-kernel device timing of this library's own launches (HIP events on
 * the launch stream; the reference's Taichi kernel profiler, renderer.py:15-16).
 * ptmi_prof_start pre-creates events for max_launches launches; render calls
 * then record around every kernel; ptmi_prof_stop synchronises, returns the
 * summed milliseconds and launch counts per kernel kind
 * {0 megakernel, 1 wf_generate, 2 wf_intersect, 3 (retired: the separate
 * wf_shade of earlier versions, no launches), 4 wf_scatter (shading and the
 * medium exit search, one launch per wavefront iteration), 5 wf_resolve,
 * 6 mk_resolve} and disables timing. One profiling session
 * per process; render calls from several host threads may record into it
 * (each launch owns its event pair; the session is mutex-guarded). */
#define PTMI_PROF_KINDS 7
int ptmi_prof_start(int32_t max_launches);
int ptmi_prof_stop(double *ms_by_kernel, uint64_t *launches_by_kernel, int32_t n_kinds);
/* As ptmi_prof_stop, plus per kind the busy time: the length of the union of
 * its launches' [start, end] event intervals. Pipelined launches of one kind
 * (two staged megakernel calls in flight on two streams, the wavefront's
 * pipes) overlap, so their summed durations exceed the GPU time they take;
 * busy / launches is the GPU time per launch. busy_ms_by_kernel may be NULL. */
int ptmi_prof_stop_busy(double *ms_by_kernel, double *busy_ms_by_kernel, uint64_t *launches_by_kernel,
                        int32_t n_kinds);

#ifdef __cplusplus
}
#endif
#endif /* PTMI_H */
