/*
 * pt_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * CPU restatement of the reference integrator
 * src/render_server/taichi_renderer/kernels.py over the reference's own data
 * layout (fields.py:25-165: per-primitive-type SoA arrays, 44-byte BVH nodes
 * as flattened by sah_bvh_builder.py:338-418). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.
 *
 * Pixel parity against Taichi itself is unpinned (Taichi cannot run here,
 * SURVEY.md §8c); the scene/BVH arrays this oracle consumes are pinned
 * bit-exactly by tests/golden fixtures generated from the reference.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>

#define OR_MAX_IMAGES 16

/* Primitive type codes, scene_compiler.py:10-12. Index of the per-type arrays. */
enum { OR_SPHERE = 0, OR_TRIANGLE = 1, OR_QUAD = 2 };

typedef struct or_scene {
    int32_t num_spheres, num_quads, num_triangles, num_bvh_nodes;
    const float *sphere_data;                              /* (ns,4) fields.py:25 */
    const float *quad_Q, *quad_u, *quad_v, *quad_normal;   /* (nq,3) fields.py:38-43 */
    const float *quad_D, *quad_w;
    const float *tri_v0, *tri_e1, *tri_e2, *tri_normal;    /* (nt,3) fields.py:29-34 */
    /* material / texture / medium arrays indexed [prim_type] (fields.py:70-138) */
    const int32_t *mat_type[3];
    const float *albedo[3], *fuzz[3], *ir[3], *emit[3];
    const int32_t *tex_type[3];
    const float *tex_scale[3], *color1[3], *color2[3];
    const int32_t *img_idx[3];
    const int32_t *is_medium[3];
    const float *density[3], *med_albedo[3];
    /* flattened BVH (sah_bvh_builder.py:392-398) */
    const float *bvh_min, *bvh_max;
    const int32_t *bvh_left, *bvh_right, *bvh_type, *bvh_idx;
    /* Perlin tables (fields.py:148-153) */
    const float *perlin_vec;
    const int32_t *perm_x, *perm_y, *perm_z;
    /* image textures: RGB8, value = u8/255 in f32 (rtw_image.py:66) */
    int32_t num_images;
    const uint8_t *images[OR_MAX_IMAGES];
    int32_t img_w[OR_MAX_IMAGES], img_h[OR_MAX_IMAGES];
    /* parent pointers of the flattened BVH (sah_bvh_builder.py:398), read by
       the stackless traversal only */
    const int32_t *bvh_parent;
} or_scene;

/* BVH traversal of traverse_bvh (kernels.py:749-759): USE_STACKLESS_TRAVERSAL
 * (kernels.py:746) False -> traverse_bvh_legacy (:625-742, the reference's
 * default), True -> traverse_bvh_stackless (:453-597). */
enum { OR_TRAV_STACK = 0, OR_TRAV_STACKLESS = 1 };

typedef struct or_frame {
    float center[3], pixel00[3], delta_u[3], delta_v[3], defocus_u[3], defocus_v[3];
    float defocus_angle;
    float bg[3];
    int32_t max_depth;
    uint32_t seed;
    int32_t width, height;
    int32_t traversal;   /* OR_TRAV_* */
} or_frame;

typedef struct or_stats {
    uint64_t segments;   /* traverse_bvh calls from the depth loop / waves */
    uint64_t medium;     /* medium-exit traversals (kernels.py:417) */
    uint64_t paths;
    uint64_t rr;         /* paths ended by Russian roulette (kernels.py:1145-1157) */
    uint64_t depth_cap;  /* paths ended by the depth / wave budget (kernels.py:1139-1141, 1383; renderer.py:313) */
} or_stats;

#ifdef __cplusplus
extern "C" {
#endif
int or_version(void);
/* variant 0 = megakernel (render_sample, kernels.py:1177), 1 = wavefront
 * (renderer.py:305-334 + kernels.py:1219-1418). Accumulates samples
 * [s_begin, s_begin+s_count) into accum (H,W,3) for the pixels of the window
 * [x0,x0+w) x [y0,y0+h). */
int or_render(const or_scene *sc, const or_frame *fr, int variant, float *accum,
              int x0, int y0, int w, int h, int s_begin, int s_count, int threads,
              or_stats *stats);
int or_traverse(const or_scene *sc, int traversal, const float *o, const float *d, float tmin, float tmax,
                float *t_out, int32_t *type_out, int32_t *idx_out);
/* one path: returns its colour contribution and counters */
int or_trace_path(const or_scene *sc, const or_frame *fr, int variant, int px, int py, int sample,
                  float *color_out, or_stats *stats);
/* math / rng probes for the known-answer tests */
void or_math_probe(int fn, const float *x, const float *y, float *out, int n);
/* per-function probes (known-answer tests against the reference's own Python,
 * tests/golden/gen_functions.py). fn, input record -> output record:
 *  0 perlin_noise    p[3] (sc's Perlin tables)           -> value
 *  1 perlin_turb     p[3], depth                          -> value
 *  2 get_sphere_uv   p[3], center[3]                      -> u, v
 *  3 reflect         v[3], n[3]                           -> r[3]
 *  4 refract         uv[3], n[3], eta                     -> r[3]
 *  5 reflectance     cosine, ref_idx                      -> value
 *  6 hit_sphere      c[3], r, o[3], d[3], tmin, tmax      -> hit, t
 *  7 hit_quad        Q, u, v, normal[3], D, w[3], o, d, tmin, tmax -> hit, t
 *  8 hit_triangle    v0, e1, e2, normal[3], o, d, tmin, tmax       -> hit, t
 * Returns the input record length of fn (0 for an unknown fn). */
int or_func_probe(const or_scene *sc, int fn, const float *in, float *out, int n);
void or_rng_probe(uint32_t seed, uint32_t pixel, uint32_t sample, int n, float *out, uint32_t *key_out);
#ifdef __cplusplus
}
#endif
#endif
