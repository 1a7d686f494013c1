/*
 * pt_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference
 * integrator (src/render_server/taichi_renderer/kernels.py). Every function
 * follows the cited lines of the reference; ti.random() is replaced by the
 * counter-based stream of include/ptmi_rng.h and transcendental functions by
 * include/ptmi_math.h (the arithmetic contract shared with the HIP kernels).
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include "pt_oracle.h"
#include "../include/ptmi_math.h"
#include "../include/ptmi_rng.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct rng_t { uint32_t key, n; } rng_t;
static inline float draw(rng_t *r) { return pt_rand(r->key, r->n++); }

static inline pt_v3 ld3(const float *a, int i) { return pt_v3f(a[3 * i], a[3 * i + 1], a[3 * i + 2]); }

/* ---------------- RNG helpers, kernels.py:16-71 ---------------- */

static pt_v3 random_in_unit_disk(rng_t *r) {                 /* kernels.py:17-25 */
    for (;;) {
        float x = draw(r) * 2.0f - 1.0f;
        float y = draw(r) * 2.0f - 1.0f;
        pt_v3 p = pt_v3f(x, y, 0.0f);
        if (pt_dot(p, p) < 1.0f) return p;
    }
}

static pt_v3 random_unit_vector(rng_t *r) {                  /* kernels.py:29-38 */
    for (;;) {
        float x = draw(r) * 2.0f - 1.0f;
        float y = draw(r) * 2.0f - 1.0f;
        float z = draw(r) * 2.0f - 1.0f;
        pt_v3 p = pt_v3f(x, y, z);
        float lensq = pt_dot(p, p);
        if (lensq < 1.0f && lensq > 1e-20f) return pt_normalize(p);
    }
}

static pt_v3 random_cosine_direction(pt_v3 normal, rng_t *r) { /* kernels.py:42-71 */
    float r1 = draw(r);
    float r2 = draw(r);
    float z = sqrtf(1.0f - r2);
    float phi = PT_2PI_F * r1;
    float sin_theta = sqrtf(r2);
    float sp, cp;
    pt_sincosf(phi, &sp, &cp);
    float x = cp * sin_theta;
    float y = sp * sin_theta;
    pt_v3 w = pt_normalize(normal);
    pt_v3 a;
    if (fabsf(w.x) < 0.9f) a = pt_v3f(1.0f, 0.0f, 0.0f);
    else if (fabsf(w.y) < 0.9f) a = pt_v3f(0.0f, 1.0f, 0.0f);
    else a = pt_v3f(0.0f, 0.0f, 1.0f);
    pt_v3 v = pt_normalize(pt_cross(a, w));   /* "SWAPPED" basis, kernels.py:67-68 */
    pt_v3 u = pt_cross(v, w);
    pt_v3 d = pt_add(pt_add(pt_scale(u, x), pt_scale(v, y)), pt_scale(w, z));
    return pt_normalize(d);
}

/* ---------------- textures, kernels.py:78-169, 924-1017 ---------------- */

static void get_sphere_uv(pt_v3 p, pt_v3 center, float *u, float *v) { /* kernels.py:79-102 */
    pt_v3 n = pt_normalize(pt_sub(p, center));
    float phi = pt_acosf(-n.y);
    float theta = pt_atan2f(-n.z, n.x) + PT_PI_F;
    *u = theta / PT_2PI_F;
    *v = phi / PT_PI_F;
}

static float perlin_noise(const or_scene *sc, pt_v3 p) {    /* kernels.py:110-151 */
    float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
    float u = p.x - fx, v = p.y - fy, w = p.z - fz;
    int32_t i = pt_f2i(fx), j = pt_f2i(fy), k = pt_f2i(fz);
#ifndef OR_NEGATIVE_CONTROL_NO_HERMITE
    float uu = u * u * (3.0f - 2.0f * u);
    float vv = v * v * (3.0f - 2.0f * v);
    float ww = w * w * (3.0f - 2.0f * w);
#else  /* tests/test_functions.py negative control only: a deliberately wrong Perlin */
    float uu = u, vv = v, ww = w;
#endif
    float accum = 0.0f;
    for (int di = 0; di < 2; ++di)
        for (int dj = 0; dj < 2; ++dj)
            for (int dk = 0; dk < 2; ++dk) {
                int32_t idx = sc->perm_x[(i + di) & 255] ^ sc->perm_y[(j + dj) & 255] ^ sc->perm_z[(k + dk) & 255];
                pt_v3 g = ld3(sc->perlin_vec, idx);
                pt_v3 wt = pt_v3f(u - (float)di, v - (float)dj, w - (float)dk);
                float fxw = di ? uu : (1.0f - uu);
                float fyw = dj ? vv : (1.0f - vv);
                float fzw = dk ? ww : (1.0f - ww);
                accum += fxw * fyw * fzw * pt_dot(g, wt);
            }
    return accum;
}

static float perlin_turb(const or_scene *sc, pt_v3 p, int depth) { /* kernels.py:155-169 */
    float accum = 0.0f, weight = 1.0f;
    pt_v3 tp = p;
    for (int o = 0; o < depth; ++o) {
        accum += weight * perlin_noise(sc, tp);
        weight *= 0.5f;
        tp = pt_scale(tp, 2.0f);
    }
    return fabsf(accum);
}

static pt_v3 eval_texture(const or_scene *sc, int pt, int pi, pt_v3 hp) { /* kernels.py:925-1017 */
    int tex = sc->tex_type[pt][pi];
    pt_v3 c1 = ld3(sc->color1[pt], pi), c2 = ld3(sc->color2[pt], pi);
    float scale = sc->tex_scale[pt][pi];
    int img = sc->img_idx[pt][pi];
    pt_v3 result = pt_v3f(1.0f, 1.0f, 1.0f);
    if (tex == 0) {
        result = c1;
    } else if (tex == 1) {
        float inv_scale = 1.0f / scale;
        int32_t xi = pt_f2i(floorf(inv_scale * hp.x));
        int32_t yi = pt_f2i(floorf(inv_scale * hp.y));
        int32_t zi = pt_f2i(floorf(inv_scale * hp.z));
        int32_t s = (int32_t)((uint32_t)xi + (uint32_t)yi + (uint32_t)zi);
        result = (s % 2 == 0) ? c1 : c2;   /* == 0 test is sign-agnostic */
    } else if (tex == 2) {
        if (pt == OR_SPHERE) {
            const float *sd = sc->sphere_data + 4 * pi;
            float u, v;
            get_sphere_uv(hp, pt_v3f(sd[0], sd[1], sd[2]), &u, &v);
            if (img >= 0 && img < sc->num_images) {
                int W = sc->img_w[img], H = sc->img_h[img];
                u = pt_maxf(0.0f, pt_minf(1.0f, u));
                v = 1.0f - pt_maxf(0.0f, pt_minf(1.0f, v));
                int32_t ii = pt_f2i(u * (float)W);
                int32_t jj = pt_f2i(v * (float)H);
                ii = ii < 0 ? 0 : (ii > W - 1 ? W - 1 : ii);
                jj = jj < 0 ? 0 : (jj > H - 1 ? H - 1 : jj);
                const uint8_t *px = sc->images[img] + 3 * ((size_t)jj * (size_t)W + (size_t)ii);
                result = pt_v3f((float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f);
            }
        } else {
            result = pt_v3f(1.0f, 0.0f, 1.0f);
        }
    } else if (tex == 3) {
        float nv = pt_sinf(scale * hp.z + 10.0f * perlin_turb(sc, hp, 3));
        result = pt_scale(pt_scale(c1, 0.5f), 1.0f + nv);
    }
    return result;
}

/* ---------------- intersection, kernels.py:208-362, 600-742 ---------------- */

typedef struct hit_t { int hit; float t; pt_v3 p, n; int type, idx; } hit_t;

static int hit_sphere(const or_scene *sc, int i, pt_v3 o, pt_v3 d, float tmin, float tmax, hit_t *h) {
    const float *s = sc->sphere_data + 4 * i;                 /* kernels.py:209-248 */
    pt_v3 c = pt_v3f(s[0], s[1], s[2]);
    float radius = s[3];
    pt_v3 oc = pt_sub(c, o);
    float a = pt_dot(d, d);
    float hh = pt_dot(d, oc);
    float cc = pt_dot(oc, oc) - radius * radius;
    float disc = hh * hh - a * cc;
    if (disc >= 0.0f) {
        float sq = sqrtf(disc);
        float root = (hh - sq) / a;
        if (root < tmin || root > tmax) root = (hh + sq) / a;
        if (root >= tmin && root <= tmax) {
            h->t = root;
            h->p = pt_add(o, pt_scale(d, root));
            h->n = pt_divs(pt_sub(h->p, c), radius);
            return 1;
        }
    }
    return 0;
}

static int hit_triangle(const or_scene *sc, int i, pt_v3 o, pt_v3 d, float tmin, float tmax, hit_t *h) {
    pt_v3 v0 = ld3(sc->tri_v0, i), e1 = ld3(sc->tri_e1, i);   /* kernels.py:252-307 */
    pt_v3 e2 = ld3(sc->tri_e2, i), n = ld3(sc->tri_normal, i);
    pt_v3 hv = pt_cross(d, e2);
    float det = pt_dot(e1, hv);
    if (fabsf(det) >= 1e-8f) {
        float inv = 1.0f / det;
        pt_v3 s = pt_sub(o, v0);
        float u = inv * pt_dot(s, hv);
        if (u >= 0.0f && u <= 1.0f) {
            pt_v3 q = pt_cross(s, e1);
            float v = inv * pt_dot(d, q);
            if (v >= 0.0f && u + v <= 1.0f) {
                float t = inv * pt_dot(e2, q);
                if (t >= tmin && t <= tmax) {
                    h->t = t;
                    h->p = pt_add(o, pt_scale(d, t));
                    h->n = (pt_dot(d, n) > 0.0f) ? pt_neg(n) : n;
                    return 1;
                }
            }
        }
    }
    return 0;
}

static int hit_quad(const or_scene *sc, int i, pt_v3 o, pt_v3 d, float tmin, float tmax, hit_t *h) {
    pt_v3 Q = ld3(sc->quad_Q, i), u = ld3(sc->quad_u, i), v = ld3(sc->quad_v, i); /* kernels.py:311-362 */
    pt_v3 n = ld3(sc->quad_normal, i), w = ld3(sc->quad_w, i);
    float D = sc->quad_D[i];
    float denom = pt_dot(n, d);
    if (fabsf(denom) >= 1e-8f) {
        float t = (D - pt_dot(n, o)) / denom;
        if (t >= tmin && t <= tmax) {
            pt_v3 ip = pt_add(o, pt_scale(d, t));
            pt_v3 pv = pt_sub(ip, Q);
            float alpha = pt_dot(w, pt_cross(pv, v));
            float beta = pt_dot(w, pt_cross(u, pv));
            if (alpha >= 0.0f && alpha <= 1.0f && beta >= 0.0f && beta <= 1.0f) {
                h->t = t;
                h->p = ip;
                h->n = (denom < 0.0f) ? n : pt_neg(n);
                return 1;
            }
        }
    }
    return 0;
}

static int hit_aabb(const float *bmin, const float *bmax, pt_v3 o, pt_v3 inv, float tmin, float tmax) {
    /* kernels.py:601-621 */
    float t0x = (bmin[0] - o.x) * inv.x, t1x = (bmax[0] - o.x) * inv.x;
    float t0y = (bmin[1] - o.y) * inv.y, t1y = (bmax[1] - o.y) * inv.y;
    float t0z = (bmin[2] - o.z) * inv.z, t1z = (bmax[2] - o.z) * inv.z;
    float mnx = pt_minf(t0x, t1x), mny = pt_minf(t0y, t1y), mnz = pt_minf(t0z, t1z);
    float mxx = pt_maxf(t0x, t1x), mxy = pt_maxf(t0y, t1y), mxz = pt_maxf(t0z, t1z);
    float lo = pt_maxf(pt_maxf(mnx, mny), pt_maxf(mnz, tmin));
    float hi = pt_minf(pt_minf(mxx, mxy), pt_minf(mxz, tmax));
    return hi >= lo;
}

static int traverse_bvh(const or_scene *sc, pt_v3 o, pt_v3 d, float tmin, float tmax, hit_t *out) {
    /* traverse_bvh_legacy, kernels.py:625-742 (active via :746-759) */
    hit_t best; memset(&best, 0, sizeof best);
    best.t = tmax;
    float closest = tmax;
    pt_v3 inv = pt_v3f(fabsf(d.x) > 1e-8f ? 1.0f / d.x : 1e8f,
                       fabsf(d.y) > 1e-8f ? 1.0f / d.y : 1e8f,
                       fabsf(d.z) > 1e-8f ? 1.0f / d.z : 1e8f);
#ifndef OR_STACK_SLOTS
#define OR_STACK_SLOTS 64   /* kernels.py:649; other values only for the tests' overflow control */
#endif
    int32_t stack[OR_STACK_SLOTS];
    int sp = 0;
    stack[sp++] = 0;
    int any = 0;
    while (sp > 0) {
        int32_t ni = stack[--sp];
        if (ni < 0 || ni >= sc->num_bvh_nodes) continue;
        const float *bmin = sc->bvh_min + 3 * ni, *bmax = sc->bvh_max + 3 * ni;
        if (!hit_aabb(bmin, bmax, o, inv, tmin, closest)) continue;
        int32_t pidx = sc->bvh_idx[ni];
        if (pidx >= 0) {
            int32_t ptype = sc->bvh_type[ni];
            hit_t h; int hit = 0;
            if (ptype == OR_SPHERE) hit = hit_sphere(sc, pidx, o, d, tmin, closest, &h);
            else if (ptype == OR_TRIANGLE) hit = hit_triangle(sc, pidx, o, d, tmin, closest, &h);
            else if (ptype == OR_QUAD) hit = hit_quad(sc, pidx, o, d, tmin, closest, &h);
            if (hit && h.t < closest) {
                any = 1;
                closest = h.t;
                best = h;
                best.type = ptype;
                best.idx = pidx;
            }
        } else {
            int32_t l = sc->bvh_left[ni], r = sc->bvh_right[ni];
            if (l >= 0 && r >= 0) {
                const float *lmn = sc->bvh_min + 3 * l, *lmx = sc->bvh_max + 3 * l;
                const float *rmn = sc->bvh_min + 3 * r, *rmx = sc->bvh_max + 3 * r;
                pt_v3 lc = pt_v3f((lmn[0] + lmx[0]) * 0.5f, (lmn[1] + lmx[1]) * 0.5f, (lmn[2] + lmx[2]) * 0.5f);
                pt_v3 rc = pt_v3f((rmn[0] + rmx[0]) * 0.5f, (rmn[1] + rmx[1]) * 0.5f, (rmn[2] + rmx[2]) * 0.5f);
                float ld = pt_dot(pt_sub(lc, o), d);
                float rd = pt_dot(pt_sub(rc, o), d);
                if (ld < rd) {
                    if (sp < OR_STACK_SLOTS) stack[sp++] = r;
                    if (sp < OR_STACK_SLOTS) stack[sp++] = l;
                } else {
                    if (sp < OR_STACK_SLOTS) stack[sp++] = l;
                    if (sp < OR_STACK_SLOTS) stack[sp++] = r;
                }
            } else {
                if (r >= 0 && sp < OR_STACK_SLOTS) stack[sp++] = r;
                if (l >= 0 && sp < OR_STACK_SLOTS) stack[sp++] = l;
            }
        }
    }
    best.hit = any;
    best.t = closest;
    if (!any) { best.t = 0.0f; best.type = 0; best.idx = 0; }
    *out = best;
    return any;
}

static int traverse_bvh_stackless(const or_scene *sc, pt_v3 o, pt_v3 d, float tmin, float tmax, hit_t *out) {
    /* traverse_bvh_stackless, kernels.py:453-597 (selected when
       USE_STACKLESS_TRAVERSAL, :746): left child first, parent pointers,
       at most 2 * num_bvh_nodes loop iterations (:487-491) */
    hit_t best; memset(&best, 0, sizeof best);
    float closest = tmax;
    int any = 0;
    pt_v3 inv = pt_v3f(fabsf(d.x) > 1e-8f ? 1.0f / d.x : 1e8f,   /* :478-482 */
                       fabsf(d.y) > 1e-8f ? 1.0f / d.y : 1e8f,
                       fabsf(d.z) > 1e-8f ? 1.0f / d.z : 1e8f);
    int32_t node = 0;
    int came = -1;   /* -1 none, 0 left, 1 right (:484-485) */
    int64_t max_it = (int64_t)sc->num_bvh_nodes * 2, it = 0;
    while (node >= 0 && it < max_it) {
        ++it;
        int up = 0;   /* ascend to the parent this iteration */
        if (came == 0) {                                      /* :497-510 */
            int32_t r = sc->bvh_right[node];
            if (r >= 0) { node = r; came = -1; continue; }
            up = 1;
        } else if (came == 1) {                               /* :511-520 */
            up = 1;
        } else if (!hit_aabb(sc->bvh_min + 3 * node, sc->bvh_max + 3 * node, o, inv, tmin, closest)) {
            up = 1;                                           /* :523-533 */
        } else if (sc->bvh_idx[node] >= 0) {                  /* leaf, :536-571 */
            int32_t pidx = sc->bvh_idx[node], ptype = sc->bvh_type[node];
            hit_t h; int hit = 0;
            if (ptype == OR_SPHERE) hit = hit_sphere(sc, pidx, o, d, tmin, closest, &h);
            else if (ptype == OR_TRIANGLE) hit = hit_triangle(sc, pidx, o, d, tmin, closest, &h);
            else if (ptype == OR_QUAD) hit = hit_quad(sc, pidx, o, d, tmin, closest, &h);
            if (hit && h.t < closest) {
                any = 1;
                closest = h.t;
                best = h;
                best.type = ptype;
                best.idx = pidx;
            }
            up = 1;
        } else {                                              /* internal, :572-595 */
            int32_t l = sc->bvh_left[node], r = sc->bvh_right[node];
            if (l >= 0) { node = l; came = -1; }
            else if (r >= 0) { node = r; came = -1; }
            else up = 1;
        }
        if (up) {   /* parent_idx >= 0: came = which child we were; else done */
            int32_t p = sc->bvh_parent[node];
            if (p < 0) break;
            came = (sc->bvh_left[p] == node) ? 0 : 1;
            node = p;
        }
    }
    best.hit = any;
    best.t = closest;
    if (!any) { best.t = 0.0f; best.type = 0; best.idx = 0; }
    *out = best;
    return any;
}

static int traverse(const or_scene *sc, int mode, pt_v3 o, pt_v3 d, float tmin, float tmax, hit_t *out) {
    /* traverse_bvh, kernels.py:749-759 */
    return mode == OR_TRAV_STACKLESS ? traverse_bvh_stackless(sc, o, d, tmin, tmax, out)
                                     : traverse_bvh(sc, o, d, tmin, tmax, out);
}

/* ---------------- constant medium, kernels.py:365-450 ---------------- */

typedef struct medium_t { int is_hit; float t_scatter; pt_v3 p; float t_exit; } medium_t;

static medium_t apply_constant_medium(const or_scene *sc, int mode, int pt, int pi, pt_v3 o, pt_v3 d,
                                      float tmin, float tmax, float t_entry, rng_t *r, or_stats *st) {
    medium_t m; m.is_hit = 0; m.t_scatter = 0.0f; m.p = pt_v3f(0.0f, 0.0f, 0.0f); m.t_exit = 0.0f;
    int is_med = sc->is_medium[pt][pi];
    float density = sc->density[pt][pi];
    if (is_med > 0) {
        hit_t ex;
        if (st) st->medium++;
        int hit_exit = traverse(sc, mode, o, d, t_entry + 0.0001f, 1e10f, &ex);
        if (hit_exit) {
            m.t_exit = ex.t;
            float t1 = pt_maxf(t_entry, tmin);
            float t2 = pt_minf(m.t_exit, tmax);
            if (t1 < t2) {
                if (t1 < 0.0f) t1 = 0.0f;
                float ray_length = sqrtf(pt_dot(d, d));
                float inside = (t2 - t1) * ray_length;
                float hit_distance = -pt_logf(pt_maxf(draw(r), 1e-10f)) / density;
                if (hit_distance < inside) {
                    m.t_scatter = t1 + hit_distance / ray_length;
                    m.p = pt_add(o, pt_scale(d, m.t_scatter));
                    m.is_hit = 1;
                }
            }
        }
    }
    return m;
}

/* ---------------- materials, kernels.py:766-917 ---------------- */

static pt_v3 reflect(pt_v3 v, pt_v3 n) { return pt_sub(v, pt_scale(n, 2.0f * pt_dot(v, n))); }

static pt_v3 refract(pt_v3 uv, pt_v3 n, float eta) {          /* kernels.py:773-778 */
    float cos_theta = pt_minf(-pt_dot(uv, n), 1.0f);
    pt_v3 perp = pt_scale(pt_add(uv, pt_scale(n, cos_theta)), eta);
    pt_v3 par = pt_scale(n, -sqrtf(fabsf(1.0f - pt_dot(perp, perp))));
    return pt_add(perp, par);
}

static float reflectance(float cosine, float ref_idx) {       /* kernels.py:782-786 */
    float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    r0 = r0 * r0;
    return r0 + (1.0f - r0) * pt_pow5f(1.0f - cosine);
}

static pt_v3 emitted(const or_scene *sc, int pt, int pi) {    /* kernels.py:790-814 */
    if (sc->mat_type[pt][pi] == 3) return ld3(sc->emit[pt], pi);
    return pt_v3f(0.0f, 0.0f, 0.0f);
}

static int scatter(const or_scene *sc, pt_v3 dir, pt_v3 hp, pt_v3 n, int pt, int pi,
                   pt_v3 *sdir, pt_v3 *att, rng_t *r) {        /* kernels.py:818-917 */
    int mt = sc->mat_type[pt][pi];
    *sdir = pt_v3f(0.0f, 0.0f, 0.0f);
    *att = pt_v3f(1.0f, 1.0f, 1.0f);
    if (mt == 0) {
        pt_v3 albedo = eval_texture(sc, pt, pi, hp);
        *sdir = random_cosine_direction(n, r);
        *att = albedo;
        return 1;
    } else if (mt == 1) {
        pt_v3 albedo = ld3(sc->albedo[pt], pi);
        float fuzz = sc->fuzz[pt][pi];
        pt_v3 refl = reflect(pt_normalize(dir), n);
        *sdir = pt_add(refl, pt_scale(random_unit_vector(r), fuzz));
        if (pt_dot(*sdir, n) > 0.0f) { *att = albedo; return 1; }
        return 0;
    } else if (mt == 2) {
        float ir = sc->ir[pt][pi];
        int front = pt_dot(dir, n) < 0.0f;
        pt_v3 nf = front ? n : pt_neg(n);
        float ratio = front ? (1.0f / ir) : ir;
        pt_v3 ud = pt_normalize(dir);
        float cos_theta = pt_minf(-pt_dot(ud, nf), 1.0f);
        float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
        int cannot = ratio * sin_theta > 1.0f;
        float u = draw(r);   /* drawn unconditionally: Taichi `or` is not short-circuit */
        if (cannot || reflectance(cos_theta, ratio) > u) *sdir = reflect(ud, nf);
        else *sdir = refract(ud, nf, ratio);
        *att = pt_v3f(1.0f, 1.0f, 1.0f);
        return 1;
    } else if (mt == 3) {
        return 0;
    } else if (mt == 4) {
        *sdir = random_unit_vector(r);
        *att = eval_texture(sc, pt, pi, hp);
        return 1;
    }
    return 0;
}

/* ---------------- ray generation, kernels.py:177-201 ---------------- */

static void get_ray(const or_frame *fr, int px, int py, rng_t *r, pt_v3 *o, pt_v3 *d) {
    float ox = draw(r) - 0.5f;
    float oy = draw(r) - 0.5f;
    pt_v3 p00 = pt_v3f(fr->pixel00[0], fr->pixel00[1], fr->pixel00[2]);
    pt_v3 du = pt_v3f(fr->delta_u[0], fr->delta_u[1], fr->delta_u[2]);
    pt_v3 dv = pt_v3f(fr->delta_v[0], fr->delta_v[1], fr->delta_v[2]);
    pt_v3 ps = pt_add(pt_add(p00, pt_scale(du, (float)px + ox)), pt_scale(dv, (float)py + oy));
    pt_v3 c = pt_v3f(fr->center[0], fr->center[1], fr->center[2]);
    pt_v3 ro = c;
    if (fr->defocus_angle > 0.0f) {
        pt_v3 p = random_in_unit_disk(r);
        pt_v3 fu = pt_v3f(fr->defocus_u[0], fr->defocus_u[1], fr->defocus_u[2]);
        pt_v3 fv = pt_v3f(fr->defocus_v[0], fr->defocus_v[1], fr->defocus_v[2]);
        ro = pt_add(pt_add(c, pt_scale(fu, p.x)), pt_scale(fv, p.y));
    }
    *o = ro;
    *d = pt_sub(ps, ro);
}

/* ---------------- megakernel path, kernels.py:1025-1170 ---------------- */

static pt_v3 trace_ray_mk(const or_scene *sc, const or_frame *fr, pt_v3 ro, pt_v3 rd, rng_t *r, or_stats *st) {
    pt_v3 color = pt_v3f(0.0f, 0.0f, 0.0f);
    pt_v3 thr = pt_v3f(1.0f, 1.0f, 1.0f);
    pt_v3 o = ro;
    pt_v3 d = pt_normalize(rd);                               /* Q1: kernels.py:1042 */
    pt_v3 bg = pt_v3f(fr->bg[0], fr->bg[1], fr->bg[2]);
    for (int depth = 0; depth < fr->max_depth; ++depth) {
        hit_t h;
        if (st) st->segments++;
        int hit = traverse(sc, fr->traversal, o, d, 0.001f, 1e10f, &h);
        if (hit) {
            int pt = h.type, pi = h.idx;
            int is_med = sc->is_medium[pt][pi];
            int scattered = 0, passthrough = 0;
            pt_v3 sdir = pt_v3f(0.0f, 0.0f, 0.0f), att = pt_v3f(1.0f, 1.0f, 1.0f);
            pt_v3 hp = h.p, n = h.n;
            if (is_med > 0) {
                medium_t m = apply_constant_medium(sc, fr->traversal, pt, pi, o, d, 0.001f, 1e10f, h.t, r, st);
                if (m.is_hit) {
                    hp = m.p;
                    n = pt_v3f(1.0f, 0.0f, 0.0f);
                    sdir = random_unit_vector(r);
                    att = ld3(sc->med_albedo[pt], pi);
                    scattered = 1;
                } else if (m.t_exit > 0.0f) {
                    passthrough = 1;
                    float ray_length = sqrtf(pt_dot(d, d));
                    float eps_t = 0.001f / ray_length;
                    o = pt_add(o, pt_scale(d, m.t_exit + eps_t));
                } else {
                    color = pt_add(color, pt_mul(thr, emitted(sc, pt, pi)));
                    scattered = scatter(sc, d, hp, n, pt, pi, &sdir, &att, r);
                }
            } else {
                color = pt_add(color, pt_mul(thr, emitted(sc, pt, pi)));
                scattered = scatter(sc, d, hp, n, pt, pi, &sdir, &att, r);
            }
            (void)n;
            if (scattered) {
                o = hp;
                d = sdir;
                thr = pt_mul(thr, att);
                if (depth + 1 >= fr->max_depth) {
                    if (st) st->depth_cap++;
                    break;
                }
                if (depth + 1 >= 5) {
                    float sp = pt_minf(pt_maxf(pt_maxf(thr.x, thr.y), thr.z), 0.95f);
                    if (draw(r) > sp) {
                        if (st) st->rr++;
                        break;
                    }
                    thr = pt_divs(thr, sp);
                }
            } else if (passthrough) {
                if (depth + 1 >= fr->max_depth && st) st->depth_cap++;  /* the loop ends: kernels.py:1054 */
            } else {
                break;
            }
        } else {
            color = pt_add(color, pt_mul(thr, bg));
            break;
        }
    }
    return color;
}

/* ---------------- wavefront path (per path), renderer.py:305-334,
 *                  kernels.py:1219-1418 ---------------- */

static pt_v3 trace_ray_wf(const or_scene *sc, const or_frame *fr, pt_v3 ro, pt_v3 rd, rng_t *r, or_stats *st) {
    /* One path's sequence of queue slots over the host bounce loop. Paths do
     * not interact, so following one path through its waves is equivalent to
     * the queue formulation; per-pixel contributions are added in wave order. */
    pt_v3 acc = pt_v3f(0.0f, 0.0f, 0.0f);
    int have = 0;
    pt_v3 o = ro, d = rd;                                      /* Q1: unnormalized */
    pt_v3 thr = pt_v3f(1.0f, 1.0f, 1.0f);
    int depth = 0;
    pt_v3 bg = pt_v3f(fr->bg[0], fr->bg[1], fr->bg[2]);
    for (int wave = 0; wave < fr->max_depth; ++wave) {       /* renderer.py:313 */
        hit_t h;
        if (st) st->segments++;
        int hit = traverse(sc, fr->traversal, o, d, 0.001f, 1e10f, &h);  /* intersect_rays :1242 */
        if (!hit) {                                           /* shade_miss_rays :1266 */
            acc = pt_add(acc, pt_mul(thr, bg));
            have = 1;
            break;
        }
        int pt = h.type, pi = h.idx;                          /* shade_and_scatter :1289 */
        int is_med = sc->is_medium[pt][pi];
        int scattered = 0;
        pt_v3 sdir = pt_v3f(0.0f, 0.0f, 0.0f), att = pt_v3f(1.0f, 1.0f, 1.0f), emit = pt_v3f(0.0f, 0.0f, 0.0f);
        pt_v3 hp = h.p;
        if (is_med > 0) {
            medium_t m = apply_constant_medium(sc, fr->traversal, pt, pi, o, d, 0.001f, 1e10f, h.t, r, st);
            if (m.is_hit) {
                hp = m.p;
                sdir = random_unit_vector(r);
                att = ld3(sc->med_albedo[pt], pi);
                scattered = 1;
            } else if (m.t_exit > 0.0f) {
                float eps_t = 0.001f / sqrtf(pt_dot(d, d));
                o = pt_add(o, pt_scale(d, m.t_exit + eps_t));
                if (wave + 1 >= fr->max_depth && st) st->depth_cap++;  /* Q14 */
                continue;                                     /* same depth, next wave */
            } else {
                emit = emitted(sc, pt, pi);
                scattered = scatter(sc, d, hp, h.n, pt, pi, &sdir, &att, r);
            }
        } else {
            emit = emitted(sc, pt, pi);
            scattered = scatter(sc, d, hp, h.n, pt, pi, &sdir, &att, r);
        }
        if (emit.x > 0.0f || emit.y > 0.0f || emit.z > 0.0f) {
            acc = pt_add(acc, pt_mul(thr, emit));
            have = 1;
        }
        if (!scattered) break;
        pt_v3 nthr = pt_mul(thr, att);
        int ndepth = depth + 1;
        if (ndepth >= fr->max_depth) {
            if (st) st->depth_cap++;
            break;
        }
        if (ndepth >= 5) {
            float sp = pt_minf(pt_maxf(pt_maxf(nthr.x, nthr.y), nthr.z), 0.95f);
            if (draw(r) > sp) {
                if (st) st->rr++;
                break;
            }
            nthr = pt_divs(nthr, sp);
        }
        o = hp; d = sdir; thr = nthr; depth = ndepth;
        if (wave + 1 >= fr->max_depth && st) st->depth_cap++;  /* Q14: no wave left */
    }
    (void)have;
    return acc;
}

static pt_v3 trace_path(const or_scene *sc, const or_frame *fr, int variant, int px, int py, int s, or_stats *st) {
    rng_t r;
    r.key = pt_path_key(fr->seed, (uint32_t)(py * fr->width + px), (uint32_t)s);
    r.n = 0;
    pt_v3 o, d;
    get_ray(fr, px, py, &r, &o, &d);
    if (st) st->paths++;
    return variant == 0 ? trace_ray_mk(sc, fr, o, d, &r, st) : trace_ray_wf(sc, fr, o, d, &r, st);
}

int or_version(void) { return 1; }

int or_render(const or_scene *sc, const or_frame *fr, int variant, float *accum,
              int x0, int y0, int w, int h, int s_begin, int s_count, int threads, or_stats *stats) {
    if (!sc || !fr || !accum || w <= 0 || (fr->traversal == OR_TRAV_STACKLESS && !sc->bvh_parent && sc->num_bvh_nodes) || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > fr->width || y0 + h > fr->height)
        return -1;
    /* num_bvh_nodes == 0 (empty world, sah_bvh_builder.py:345-355) is legal: the root pop is
       skipped as an invalid node (kernels.py:660) and every path misses */
    uint64_t seg = 0, med = 0, paths = 0, rr = 0, cap = 0;
    long npix = (long)w * (long)h;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 8) reduction(+ : seg, med, paths, rr, cap)
#endif
    for (long q = 0; q < npix; ++q) {
        int px = x0 + (int)(q % w), py = y0 + (int)(q / w);
        or_stats st = {0, 0, 0, 0, 0};
        float *a = accum + 3 * ((size_t)py * (size_t)fr->width + (size_t)px);
        for (int s = s_begin; s < s_begin + s_count; ++s) {
            pt_v3 c = trace_path(sc, fr, variant, px, py, s, &st);
            a[0] += c.x; a[1] += c.y; a[2] += c.z;          /* render_sample :1187 */
        }
        seg += st.segments; med += st.medium; paths += st.paths; rr += st.rr; cap += st.depth_cap;
    }
    if (stats) {
        stats->segments += seg; stats->medium += med; stats->paths += paths;
        stats->rr += rr; stats->depth_cap += cap;
    }
    return 0;
}

int or_traverse(const or_scene *sc, int traversal, const float *o, const float *d, float tmin, float tmax,
                float *t_out, int32_t *type_out, int32_t *idx_out) {
    hit_t h;
    int hit = traverse(sc, traversal, pt_v3f(o[0], o[1], o[2]), pt_v3f(d[0], d[1], d[2]), tmin, tmax, &h);
    *t_out = h.t; *type_out = hit ? h.type : -1; *idx_out = hit ? h.idx : -1;
    return hit;
}

int or_trace_path(const or_scene *sc, const or_frame *fr, int variant, int px, int py, int sample,
                  float *color_out, or_stats *stats) {
    pt_v3 c = trace_path(sc, fr, variant, px, py, sample, stats);
    color_out[0] = c.x; color_out[1] = c.y; color_out[2] = c.z;
    return 0;
}

void or_math_probe(int fn, const float *x, const float *y, float *out, int n) {
    for (int i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = pt_sinf(x[i]); break;
        case 1: out[i] = pt_cosf(x[i]); break;
        case 2: out[i] = pt_logf(x[i]); break;
        case 3: out[i] = pt_acosf(x[i]); break;
        case 4: out[i] = pt_atan2f(x[i], y[i]); break;
        case 5: out[i] = pt_pow5f(x[i]); break;
        case 6: out[i] = pt_div_by(x[i], y[i], pt_recip_for_div(y[i])); break;  /* test of the HIP-side helper */
        default: out[i] = 0.0f;
        }
    }
}

void or_rng_probe(uint32_t seed, uint32_t pixel, uint32_t sample, int n, float *out, uint32_t *key_out) {
    uint32_t key = pt_path_key(seed, pixel, sample);
    if (key_out) *key_out = key;
    for (int i = 0; i < n; ++i) out[i] = pt_rand(key, (uint32_t)i);
}

int or_func_probe(const or_scene *sc, int fn, const float *in, float *out, int n) {
    static const int in_len[9] = {3, 4, 6, 6, 7, 2, 12, 24, 20};
    static const int out_len[9] = {1, 1, 2, 3, 3, 1, 2, 2, 2};
    if (fn < 0 || fn > 8) return 0;
    for (int i = 0; i < n; ++i) {
        const float *x = in + (size_t)i * in_len[fn];
        float *y = out + (size_t)i * out_len[fn];
        pt_v3 a = pt_v3f(x[0], x[1], x[2]);
        switch (fn) {
        case 0: y[0] = perlin_noise(sc, a); break;
        case 1: y[0] = perlin_turb(sc, a, (int)x[3]); break;
        case 2: get_sphere_uv(a, pt_v3f(x[3], x[4], x[5]), &y[0], &y[1]); break;
        case 3: { pt_v3 r = reflect(a, pt_v3f(x[3], x[4], x[5])); y[0] = r.x; y[1] = r.y; y[2] = r.z; } break;
        case 4: { pt_v3 r = refract(a, pt_v3f(x[3], x[4], x[5]), x[6]); y[0] = r.x; y[1] = r.y; y[2] = r.z; } break;
        case 5: y[0] = reflectance(x[0], x[1]); break;
        default: {   /* one primitive in a scratch scene */
            or_scene one = *sc;
            hit_t h; int hit = 0;
            const float *r = x + in_len[fn] - 8;   /* o[3], d[3], tmin, tmax */
            pt_v3 o = pt_v3f(r[0], r[1], r[2]), d = pt_v3f(r[3], r[4], r[5]);
            if (fn == 6) {
                one.sphere_data = x;
                hit = hit_sphere(&one, 0, o, d, r[6], r[7], &h);
            } else if (fn == 7) {
                one.quad_Q = x; one.quad_u = x + 3; one.quad_v = x + 6; one.quad_normal = x + 9;
                one.quad_D = x + 12; one.quad_w = x + 13;
                hit = hit_quad(&one, 0, o, d, r[6], r[7], &h);
            } else {
                one.tri_v0 = x; one.tri_e1 = x + 3; one.tri_e2 = x + 6; one.tri_normal = x + 9;
                hit = hit_triangle(&one, 0, o, d, r[6], r[7], &h);
            }
            y[0] = (float)hit;
            y[1] = hit ? h.t : 0.0f;
        }
        }
    }
    return in_len[fn];
}
