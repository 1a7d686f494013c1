"""TEST INFRASTRUCTURE ONLY — ctypes bridge to the CPU oracle (pt_oracle.c).

The oracle restates src/render_server/taichi_renderer/kernels.py on the
reference's own array layout. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker.
Scene/BVH arrays are pinned to the reference by tests/golden fixtures; pixel
values are pinned to this restatement (Taichi cannot run: parity vs Taichi
pixels is unpinned).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, '_build', 'libptoracle.so')
MAX_IMAGES = 16

P = C.c_void_p
f3 = C.c_float * 3


class OrScene(C.Structure):
    _fields_ = [('num_spheres', C.c_int32), ('num_quads', C.c_int32), ('num_triangles', C.c_int32),
                ('num_bvh_nodes', C.c_int32),
                ('sphere_data', P), ('quad_Q', P), ('quad_u', P), ('quad_v', P), ('quad_normal', P),
                ('quad_D', P), ('quad_w', P), ('tri_v0', P), ('tri_e1', P), ('tri_e2', P), ('tri_normal', P),
                ('mat_type', P * 3), ('albedo', P * 3), ('fuzz', P * 3), ('ir', P * 3), ('emit', P * 3),
                ('tex_type', P * 3), ('tex_scale', P * 3), ('color1', P * 3), ('color2', P * 3),
                ('img_idx', P * 3), ('is_medium', P * 3), ('density', P * 3), ('med_albedo', P * 3),
                ('bvh_min', P), ('bvh_max', P), ('bvh_left', P), ('bvh_right', P), ('bvh_type', P), ('bvh_idx', P),
                ('perlin_vec', P), ('perm_x', P), ('perm_y', P), ('perm_z', P),
                ('num_images', C.c_int32), ('images', P * MAX_IMAGES), ('img_w', C.c_int32 * MAX_IMAGES),
                ('img_h', C.c_int32 * MAX_IMAGES), ('bvh_parent', P)]


class OrFrame(C.Structure):
    _fields_ = [('center', f3), ('pixel00', f3), ('delta_u', f3), ('delta_v', f3), ('defocus_u', f3),
                ('defocus_v', f3), ('defocus_angle', C.c_float), ('bg', f3), ('max_depth', C.c_int32),
                ('seed', C.c_uint32), ('width', C.c_int32), ('height', C.c_int32), ('traversal', C.c_int32)]


class OrStats(C.Structure):
    _fields_ = [('segments', C.c_uint64), ('medium', C.c_uint64), ('paths', C.c_uint64), ('rr', C.c_uint64),
                ('depth_cap', C.c_uint64)]


_lib = None


def build():
    subprocess.run(['make', '-s', '-C', _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = load_variant(LIB)
    return _lib


def load_variant(path):
    """A libptoracle build at `path` (the tests' negative-control builds of
    pt_oracle.c with a switch changed), with the entry points typed."""
    lib = C.CDLL(path)
    lib.or_render.argtypes = [C.POINTER(OrScene), C.POINTER(OrFrame), C.c_int, P, C.c_int, C.c_int, C.c_int,
                              C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(OrStats)]
    lib.or_traverse.argtypes = [C.POINTER(OrScene), C.c_int, P, P, C.c_float, C.c_float, P, P, P]
    lib.or_trace_path.argtypes = [C.POINTER(OrScene), C.POINTER(OrFrame), C.c_int, C.c_int, C.c_int, C.c_int,
                                  P, C.POINTER(OrStats)]
    lib.or_math_probe.argtypes = [C.c_int, P, P, P, C.c_int]
    lib.or_rng_probe.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, P, P]
    lib.or_func_probe.argtypes = [C.POINTER(OrScene), C.c_int, P, P, C.c_int]
    lib.or_func_probe.restype = C.c_int
    return lib


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


class OracleScene:
    """or_scene over a ptmi.scene_data.SceneArrays (reference layout)."""

    def __init__(self, sa):
        self.sa = sa
        keep = []

        def c(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return _ptr(a)

        s = OrScene()
        s.num_spheres, s.num_quads, s.num_triangles = sa.num_spheres, sa.num_quads, sa.num_triangles
        s.num_bvh_nodes = sa.num_bvh_nodes
        f32, i32 = np.float32, np.int32
        s.sphere_data = c(sa.sphere_data, f32)
        q = sa.quads
        s.quad_Q, s.quad_u, s.quad_v = c(q['quad_Q'], f32), c(q['quad_u'], f32), c(q['quad_v'], f32)
        s.quad_normal, s.quad_D, s.quad_w = c(q['quad_normal'], f32), c(q['quad_D'], f32), c(q['quad_w'], f32)
        t = sa.tris
        s.tri_v0, s.tri_e1 = c(t['triangle_v0'], f32), c(t['triangle_edge1'], f32)
        s.tri_e2, s.tri_normal = c(t['triangle_edge2'], f32), c(t['triangle_normal'], f32)
        for pt in range(3):
            m = sa.mats(pt)
            s.mat_type[pt] = c(m['material_type'], i32)
            s.albedo[pt] = c(m['material_albedo'], f32)
            s.fuzz[pt] = c(m['material_fuzz'], f32)
            s.ir[pt] = c(m['material_ir'], f32)
            s.emit[pt] = c(m['material_emit_color'], f32)
            s.tex_type[pt] = c(m['texture_type'], i32)
            s.tex_scale[pt] = c(m['texture_scale'], f32)
            s.color1[pt] = c(m['texture_color1'], f32)
            s.color2[pt] = c(m['texture_color2'], f32)
            s.img_idx[pt] = c(m['texture_image_idx'], i32)
            s.is_medium[pt] = c(m['is_constant_medium'], i32)
            s.density[pt] = c(m['medium_density'], f32)
            s.med_albedo[pt] = c(m['medium_albedo'], f32)
        b = sa.bvh
        s.bvh_min, s.bvh_max = c(b['bvh_bbox_min'], f32), c(b['bvh_bbox_max'], f32)
        s.bvh_left, s.bvh_right = c(b['bvh_left_child'], i32), c(b['bvh_right_child'], i32)
        s.bvh_type, s.bvh_idx = c(b['bvh_prim_type'], i32), c(b['bvh_prim_idx'], i32)
        s.bvh_parent = c(b['bvh_parent'], i32)
        p = sa.perlin
        s.perlin_vec = c(p['perlin_randvec'], f32)
        s.perm_x, s.perm_y, s.perm_z = c(p['perlin_perm_x'], i32), c(p['perlin_perm_y'], i32), c(p['perlin_perm_z'], i32)
        s.num_images = len(sa.images)
        for k, im in enumerate(sa.images):
            s.images[k] = c(im, np.uint8)
            s.img_h[k], s.img_w[k] = im.shape[0], im.shape[1]
        self.s = s
        self._keep = keep


TRAVERSALS = {'stack': 0, 'stackless': 1}  # traverse_bvh_legacy / traverse_bvh_stackless (kernels.py:746)


def make_frame(cam, bg, max_depth, seed, width, height, traversal='stack'):
    f = OrFrame()
    f.traversal = TRAVERSALS[traversal]
    for k in ('center', 'pixel00', 'delta_u', 'delta_v', 'defocus_u', 'defocus_v'):
        v = np.asarray(cam[k], np.float32)
        for i in range(3):
            getattr(f, k)[i] = float(v[i])
    f.defocus_angle = float(np.float32(cam['defocus_angle']))
    bgv = np.asarray(bg, np.float32)
    for i in range(3):
        f.bg[i] = float(bgv[i])
    f.max_depth, f.seed, f.width, f.height = int(max_depth), int(seed) & 0xffffffff, int(width), int(height)
    return f


def render(oscene, frame, variant, accum, window, s_begin, s_count, threads=0, lib=None):
    """variant: 'mk' | 'wf'. accum (H, W, 3) f32 numpy, updated in place.
    lib: a load_variant() build instead of the oracle."""
    assert accum.dtype == np.float32 and accum.flags['C_CONTIGUOUS']
    assert accum.shape == (frame.height, frame.width, 3)
    x0, y0, w, h = window
    st = OrStats()
    rc = (lib or load()).or_render(C.byref(oscene.s), C.byref(frame), 0 if variant == 'mk' else 1, _ptr(accum),
                          x0, y0, w, h, s_begin, s_count, threads, C.byref(st))
    if rc != 0:
        raise RuntimeError(f'or_render failed: {rc}')
    return {'segments': st.segments, 'medium': st.medium, 'paths': st.paths, 'rr': st.rr,
            'depth_cap': st.depth_cap}


def traverse(oscene, o, d, tmin=0.001, tmax=1e10, traversal='stack'):
    o = np.asarray(o, np.float32)
    d = np.asarray(d, np.float32)
    t = np.zeros(1, np.float32)
    ty = np.zeros(1, np.int32)
    ix = np.zeros(1, np.int32)
    hit = load().or_traverse(C.byref(oscene.s), TRAVERSALS[traversal], _ptr(o), _ptr(d), tmin, tmax, _ptr(t), _ptr(ty), _ptr(ix))
    return bool(hit), float(t[0]), int(ty[0]), int(ix[0])


MATH_FNS = {'sin': 0, 'cos': 1, 'log': 2, 'acos': 3, 'atan2': 4, 'pow5': 5, 'div_by': 6}


def math_probe(fn, x, y=None):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), np.float32)
    out = np.zeros_like(x)
    load().or_math_probe(MATH_FNS[fn], _ptr(x), _ptr(y), _ptr(out), x.size)
    return out


def rng_probe(seed, pixel, sample, n):
    out = np.zeros(n, np.float32)
    key = np.zeros(1, np.uint32)
    load().or_rng_probe(seed, pixel, sample, n, _ptr(out), _ptr(key))
    return out, int(key[0])


# or_func_probe: function -> (id, input record length, output record length)
FUNCS = {'perlin_noise': (0, 3, 1), 'perlin_turb': (1, 4, 1), 'sphere_uv': (2, 6, 2), 'reflect': (3, 6, 3),
         'refract': (4, 7, 3), 'reflectance': (5, 2, 1), 'hit_sphere': (6, 12, 2), 'hit_quad': (7, 24, 2),
         'hit_triangle': (8, 20, 2)}


def func_probe(oscene, fn, records):
    """One kernels.py function of the oracle on (n, in_len) f32 input records
    (layouts in pt_oracle.h, or_func_probe); the Perlin functions use
    oscene's tables. Returns (n, out_len) f32."""
    fid, n_in, n_out = FUNCS[fn]
    x = np.ascontiguousarray(records, np.float32).reshape(-1, n_in)
    out = np.zeros((x.shape[0], n_out), np.float32)
    got = load().or_func_probe(C.byref(oscene.s), fid, _ptr(x), _ptr(out), x.shape[0])
    if got != n_in:
        raise RuntimeError(f'or_func_probe({fn}) expects {got} inputs per record')
    return out
