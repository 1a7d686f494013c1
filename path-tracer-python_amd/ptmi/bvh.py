"""BVH compile surface (reference: src/render_server/taichi_renderer/bvh_compiler.py).

``build_sah`` runs the native binned-SAH builder of libptmi
(csrc/pt_bvh_build.cpp, bit-exact with sah_bvh_builder.py under NumPy >= 2)
and returns the reference's 7 flattened arrays + ``num_bvh_nodes``.
``compile_bvh(world, spheres, quads, triangles)`` keeps the reference's
signature (bvh_compiler.py:132) and takes the primitive lists that
``compile_scene`` returned.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


def _f32(a, cols):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1, cols))
    return a


def build_sah(spheres=None, quads=None, tris=None):
    """spheres (N,4) {c.xyz, r}; quads (N,9) {Q,u,v}; tris (N,9) {v0,v1,v2}; all cast to f32."""
    sp = _f32(spheres if spheres is not None else np.zeros((0, 4)), 4)
    qd = _f32(quads if quads is not None else np.zeros((0, 9)), 9)
    tr = _f32(tris if tris is not None else np.zeros((0, 9)), 9)
    n_prims = sp.shape[0] + qd.shape[0] + tr.shape[0]
    cap = max(1, 2 * n_prims - 1)
    out = {
        'bvh_bbox_min': np.zeros((cap, 3), np.float32), 'bvh_bbox_max': np.zeros((cap, 3), np.float32),
        'bvh_left_child': np.full(cap, -1, np.int32), 'bvh_right_child': np.full(cap, -1, np.int32),
        'bvh_parent': np.full(cap, -1, np.int32), 'bvh_prim_type': np.zeros(cap, np.int32),
        'bvh_prim_idx': np.full(cap, -1, np.int32),
    }
    n = C.c_int32(0)

    def p(a):
        return C.c_void_p(a.ctypes.data) if a.size else None

    lib = _lib.load()
    _lib.check(lib.ptmi_bvh_build_sah(p(sp), sp.shape[0], p(qd), qd.shape[0], p(tr), tr.shape[0],
                                      p(out['bvh_bbox_min']), p(out['bvh_bbox_max']), p(out['bvh_left_child']),
                                      p(out['bvh_right_child']), p(out['bvh_parent']), p(out['bvh_prim_type']),
                                      p(out['bvh_prim_idx']), C.byref(n)), 'ptmi_bvh_build_sah')
    k = n.value
    res = {key: v[:k].copy() for key, v in out.items()}
    if k == 0:  # sah_bvh_builder.py:345-355 empty flatten
        res = {'bvh_bbox_min': np.zeros((0, 3), np.float32), 'bvh_bbox_max': np.zeros((0, 3), np.float32),
               'bvh_left_child': np.array([], np.int32), 'bvh_right_child': np.array([], np.int32),
               'bvh_parent': np.array([], np.int32), 'bvh_prim_type': np.array([], np.int32),
               'bvh_prim_idx': np.array([], np.int32)}
    res['num_bvh_nodes'] = k
    return res


def _center0(sphere):
    c = sphere.center.at(0.0)  # moving spheres use the t=0 centre (sah_bvh_builder.py:434, 463)
    return c


def primitive_inputs(spheres, quads, triangles):
    """f32 builder inputs from primitive objects, as sah_bvh_builder.py:462-479 forms them."""
    sp = np.zeros((len(spheres), 4), np.float32)
    for i, s in enumerate(spheres):
        c = _center0(s)
        sp[i, :3] = np.array([c.x, c.y, c.z], np.float32)
        sp[i, 3] = np.float32(s.radius)
    qd = np.zeros((len(quads), 9), np.float32)
    for i, q in enumerate(quads):
        qd[i] = np.array([q.Q.x, q.Q.y, q.Q.z, q.u.x, q.u.y, q.u.z, q.v.x, q.v.y, q.v.z], np.float64).astype(np.float32)
    tr = np.zeros((len(triangles), 9), np.float32)
    for i, t in enumerate(triangles):
        tr[i] = np.array([t.v0.x, t.v0.y, t.v0.z, t.v1.x, t.v1.y, t.v1.z, t.v2.x, t.v2.y, t.v2.z],
                         np.float64).astype(np.float32)
    return sp, qd, tr


def compile_bvh(world, spheres, quads=None, triangles=None):
    """bvh_compiler.compile_bvh (bvh_compiler.py:132-168); SAH path (USE_SAH_BVH = True)."""
    quads = quads or []
    triangles = triangles or []
    sp, qd, tr = primitive_inputs(spheres, quads, triangles)
    return build_sah(sp, qd, tr)
