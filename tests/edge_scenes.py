"""Edge-case scenes for the parity tests (test infrastructure only):

* ``empty``: no primitives at all (every path misses: accum = bg per sample);
* ``single``: one sphere, so the BVH root is itself a leaf (root_ref < 0);
* ``chain<N>``: N small spheres in a row under a hand-built *linear* BVH
  (every internal node has a leaf left child and an internal right child), so
  the deepest leaf sits at depth N-1 and the integrator must dispatch its 17-
  to 20-slot (N = 17..20) or 24-, 32- or 64-slot traversal kernels, most of
  which the BASELINE scenes (leaf depth <= 16) never reach.
* ``chainx<N>``: the same spheres seen along -x from the chain's +x end, with
  the linear BVH's leaves ordered by x, far (-x) end first, and the ground
  sphere deepest. Each internal node's box then projects nearer than its leaf
  child, so the reference's stack (kernels.py:705-732) keeps one far leaf per
  level and, past 64 entries, drops the pushes (kernels.py:719-740): for N > 64
  the deep end of the chain (the near spheres and the ground) is never
  visited. The overflow semantics the integrators must reproduce (leaf depth
  N - 1 > 62). The flattened arrays follow the reference's layout
  (sah_bvh_builder.py:338-418 flatten: preorder, left child at i + 1, node
  box = union of the children's boxes, internal prim_type/prim_idx = -1).
* ``marble``: noise-textured Lambertian spheres at four scales over a
  noise-textured ground, with a solid Lambertian, a metal sphere and a
  light: most shading rounds of the megakernel hold several Perlin hits, so
  the wave-cooperative turbulence (perlin_turb3_wave) runs several passes,
  with odd and even counts.
"""
from __future__ import annotations

import random

import numpy as np

from ptmi import scene_data as sd
from ptmi.core import (Sphere, camera, color, diffuse_light, hittable_list, lambertian, metal, noise_texture,
                       point3, vec3)
from ptmi.scenes import _wrap

BG = (0.6, 0.7, 0.9)


def _camera(width, along_x=False):
    cam = camera()
    cam.aspect_ratio = 16.0 / 9.0
    cam.img_width = width
    cam.vfov = 40
    cam.lookfrom = point3(12, 0.8, 0.5) if along_x else point3(0, 1.5, 8)
    cam.lookat = point3(-4, 0, -1) if along_x else point3(0, 0.2, 0)
    cam.vup = vec3(0, 1, 0)
    cam.initialize()
    return sd.camera_upload(cam)


def _row(n):
    w = hittable_list()
    for k in range(n):
        x = -4.0 + 8.0 * k / max(1, n - 1)
        m = metal(color(0.8, 0.8, 0.7), 0.1) if k % 3 == 0 else lambertian.from_color(color(0.2 + 0.6 * (k % 2), 0.5, 0.3))
        w.add(Sphere.stationary(point3(x, 0.3 * (k % 4), -0.5 * (k % 5)), 0.35, m))
    w.add(Sphere.stationary(point3(0, -100.4, 0), 100.0, lambertian.from_color(color(0.5, 0.5, 0.5))))
    return w


def _linear_bvh(sa, order=None):
    """Reference-layout flattened arrays of a linear BVH over the scene's
    spheres (leaf i = sphere order[i], default sphere i; the last internal
    node holds the last two)."""
    ns = sa.num_spheres
    assert ns >= 2 and sa.num_quads == 0 and sa.num_triangles == 0
    order = np.arange(ns) if order is None else np.asarray(order)
    c = sa.sphere_data[:, :3].astype(np.float32)
    r = sa.sphere_data[:, 3:4].astype(np.float32)
    lo, hi = c - r, c + r  # sphere bbox as the reference computes it (hittable.py: center -/+ radius)
    n = 2 * ns - 1
    bmin = np.zeros((n, 3), np.float32)
    bmax = np.zeros((n, 3), np.float32)
    left = np.full(n, -1, np.int32)
    right = np.full(n, -1, np.int32)
    parent = np.full(n, -1, np.int32)
    ptype = np.full(n, -1, np.int32)
    pidx = np.full(n, -1, np.int32)
    # preorder: internal node for sphere k at 2k, its leaf at 2k + 1; the
    # last sphere is the right leaf of the last internal node
    for k in range(ns - 1):
        node, leaf = 2 * k, 2 * k + 1
        left[node] = leaf
        right[node] = node + 2
        parent[leaf] = node
        parent[node + 2] = node
        ptype[leaf], pidx[leaf] = sd.PRIM_SPHERE, order[k]
        bmin[leaf], bmax[leaf] = lo[order[k]], hi[order[k]]
    last = n - 1
    ptype[last], pidx[last] = sd.PRIM_SPHERE, order[ns - 1]
    bmin[last], bmax[last] = lo[order[ns - 1]], hi[order[ns - 1]]
    for k in range(ns - 2, -1, -1):  # unions bottom-up
        node = 2 * k
        bmin[node] = np.minimum(bmin[left[node]], bmin[right[node]])
        bmax[node] = np.maximum(bmax[left[node]], bmax[right[node]])
    return {'bvh_bbox_min': bmin, 'bvh_bbox_max': bmax, 'bvh_left_child': left, 'bvh_right_child': right,
            'bvh_parent': parent, 'bvh_prim_type': ptype, 'bvh_prim_idx': pidx}


_cache = {}


def edge_scene(name, width=96):
    """(SceneArrays, camera upload dict, background) of an edge-case scene."""
    key = (name, width)
    if key in _cache:
        return _cache[key]
    if name == 'empty':
        sa = sd.compile_world(_wrap(_row(1).objects))
        sa.sphere_data = sa.sphere_data[:0]
        sa.sphere_mats = {k: np.asarray(v)[:0] for k, v in sa.sphere_mats.items()}
        sa.bvh = {k: np.asarray(v)[:0] for k, v in sa.bvh.items()}
    elif name == 'single':
        w = hittable_list()
        w.add(Sphere.stationary(point3(0, 0.3, 0), 1.2, lambertian.from_color(color(0.7, 0.3, 0.2))))
        sa = sd.compile_world(_wrap(w.objects))
    elif name.startswith('chain'):
        n = int(name[6:] if name.startswith('chainx') else name[5:])
        sa = sd.compile_world(_wrap(_row(n - 1).objects))  # + the ground sphere
        order = None
        if name.startswith('chainx'):  # leaves by x ascending (far to near), the ground sphere deepest
            small = sa.sphere_data[:, 3] < 50
            order = np.concatenate([np.flatnonzero(small)[np.argsort(sa.sphere_data[small, 0], kind='stable')],
                                    np.flatnonzero(~small)])
        sa.bvh = _linear_bvh(sa, order)
    elif name == 'marble':
        random.seed(7)
        w = hittable_list()
        w.add(Sphere.stationary(point3(0, -100.4, 0), 100.0, lambertian.from_texture(noise_texture(4.0))))
        for k, (x, scale) in enumerate([(-2.4, 1.0), (-0.8, 3.0), (0.8, 6.0), (2.4, 12.0)]):
            w.add(Sphere.stationary(point3(x, 0.5, -0.3 * k), 0.75, lambertian.from_texture(noise_texture(scale))))
        w.add(Sphere.stationary(point3(0.0, 1.9, -1.0), 0.6, lambertian.from_color(color(0.7, 0.6, 0.2))))
        w.add(Sphere.stationary(point3(-1.5, 1.6, 0.8), 0.4, metal(color(0.8, 0.8, 0.8), 0.2)))
        w.add(Sphere.stationary(point3(1.6, 1.7, 0.5), 0.35, diffuse_light.from_color(color(4.0, 4.0, 4.0))))
        sa = sd.compile_world(_wrap(w.objects))
    else:
        raise KeyError(name)
    _cache[key] = (sa, _camera(width, along_x=name.startswith('chainx')), BG)
    return _cache[key]
