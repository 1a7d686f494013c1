#!/usr/bin/env python3
"""Function-level goldens from the reference's own Python (known-answer vectors).

TEST INFRASTRUCTURE ONLY. Run in the build container (where /root/reference
exists); never at test time and never on the GPU box. It imports the
reference's pure-Python modules read-only (no bytecode written) and saves
data only, to tests/golden/functions.npz:

  * perlin_noise / perlin_turb — core/perlin.py:19-84 (`noise`, `turb`), the
    same algorithm as the kernels' perlin_noise / perlin_turb
    (kernels.py:109-169), evaluated with the Perlin tables of the
    vol2_final_scene fixture (the f32 values the renderer uploads) loaded into
    a reference `perlin` instance. Points include negative coordinates (the
    `& 255` wrap), integer lattice boundaries, and vol2-like hit
    points with the octave scalings 2p, 4p. turb at depth 3 (the kernels'
    noise texture, kernels.py:1013-1015) and 7 (core/texture.py:90).
  * sphere_uv — core/sphere.py:67-76 `get_sphere_uv` on the outward normal
    (kernels.py:79-102 normalises p - center first, Q30).
  * reflect / refract — util/vec3.py:285-292 (kernels.py:766-778).
  * reflectance — core/material.py:90-93 dielectric._reflectance (Schlick,
    kernels.py:781-786).
  * hit_sphere / hit_quad / hit_triangle — core/sphere.py:34-60,
    core/quad.py:34-59, core/triangle.py:54-95 on random rays, hit flag and t
    (kernels.py:208-362). Only robust cases are kept (discriminant,
    barycentric and interval margins well away from 0), since the reference
    evaluates in float64 and the kernels in float32; the reference's open
    `surrounds` interval vs the kernels' closed one (Q17) never matters there.

Inputs are float32 values (the oracle's input records, pt_oracle.h
or_func_probe); the reference evaluates them as float64. Quad normal / D / w
and triangle edges / normal are the reference objects' own float64 values
rounded to float32, which is what compile_scene uploads.
"""
import math
import os
import random
import sys
import types

import numpy as np

REF_SRC = '/root/reference/src'
HERE = os.path.dirname(os.path.abspath(__file__))
f32 = np.float32


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    sys.modules.setdefault('pywavefront', types.ModuleType('pywavefront'))  # core/mesh.py only
    from core.perlin import perlin
    from core.sphere import Sphere
    from core.quad import quad
    from core.triangle import triangle
    from core.material import dielectric, lambertian
    from core.interval import interval
    from core.hittable import hit_record
    from util import Ray, vec3
    from util.vec3 import reflect, refract
    return types.SimpleNamespace(**locals())


def _r32(a):
    return np.asarray(a, np.float64).astype(f32)


def main():
    R = _import_reference()
    rng = np.random.default_rng(20261017)
    out = {}
    V = R.vec3

    def v3(a):
        return V(float(a[0]), float(a[1]), float(a[2]))

    # ---------------- Perlin (core/perlin.py with the fixture tables) ----------------
    fx = np.load(os.path.join(HERE, 'vol2_final_scene.npz'), allow_pickle=False)
    pv = fx['perlin_randvec'].astype(f32)
    random.seed(0)  # the constructor draws tables; they are replaced below
    per = R.perlin()
    per.randvec = [V(float(p[0]), float(p[1]), float(p[2])) for p in pv]
    per.perm_x = [int(x) for x in fx['perlin_perm_x']]
    per.perm_y = [int(x) for x in fx['perlin_perm_y']]
    per.perm_z = [int(x) for x in fx['perlin_perm_z']]
    pts = [rng.uniform(-300, 300, (1500, 3)),
           rng.uniform(-4, 4, (600, 3)),
           np.round(rng.uniform(-50, 50, (300, 3))) + rng.choice([0.0, 1e-6, -1e-6, 0.5], (300, 3)),
           rng.uniform([170, 230, 250], [270, 330, 350], (600, 3)),
           rng.uniform(-1000, 1000, (300, 3))]
    P = _r32(np.concatenate(pts))
    P = np.concatenate([P, P[-900:-300] * f32(2), P[-900:-300] * f32(4)])  # octave scalings, exact in f32
    out['perlin_noise_in'] = P
    out['perlin_noise_out'] = np.array([per.noise(v3(p)) for p in P], np.float64)
    T = P[rng.choice(len(P), 2000, replace=False)]
    depth = np.where(np.arange(len(T)) < 1500, 3, 7).astype(f32)
    out['perlin_turb_in'] = np.concatenate([T, depth[:, None]], axis=1).astype(f32)
    out['perlin_turb_out'] = np.array([per.turb(v3(p), int(d)) for p, d in zip(T, depth)], np.float64)

    # ---------------- sphere UV ----------------
    n = rng.normal(size=(4000, 3))
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    c = rng.uniform(-100, 100, (4000, 3))
    r = rng.uniform(0.5, 50, (4000, 1))
    p = _r32(c + r * n)
    c = _r32(c)
    nn = (p.astype(np.float64) - c) / np.linalg.norm(p.astype(np.float64) - c, axis=1, keepdims=True)
    # away from the poles (acos' slope) and from the atan2 branch cut (u 0 <-> 1)
    keep = (np.abs(nn[:, 1]) < 0.999) & ~((np.abs(nn[:, 2]) < 1e-3) & (nn[:, 0] < 0))
    p, c, nn = p[keep][:2000], c[keep][:2000], nn[keep][:2000]
    out['sphere_uv_in'] = np.concatenate([p, c], axis=1)
    out['sphere_uv_out'] = np.array([R.Sphere.get_sphere_uv(v3(x)) for x in nn], np.float64)

    # ---------------- reflect / refract / reflectance ----------------
    d = rng.normal(size=(1500, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    nrm = rng.normal(size=(1500, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm = np.where((np.sum(d * nrm, axis=1) > 0)[:, None], -nrm, nrm)  # facing the ray, as shading sees it
    d, nrm = _r32(d), _r32(nrm)
    out['reflect_in'] = np.concatenate([d * f32(3), nrm], axis=1)  # reflect is used on unnormalised d too (Q5)
    out['reflect_out'] = np.array([_xyz(R.reflect(v3(a[:3]), v3(a[3:]))) for a in out['reflect_in']])
    eta = _r32(rng.choice([1 / 1.5, 1.5, 1 / 1.33, 1.33, 1 / 2.4, 1.0], 1500))
    ref_in = np.concatenate([d, nrm, eta[:, None]], axis=1)
    # sqrt(|1 - |r_perp|^2|) is ill-conditioned at the critical angle: keep
    # cases whose radicand is away from 0 (either side, the abs is the reference's)
    ct = np.minimum(-np.sum(d.astype(np.float64) * nrm, axis=1), 1.0)
    perp = eta[:, None].astype(np.float64) * (d + ct[:, None] * nrm)
    out['refract_in'] = ref_in[np.abs(1.0 - np.sum(perp * perp, axis=1)) > 1e-2]
    out['refract_out'] = np.array([_xyz(R.refract(v3(a[:3]), v3(a[3:6]), float(a[6]))) for a in out['refract_in']])
    cosv = _r32(np.concatenate([rng.uniform(0, 1, 1400), [0.0, 1.0, 0.5, 1e-3, 0.999]]))
    ir = _r32(rng.choice([1.5, 1 / 1.5, 2.4, 1 / 2.4, 1.33, 1.0], len(cosv)))
    out['reflectance_in'] = np.stack([cosv, ir], axis=1)
    die = R.dielectric(1.5)
    out['reflectance_out'] = np.array([die._reflectance(float(a), float(b)) for a, b in zip(cosv, ir)], np.float64)

    # ---------------- primitive hits ----------------
    mat = R.lambertian.__new__(R.lambertian)
    tmin, tmax = 0.001, 1e10

    def ray_hit(obj, o, dd, t0, t1):
        rec = R.hit_record()
        ok = obj.hit(R.Ray(v3(o), v3(dd)), R.interval.from_floats(float(t0), float(t1)), rec)
        return (1.0, rec.t) if ok else (0.0, 0.0)

    recs, res = [], []
    while len(recs) < 2000:
        cc = rng.uniform(-100, 100, 3)
        rad = rng.uniform(0.5, 60)
        o = rng.uniform(-300, 300, 3)
        aim = cc + rng.normal(size=3) * rad * 0.9 - o
        dd = aim * rng.uniform(0.2, 3.0) / np.linalg.norm(aim)  # unnormalised directions (wavefront, Q1)
        cc, rad, o, dd = _r32(cc), f32(rad), _r32(o), _r32(dd)
        t1 = f32(rng.choice([tmax, 1e10, 50.0, 200.0]))
        oc = cc.astype(np.float64) - o
        a = dd.astype(np.float64) @ dd
        h = dd.astype(np.float64) @ oc
        disc = h * h - a * (oc @ oc - float(rad) ** 2)
        if abs(disc) < 1e-3 * h * h:
            continue
        roots = [(h - math.sqrt(disc)) / a, (h + math.sqrt(disc)) / a] if disc > 0 else []
        if any(abs(x - tmin) < 1e-3 * max(1, abs(x)) or abs(x - t1) < 1e-3 * max(1, abs(x)) for x in roots):
            continue
        sph = R.Sphere.stationary(v3(cc), float(rad), mat)
        recs.append(np.concatenate([cc, [rad], o, dd, [tmin, t1]]))
        res.append(ray_hit(sph, o, dd, tmin, t1))
    out['hit_sphere_in'] = np.array(recs, f32)
    out['hit_sphere_out'] = np.array(res, np.float64)

    recs, res = [], []
    while len(recs) < 2000:
        Q = _r32(rng.uniform(-200, 200, 3))
        u = _r32(rng.normal(size=3) * rng.uniform(1, 100))
        v = _r32(rng.normal(size=3) * rng.uniform(1, 100))
        q = R.quad(v3(Q), v3(u), v3(v), mat)
        o = _r32(rng.uniform(-300, 300, 3))
        tgt = Q.astype(np.float64) + rng.uniform(-0.3, 1.3) * u + rng.uniform(-0.3, 1.3) * v
        dd = _r32((tgt - o) * rng.uniform(0.2, 3.0) / np.linalg.norm(tgt - o))
        nq, D, w = np.array(_xyz(q.normal)), q.D, np.array(_xyz(q.w))
        denom = nq @ dd.astype(np.float64)
        if abs(denom) < 2e-2 * np.linalg.norm(dd):  # grazing: t ill-conditioned in float32
            continue
        t = (D - nq @ o.astype(np.float64)) / denom
        if abs(t - tmin) < 1e-3 * max(1, abs(t)):
            continue
        ip = o + dd.astype(np.float64) * t - Q
        al, be = w @ np.cross(ip, v.astype(np.float64)), w @ np.cross(u.astype(np.float64), ip)
        if min(abs(al), abs(al - 1), abs(be), abs(be - 1)) < 1e-4:
            continue
        recs.append(np.concatenate([Q, u, v, _r32(nq), [f32(D)], _r32(w), o, dd, [tmin, tmax]]))
        res.append(ray_hit(q, o, dd, tmin, tmax))
    out['hit_quad_in'] = np.array(recs, f32)
    out['hit_quad_out'] = np.array(res, np.float64)

    recs, res = [], []
    while len(recs) < 2000:
        v0 = _r32(rng.uniform(-200, 200, 3))
        v1 = _r32(v0 + rng.normal(size=3) * rng.uniform(1, 100))
        v2 = _r32(v0 + rng.normal(size=3) * rng.uniform(1, 100))
        tri = R.triangle(v3(v0), v3(v1), v3(v2), mat)
        e1, e2 = np.array(_xyz(tri.edge1)), np.array(_xyz(tri.edge2))
        o = _r32(rng.uniform(-300, 300, 3))
        b1, b2 = rng.uniform(-0.3, 1.2, 2)
        tgt = v0.astype(np.float64) + b1 * e1 + b2 * e2
        dd = _r32((tgt - o) * rng.uniform(0.2, 3.0) / np.linalg.norm(tgt - o))
        hv = np.cross(dd.astype(np.float64), e2)
        det = e1 @ hv
        if abs(det) < 1e-3 * np.linalg.norm(e1) * np.linalg.norm(hv) or \
                abs(np.array(_xyz(tri.normal)) @ dd) < 2e-2 * np.linalg.norm(dd):  # grazing
            continue
        s = o.astype(np.float64) - v0
        uu = (s @ hv) / det
        qv = np.cross(s, e1)
        vv = (dd.astype(np.float64) @ qv) / det
        t = (e2 @ qv) / det
        if min(abs(uu), abs(uu - 1), abs(vv), abs(uu + vv - 1)) < 1e-4 or abs(t - tmin) < 1e-3 * max(1, abs(t)):
            continue
        recs.append(np.concatenate([v0, _r32(e1), _r32(e2), _r32(_xyz(tri.normal)), o, dd, [tmin, tmax]]))
        res.append(ray_hit(tri, o, dd, tmin, tmax))
    out['hit_triangle_in'] = np.array(recs, f32)
    out['hit_triangle_out'] = np.array(res, np.float64)

    for k in list(out):
        if k.endswith('_in'):
            out[k] = np.ascontiguousarray(out[k], f32)
    out['perlin_tables'] = np.array('vol2_final_scene.npz')
    np.savez_compressed(os.path.join(HERE, 'functions.npz'), **out)
    for k, a in out.items():
        if k.endswith('_out'):
            print(k, a.shape, 'hits' if k.startswith('hit') else '', int(a[:, 0].sum()) if k.startswith('hit') else '')


def _xyz(v):
    return [v.x, v.y, v.z]


if __name__ == '__main__':
    main()
