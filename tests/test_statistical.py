"""Statistical pin of the oracle against the reference's own integrator.

tests/golden/stat_<scene>.npz hold per-pixel means and variances of the
reference's pure-Python path tracer (core/camera.py ray_color, 4096 spp) on two
sphere scenes (tests/golden/gen_statistical.py): all-Lambertian under a sky,
and glass / mirror / Lambertian spheres lit by an emissive sphere. The same scene built
from ptmi.core, compiled (compile_scene + native SAH) and rendered by the C
oracle — which the GPU matches bit for bit (tests/test_gpu_parity.py) — must
have the same per-pixel expectation: the Taichi-kernel semantics the oracle
restates differ from the Python integrator only in expectation-preserving ways
(RR, Q4 basis, Q28 extra dielectric draw, RNG) or negligibly (the Q13 depth
cap). Metal is used with fuzz 0: with fuzz the two integrators differ (the
kernels normalise the incoming direction before adding fuzz and absorb
below-surface reflections, Q5; core/material.py does neither).

Test: z = (m_oracle - m_ref) / sqrt(se_oracle^2 + se_ref^2) over 32x18x3
values (pooled per-sample variance, 16384 oracle samples); the mean of z^2 must
be ~1 (chi-square / dof) and no |z| may be extreme. A wrong BRDF, normal,
camera mapping or sky term shifts whole regions
by many standard errors.
"""
import json
import os

import numpy as np
import pytest

import oracle
from ptmi import scene_data as sd
from ptmi.core import (Sphere, camera, color, dielectric, diffuse_light, hittable_list, lambertian, metal, point3,
                       vec3)
from ptmi.scenes import _wrap

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _scene(name):
    with open(os.path.join(HERE, f'stat_{name}.json')) as f:
        sc = json.load(f)
    w = hittable_list()
    for c, r, (kind, p) in sc['spheres']:
        mat = {'lambertian': lambda: lambertian.from_color(color(*p)),
               'diffuse_light': lambda: diffuse_light.from_color(color(*p)),
               'dielectric': lambda: dielectric(p), 'metal': lambda: metal(color(*p), 0.0)}[kind]()
        w.add(Sphere.stationary(point3(*c), r, mat))
    world = _wrap(w.objects)
    cam = camera()
    cam.aspect_ratio = sc['aspect']
    cam.img_width = sc['width']
    cam.vfov = sc['vfov']
    cam.lookfrom = point3(*sc['lookfrom'])
    cam.lookat = point3(*sc['lookat'])
    cam.vup = vec3(*sc['vup'])
    cam.initialize()
    return sc, world, cam


@pytest.mark.parametrize('name', ['lambert', 'materials'])
def test_oracle_matches_reference_integrator_in_expectation(name):
    sc, world, cam = _scene(name)
    ref = np.load(os.path.join(HERE, f'stat_{name}.npz'))
    m_ref, v_ref, n_ref = ref['mean'], ref['var'], int(ref['n'])
    sa = sd.compile_world(world)
    cu = sd.camera_upload(cam)
    W, H = cu['width'], cu['height']
    assert (H, W, 3) == m_ref.shape
    osc = oracle.OracleScene(sa)
    fr = oracle.make_frame(cu, tuple(sc['background']), sc['max_depth'], 7, W, H)
    batches, per = 16, 1024  # independent sample batches -> the oracle's per-sample variance
    means = []
    for b in range(batches):
        acc = np.zeros((H, W, 3), np.float32)
        oracle.render(osc, fr, 'mk', acc, (0, 0, W, H), b * per, per)
        means.append(acc.astype(np.float64) / per)
    means = np.stack(means)
    n_or = batches * per
    m_or = means.mean(axis=0)
    v_or = means.var(axis=0, ddof=1) * per
    # pooled per-sample variance (a rare-event pixel can show zero variance in
    # one run), plus a floor for the f32 accumulation error of the constant-sky
    # pixels (1024 f32 additions of the same value per batch)
    vp = np.maximum(v_ref, v_or)
    z = (m_or - m_ref) / np.sqrt(vp / n_ref + vp / n_or + (3e-5 * np.abs(m_ref)) ** 2 + 1e-14)
    noisy = vp > 1e-10  # constant-sky values carry no sampling noise: checked by |z| only
    chi = float(np.mean(z[noisy] ** 2))
    print(f'chi2/dof = {chi:.3f} over {int(noisy.sum())} values, max|z| = {np.abs(z).max():.2f}, image means oracle {m_or.mean((0, 1))} '
          f'reference {m_ref.mean((0, 1))}')
    assert 0.6 < chi < 1.35  # pooled max(variance) makes chi2 < 1 when the two agree
    assert np.abs(z).max() < 5.5
    assert np.allclose(m_or.mean((0, 1)), m_ref.mean((0, 1)), atol=3e-3)
