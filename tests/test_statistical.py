"""Statistical pin of the oracle against the reference's own integrator.

tests/golden/stat_<scene>.npz hold per-pixel means and variances of the
reference's pure-Python path tracer (core/camera.py ray_color, 4096 spp) on five
scenes (tests/golden/gen_statistical.py, which documents each): all-Lambertian
spheres under a sky; glass / mirror / Lambertian spheres lit by an emissive
sphere; an open box of Lambertian quads lit by a quad light with a checker-
and an image-textured sphere through a defocus camera; the same box around a
Lambertian octahedron and a mirror tetrahedron (triangles); and an isolated
constant-medium sphere (first free-flight segment: density, exit search,
transmittance). The same scene built
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
from ptmi.core import (Sphere, camera, checker_texture, color, constant_medium, dielectric, diffuse_light,
                       hittable_list, image_texture, lambertian, metal, point3, quad, triangle, vec3)
from ptmi.scenes import _wrap

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _material(spec):
    kind, p = spec[0], spec[1:]
    if kind == 'lambertian':
        return lambertian.from_color(color(*p[0]))
    if kind == 'checker':
        return lambertian.from_texture(checker_texture.from_colors(p[0], color(*p[1]), color(*p[2])))
    if kind == 'image':
        return lambertian.from_texture(image_texture(p[0]))
    if kind == 'diffuse_light':
        return diffuse_light.from_color(color(*p[0]))
    if kind == 'dielectric':
        return dielectric(p[0])
    if kind == 'metal':
        return metal(color(*p[0]), 0.0)
    raise ValueError(kind)


def _scene(name):
    with open(os.path.join(HERE, f'stat_{name}.json')) as f:
        sc = json.load(f)
    w = hittable_list()
    for c, r, spec in sc.get('spheres', []):
        w.add(Sphere.stationary(point3(*c), r, _material(spec)))
    for q, u, v, spec in sc.get('quads', []):
        w.add(quad(point3(*q), vec3(*u), vec3(*v), _material(spec)))
    for v0, v1, v2, spec in sc.get('triangles', []):
        w.add(triangle(point3(*v0), point3(*v1), point3(*v2), _material(spec)))
    for c, r, density, albedo in sc.get('media', []):
        boundary = Sphere.stationary(point3(*c), r, lambertian.from_color(color(0.5, 0.5, 0.5)))
        w.add(constant_medium.from_color(boundary, color(*albedo), density))
    world = _wrap(w.objects)
    cam = camera()
    cam.defocus_angle = sc.get('defocus_angle', 0.0)
    cam.focus_distance = sc.get('focus_distance', 10.0)
    cam.aspect_ratio = sc['aspect']
    cam.img_width = sc['width']
    cam.vfov = sc['vfov']
    cam.lookfrom = point3(*sc['lookfrom'])
    cam.lookat = point3(*sc['lookat'])
    cam.vup = vec3(*sc['vup'])
    cam.initialize()
    return sc, world, cam


SCENES = ['lambert', 'materials', 'quads', 'mesh', 'medium']


def oracle_stats(name, perturb=None):
    """Per-pixel mean / per-sample variance of the oracle (16 x 1024 samples)
    and the reference golden. perturb(SceneArrays) edits the compiled scene
    (the negative-control tests)."""
    sc, world, cam = _scene(name)
    ref = np.load(os.path.join(HERE, f'stat_{name}.npz'))
    sa = sd.compile_world(world)
    if perturb is not None:
        perturb(sa)
    cu = sd.camera_upload(cam)
    W, H = cu['width'], cu['height']
    osc = oracle.OracleScene(sa)
    fr = oracle.make_frame(cu, tuple(sc['background']), sc.get('kernel_max_depth', sc['max_depth']), 7, W, H)
    batches, per = 16, 1024  # independent sample batches -> the oracle's per-sample variance
    means = []
    for b in range(batches):
        acc = np.zeros((H, W, 3), np.float32)
        oracle.render(osc, fr, 'mk', acc, (0, 0, W, H), b * per, per)
        means.append(acc.astype(np.float64) / per)
    means = np.stack(means)
    return means.mean(axis=0), means.var(axis=0, ddof=1) * per, batches * per, ref


def z_scores(m_or, v_or, n_or, ref):
    m_ref, v_ref, n_ref = ref['mean'], ref['var'], int(ref['n'])
    # pooled per-sample variance (a rare-event pixel can show zero variance in
    # one run), plus a floor for the f32 accumulation error of the constant-sky
    # pixels (1024 f32 additions of the same value per batch)
    vp = np.maximum(v_ref, v_or)
    z = (m_or - m_ref) / np.sqrt(vp / n_ref + vp / n_or + (3e-5 * np.abs(m_ref)) ** 2 + 1e-14)
    noisy = vp > 1e-10  # constant-sky values carry no sampling noise: checked by |z| only
    return z, float(np.mean(z[noisy] ** 2)), int(noisy.sum())


def coherent_bias(z):
    """sum(z) / sqrt(n): ~N(0, 1) when the two agree; a small shift shared by
    many pixels (a 2.5 % albedo or density change) adds up here long before
    it shows in any single pixel or in chi-square."""
    return float(z.sum() / np.sqrt(z.size))


@pytest.mark.parametrize('name', SCENES)
def test_oracle_matches_reference_integrator_in_expectation(name):
    m_or, v_or, n_or, ref = oracle_stats(name)
    m_ref = ref['mean']
    assert m_or.shape == m_ref.shape
    z, chi, nv = z_scores(m_or, v_or, n_or, ref)
    cb = coherent_bias(z)
    print(f'{name}: chi2/dof = {chi:.3f} over {nv} values, max|z| = {np.abs(z).max():.2f}, sum(z)/sqrt(n) = {cb:.2f}, '
          f'image means oracle {m_or.mean((0, 1))} reference {m_ref.mean((0, 1))}')
    assert 0.6 < chi < 1.35  # pooled max(variance) makes chi2 < 1 when the two agree
    assert np.abs(z).max() < 5.5
    assert abs(cb) < 4.5
    assert np.allclose(m_or.mean((0, 1)), m_ref.mean((0, 1)), atol=3e-3)


def _scale_albedo(pt, idx, f):
    def edit(sa):  # a solid texture's colour is the albedo the kernels evaluate (texture_color1)
        for k in ('material_albedo', 'texture_color1'):
            a = sa.mats(pt)[k]
            a[idx] = a[idx] * np.float32(f)
    return edit


def _scale_density(pt, idx, f):
    def edit(sa):
        d = sa.mats(pt)['medium_density']
        d[idx] = d[idx] * np.float32(f)
    return edit


def _perturbations():
    """name -> scene edit the chi-square must reject (2.5 % of one albedo or density)."""
    out = {}
    sc, world, _ = _scene('quads')
    sa = sd.compile_world(world)
    # the back wall: the largest Lambertian quad in view (type 1 = quads)
    emit = sa.mats(sd.PRIM_QUAD)['material_emit_color']
    lam = [i for i in range(sa.num_quads) if not np.any(emit[i])]
    assert len(lam) == 5
    out['quads-wall-albedo'] = ('quads', _scale_albedo(sd.PRIM_QUAD, lam[2], 0.975))  # back wall
    sc, world, _ = _scene('medium')
    sa = sd.compile_world(world)
    med = [i for i in range(sa.num_spheres) if sa.mats(sd.PRIM_SPHERE)['is_constant_medium'][i]]
    assert len(med) == 1
    out['medium-density'] = ('medium', _scale_density(sd.PRIM_SPHERE, med[0], 1.025))
    return out


@pytest.mark.parametrize('case', ['quads-wall-albedo', 'medium-density'])
def test_small_perturbation_is_rejected(case):
    """Negative control: the test has the power to see a 2.5 % change."""
    name, edit = _perturbations()[case]
    m_or, v_or, n_or, ref = oracle_stats(name, edit)
    z, chi, nv = z_scores(m_or, v_or, n_or, ref)
    cb = coherent_bias(z)
    print(f'{case}: chi2/dof = {chi:.3f}, max|z| = {np.abs(z).max():.2f}, sum(z)/sqrt(n) = {cb:.2f}')
    assert chi > 1.35 or np.abs(z).max() >= 5.5 or abs(cb) >= 4.5
