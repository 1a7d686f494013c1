#!/usr/bin/env python3
"""Statistical golden: the reference's own path tracer on a Lambertian scene.

TEST INFRASTRUCTURE ONLY (run in the build container, where /root/reference
exists; never at test time, never on the GPU box). It imports the reference's
pure-Python integrator read-only — core/camera.py `get_ray` + `ray_color`
(camera.py:74-137), core/material.py lambertian, util/vec3.py
random_cosine_direction — renders a small all-Lambertian scene (spheres over a
ground sphere, constant sky) and saves the per-pixel mean and variance of the
sample colours (float64) to stat_lambert.npz, plus the scene in
stat_lambert.json. SURVEY.md §8c item (6).

Why this pins the oracle: for Lambertian spheres seen from outside under a
constant sky, the Taichi kernels' semantics (kernels.py) and the Python
integrator differ only in ways that keep the expectation: RR (both unbiased;
disabled here on the Python side), the cosine-sampling basis (Q4, same
distribution), the depth cap (Q13; albedo <= 0.8 makes bounces beyond 49
negligible) and the RNG. tests/test_statistical.py compares the oracle's
per-pixel means against these, within the standard errors of both.
"""
import json
import multiprocessing as mp
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SCENES = {
    # all-Lambertian spheres under a constant sky
    'lambert': {
        'width': 32, 'aspect': 16.0 / 9.0, 'vfov': 30.0, 'lookfrom': [0.0, 0.6, 3.0], 'lookat': [0.0, 0.1, -1.0],
        'vup': [0.0, 1.0, 0.0], 'background': [0.7, 0.8, 1.0], 'max_depth': 50,
        'spheres': [  # center, radius, material
            [[0.0, -100.5, -1.0], 100.0, ['lambertian', [0.8, 0.8, 0.0]]],
            [[0.0, 0.0, -1.2], 0.5, ['lambertian', [0.1, 0.2, 0.5]]],
            [[-1.0, 0.0, -1.0], 0.5, ['lambertian', [0.8, 0.6, 0.2]]],
            [[1.0, -0.1, -0.9], 0.4, ['lambertian', [0.7, 0.7, 0.7]]],
            [[0.35, -0.35, -0.45], 0.15, ['lambertian', [0.2, 0.8, 0.3]]],
        ],
    },
    # glass, mirror (fuzz 0) and Lambertian spheres lit by an emissive sphere, black background
    'materials': {
        'width': 32, 'aspect': 16.0 / 9.0, 'vfov': 34.0, 'lookfrom': [0.0, 0.7, 3.0], 'lookat': [0.0, 0.2, -1.0],
        'vup': [0.0, 1.0, 0.0], 'background': [0.0, 0.0, 0.0], 'max_depth': 50,
        'spheres': [
            [[0.0, -100.5, -1.0], 100.0, ['lambertian', [0.6, 0.6, 0.6]]],
            [[0.0, 2.0, -1.2], 1.0, ['diffuse_light', [3.0, 3.0, 3.0]]],
            [[-1.05, 0.0, -1.0], 0.5, ['dielectric', 1.5]],
            [[1.05, 0.0, -1.0], 0.5, ['metal', [0.8, 0.6, 0.2]]],
            [[0.0, -0.05, -1.4], 0.45, ['lambertian', [0.2, 0.3, 0.7]]],
        ],
    },
}
SPP = 4096
NAME = 'lambert'


def _build():
    from gen_fixtures import _install_stubs
    _install_stubs()
    from core import Sphere, hittable_list, camera  # noqa: E402
    from core.material import dielectric, diffuse_light, lambertian, metal  # noqa: E402
    from util import color, point3, vec3  # noqa: E402
    SCENE = SCENES[NAME]
    world = hittable_list()
    for c, r, (kind, p) in SCENE['spheres']:
        mat = {'lambertian': lambda: lambertian.from_color(color(*p)),
               'diffuse_light': lambda: diffuse_light.from_color(color(*p)),
               'dielectric': lambda: dielectric(p), 'metal': lambda: metal(color(*p), 0.0)}[kind]()
        world.add(Sphere.stationary(point3(*c), r, mat))
    cam = camera()
    cam.aspect_ratio = SCENE['aspect']
    cam.img_width = SCENE['width']
    cam.samples_per_pixel = SPP
    cam.vfov = SCENE['vfov']
    cam.lookfrom = point3(*SCENE['lookfrom'])
    cam.lookat = point3(*SCENE['lookat'])
    cam.vup = vec3(*SCENE['vup'])
    cam.initialize()
    cam.max_depth = SCENE['max_depth']
    cam.background = color(*SCENE['background'])
    cam.russian_roulette_enabled = False
    return world, cam


def _rows(args):
    rows, = args
    world, cam = _build()
    out = []
    for j in rows:
        random.seed(1000 + j)
        line = []
        for i in range(cam.img_width):
            s = np.zeros(3)
            s2 = np.zeros(3)
            for _ in range(SPP):
                c = cam.ray_color(cam.get_ray(i, j), cam.max_depth, world)
                v = np.array([c.x, c.y, c.z])
                s += v
                s2 += v * v
            line.append((s, s2))
        out.append((j, line))
    return out


def main():
    global NAME
    for NAME in SCENES:
        render_one()


def render_one():
    SCENE = SCENES[NAME]
    _, cam = _build()
    W, H = cam.img_width, cam.img_height
    chunks = [list(range(j, H, 8)) for j in range(8)]
    with mp.get_context('fork').Pool(8) as pool:
        parts = pool.map(_rows, [(c,) for c in chunks])
    mean = np.zeros((H, W, 3))
    var = np.zeros((H, W, 3))
    for part in parts:
        for j, line in part:
            for i, (s, s2) in enumerate(line):
                m = s / SPP
                mean[j, i] = m
                var[j, i] = np.maximum(s2 / SPP - m * m, 0.0) * SPP / (SPP - 1)
    np.savez_compressed(os.path.join(HERE, f'stat_{NAME}.npz'), mean=mean, var=var, n=np.int64(SPP))
    with open(os.path.join(HERE, f'stat_{NAME}.json'), 'w') as f:
        json.dump(dict(SCENE, spp=SPP, height=H), f, indent=1)
    print(NAME, 'mean image', mean.mean(axis=(0, 1)), 'size', W, H)


if __name__ == '__main__':
    main()
