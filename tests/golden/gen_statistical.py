#!/usr/bin/env python3
"""Statistical goldens: the reference's own path tracer on small scenes.

TEST INFRASTRUCTURE ONLY (run in the build container, where /root/reference
exists; never at test time, never on the GPU box). It imports the reference's
pure-Python integrator read-only — core/camera.py `get_ray` + `ray_color`
(camera.py:74-137), core/material.py, core/quad.py, core/texture.py,
core/constant_medium.py, util/vec3.py — renders each scene below at SPP
samples per pixel and saves the per-pixel mean and variance of the sample
colours (float64) to stat_<scene>.npz, plus the scene in stat_<scene>.json.
SURVEY.md §8c item (6). Usage: gen_statistical.py [scene ...] (default: all).

Why this pins the oracle: on these scenes the Taichi kernels' semantics
(kernels.py) and the Python integrator differ only in ways that keep the
expectation: RR (both unbiased; disabled here on the Python side), the
cosine-sampling basis (Q4, same distribution), the extra dielectric draw
(Q28), the depth cap (Q13; albedo <= 0.8 makes bounces beyond 49 negligible)
and the RNG. tests/test_statistical.py compares the oracle's per-pixel means
against these, within the standard errors of both.

  * lambert    — Lambertian spheres under a constant sky;
  * materials  — glass, mirror (fuzz 0) and Lambertian spheres lit by an
                 emissive sphere;
  * quads      — an open box of Lambertian quads (normals face-flipped toward
                 the ray in both integrators, quad.py:61 / Q2) lit by an
                 emissive quad (emission from both sides in both, Q6), a
                 checker-textured sphere (floor-mod parity, texture.py:47-56 /
                 Q9) and an image-textured sphere (the earthmap, sphere UV +
                 v flip, sphere.py:72-82, texture.py:66-79 / Q8, Q30), seen
                 through a defocus camera (camera.py:64-67, 128-131);
  * mesh       — the same open quad box and light around a Lambertian
                 octahedron and a mirror (fuzz 0) tetrahedron: triangles
                 (core/triangle.py, Moller-Trumbore, normal flipped toward the
                 ray as the kernels do, Q2 / Q18) in a composed render, the
                 triangle half of C4's cornell_mesh_fog;
  * medium     — an isolated constant-medium sphere (nothing inside it)
                 against the sky and an emissive sphere. The two integrators
                 agree on the first free-flight segment only: entry at the
                 boundary, exit at the boundary's far side (kernels.py:417-419
                 finds it as the closest hit beyond the entry), free flight
                 -1/density * log(u) (constant_medium.py:31-58 / Q10, Q24).
                 After a scatter inside, the kernels treat the far wall as a
                 new entry with no exit and shade it as a surface (Q10), the
                 Python medium samples again: different transport. So the
                 Python side runs at max_depth 1 (a scattered path adds
                 nothing) and the kernels at max_depth 2 (the passthrough
                 consumes one wave / loop iteration, Q11, Q14; a path that
                 scattered ends at the wall's fallback shading with 0): both
                 then measure exactly transmittance x what lies behind.
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
    # Each scene: camera, background, max_depth (the Python integrator's;
    # 'kernel_max_depth' for the oracle when different), and objects:
    # spheres [center, radius, material], quads [Q, u, v, material], media
    # [boundary sphere center, radius, density, albedo]. Materials:
    # ['lambertian', rgb], ['checker', scale, rgb even, rgb odd],
    # ['image', 'earthmap.jpg'], ['diffuse_light', rgb], ['dielectric', ir],
    # ['metal', rgb] (fuzz 0).
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
    # open quad box lit by a quad light, checker + earthmap spheres, defocus camera
    'quads': {
        'width': 32, 'aspect': 16.0 / 9.0, 'vfov': 40.0, 'lookfrom': [0.0, 1.0, 4.2], 'lookat': [0.0, 0.9, 0.0],
        'vup': [0.0, 1.0, 0.0], 'background': [0.0, 0.0, 0.0], 'max_depth': 50,
        'defocus_angle': 1.5, 'focus_distance': 4.0,
        'spheres': [
            [[-0.6, 0.45, -0.2], 0.45, ['checker', 0.2, [0.1, 0.25, 0.1], [0.8, 0.8, 0.75]]],
            [[0.65, 0.5, 0.1], 0.5, ['image', 'earthmap.jpg']],
        ],
        'quads': [  # Q, u, v, material
            [[-2.0, 0.0, -1.5], [4.0, 0.0, 0.0], [0.0, 0.0, 3.5], ['lambertian', [0.7, 0.7, 0.7]]],   # floor
            [[-2.0, 0.0, -1.5], [0.0, 2.4, 0.0], [4.0, 0.0, 0.0], ['lambertian', [0.6, 0.6, 0.65]]],  # back
            [[-2.0, 0.0, -1.5], [0.0, 0.0, 3.5], [0.0, 2.4, 0.0], ['lambertian', [0.65, 0.1, 0.1]]],  # left
            [[2.0, 0.0, -1.5], [0.0, 2.4, 0.0], [0.0, 0.0, 3.5], ['lambertian', [0.12, 0.5, 0.15]]],  # right
            [[-2.0, 2.4, -1.5], [4.0, 0.0, 0.0], [0.0, 0.0, 3.5], ['lambertian', [0.7, 0.7, 0.7]]],   # ceiling
            [[-0.6, 2.38, -0.7], [1.2, 0.0, 0.0], [0.0, 0.0, 1.0], ['diffuse_light', [6.0, 6.0, 6.0]]],  # light
        ],
    },
    # triangles: a Lambertian octahedron and a mirror (fuzz 0) tetrahedron in
    # the open quad box under the quad light (the mesh half of C4's scene)
    'mesh': {
        'width': 32, 'aspect': 16.0 / 9.0, 'vfov': 40.0, 'lookfrom': [0.0, 1.0, 4.2], 'lookat': [0.0, 0.9, 0.0],
        'vup': [0.0, 1.0, 0.0], 'background': [0.0, 0.0, 0.0], 'max_depth': 50,
        'quads': [
            [[-2.0, 0.0, -1.5], [4.0, 0.0, 0.0], [0.0, 0.0, 3.5], ['lambertian', [0.7, 0.7, 0.7]]],   # floor
            [[-2.0, 0.0, -1.5], [0.0, 2.4, 0.0], [4.0, 0.0, 0.0], ['lambertian', [0.6, 0.6, 0.65]]],  # back
            [[-2.0, 0.0, -1.5], [0.0, 0.0, 3.5], [0.0, 2.4, 0.0], ['lambertian', [0.65, 0.1, 0.1]]],  # left
            [[2.0, 0.0, -1.5], [0.0, 2.4, 0.0], [0.0, 0.0, 3.5], ['lambertian', [0.12, 0.5, 0.15]]],  # right
            [[-2.0, 2.4, -1.5], [4.0, 0.0, 0.0], [0.0, 0.0, 3.5], ['lambertian', [0.7, 0.7, 0.7]]],   # ceiling
            [[-0.6, 2.38, -0.7], [1.2, 0.0, 0.0], [0.0, 0.0, 1.0], ['diffuse_light', [6.0, 6.0, 6.0]]],  # light
        ],
        'triangles': [],  # filled below: v0, v1, v2, material
    },
    # isolated constant-medium sphere against the sky and an emissive sphere
    'medium': {
        'width': 32, 'aspect': 16.0 / 9.0, 'vfov': 34.0, 'lookfrom': [0.0, 0.3, 4.0], 'lookat': [0.0, 0.0, 0.0],
        'vup': [0.0, 1.0, 0.0], 'background': [0.7, 0.8, 1.0], 'max_depth': 1, 'kernel_max_depth': 2,
        'spheres': [
            [[0.9, 0.3, -2.0], 0.8, ['diffuse_light', [2.0, 1.2, 0.4]]],
        ],
        'media': [  # boundary sphere center, radius, density, albedo
            [[-0.2, 0.0, 0.0], 0.9, 0.9, [0.8, 0.8, 0.8]],
        ],
    },
}


def _solids():
    """The 'mesh' scene's triangles: an octahedron (8) and a tetrahedron (4),
    counter-clockwise seen from outside."""
    tris = []
    c, r = (-0.6, 0.5, -0.2), 0.45
    px, nx, py, ny, pz, nz = ([c[0] + r, c[1], c[2]], [c[0] - r, c[1], c[2]], [c[0], c[1] + r, c[2]],
                              [c[0], c[1] - r, c[2]], [c[0], c[1], c[2] + r], [c[0], c[1], c[2] - r])
    for a, b, t in ((px, py, pz), (py, nx, pz), (nx, ny, pz), (ny, px, pz),
                    (py, px, nz), (nx, py, nz), (ny, nx, nz), (px, ny, nz)):
        tris.append([a, b, t, ['lambertian', [0.75, 0.55, 0.2]]])
    v = [[0.65, 0.9, 0.1], [0.25, 0.02, -0.15], [1.05, 0.02, -0.15], [0.65, 0.02, 0.55]]
    for a, b, t in ((1, 3, 2), (0, 1, 2), (0, 2, 3), (0, 3, 1)):
        tris.append([v[a], v[b], v[t], ['metal', [0.85, 0.85, 0.9]]])
    return tris


SCENES['mesh']['triangles'] = _solids()
SPP = 4096
NAME = 'lambert'


REF_IMAGES = '/root/reference/src/assets/images'


def _material(spec):
    from core.material import dielectric, diffuse_light, lambertian, metal  # noqa: E402
    from core.texture import checker_texture, image_texture  # noqa: E402
    from util import color  # noqa: E402
    kind, p = spec[0], spec[1:]
    if kind == 'lambertian':
        return lambertian.from_color(color(*p[0]))
    if kind == 'checker':
        return lambertian.from_texture(checker_texture.from_colors(p[0], color(*p[1]), color(*p[2])))
    if kind == 'image':
        return lambertian.from_texture(image_texture(os.path.join(REF_IMAGES, p[0])))
    if kind == 'diffuse_light':
        return diffuse_light.from_color(color(*p[0]))
    if kind == 'dielectric':
        return dielectric(p[0])
    if kind == 'metal':
        return metal(color(*p[0]), 0.0)
    raise ValueError(kind)


def _build():
    from gen_fixtures import _install_stubs
    _install_stubs()
    from core import Sphere, hittable_list, camera  # noqa: E402
    from core.constant_medium import constant_medium  # noqa: E402
    from core.material import lambertian  # noqa: E402
    from core.quad import quad  # noqa: E402
    from core.triangle import triangle  # noqa: E402
    from util import color, point3, vec3  # noqa: E402
    SCENE = SCENES[NAME]
    world = hittable_list()
    for c, r, spec in SCENE.get('spheres', []):
        world.add(Sphere.stationary(point3(*c), r, _material(spec)))
    for q, u, v, spec in SCENE.get('quads', []):
        world.add(quad(point3(*q), vec3(*u), vec3(*v), _material(spec)))
    for v0, v1, v2, spec in SCENE.get('triangles', []):
        world.add(triangle(point3(*v0), point3(*v1), point3(*v2), _material(spec)))
    for c, r, density, albedo in SCENE.get('media', []):
        boundary = Sphere.stationary(point3(*c), r, lambertian.from_color(color(0.5, 0.5, 0.5)))
        world.add(constant_medium.from_color(boundary, color(*albedo), density))
    cam = camera()
    cam.defocus_angle = SCENE.get('defocus_angle', 0.0)
    cam.focus_distance = SCENE.get('focus_distance', 10.0)
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
    for NAME in (sys.argv[1:] or SCENES):
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
