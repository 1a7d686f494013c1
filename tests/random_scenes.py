"""Seeded random worlds for the parity fuzz tests (test infrastructure only).

Each seed draws a small world from every primitive and material kind the
integrator handles (kernels.py:208-362 hits, :1020-1176 materials, :924-1017
textures, :421-448 media): spheres (stationary and moving), quads, lone
triangles, boxes, Lambertian / metal (fuzz 0 and > 0) / dielectric / light
materials with solid, checker, image and Perlin textures, and sphere or box
media. Camera pose, field of view, defocus, background and max_depth are
drawn too, so the fuzz cases reach branch mixes the fixed scenes do not.
The scenes go through the same compile path (scene_data.compile_world: the
reference's scene compiler and SAH builder) as every other parity scene.
"""
from __future__ import annotations

import random

from ptmi import scene_data as sd
from ptmi.core import (Sphere, camera, checker_texture, color, constant_medium, dielectric, diffuse_light,
                       hittable_list, image_texture, lambertian, metal, noise_texture, point3, quad, triangle,
                       vec3)
from ptmi.scenes import _wrap, box

_cache = {}


def _material(r, earth):
    k = r.random()
    c = color(r.uniform(0.05, 0.95), r.uniform(0.05, 0.95), r.uniform(0.05, 0.95))
    if k < 0.30:
        return lambertian.from_color(c)
    if k < 0.40:
        return lambertian.from_texture(checker_texture.from_colors(r.uniform(0.2, 1.0), c,
                                                                   color(0.9, 0.9, 0.9)))
    if k < 0.47:
        return lambertian.from_texture(noise_texture(r.uniform(0.5, 6.0)))
    if k < 0.53:
        return lambertian.from_texture(earth)
    if k < 0.70:
        return metal(c, 0.0 if r.random() < 0.4 else r.uniform(0.05, 0.8))
    if k < 0.85:
        return dielectric(r.choice([1.33, 1.5, 1.0 / 1.5, 2.4]))
    return diffuse_light.from_color(color(r.uniform(1, 6), r.uniform(1, 6), r.uniform(1, 6)))


def _p(r, s=3.0):
    return point3(r.uniform(-s, s), r.uniform(-0.5, s), r.uniform(-s, s))


def random_world(seed):
    """(world hittable list, background, max_depth, camera) for one seed."""
    r = random.Random(seed)
    earth = image_texture(sd.load_earthmap())
    w = hittable_list()
    if r.random() < 0.7:  # ground
        w.add(Sphere.stationary(point3(0, -1000, 0), 1000, _material(r, earth)))
    for _ in range(r.randint(3, 14)):
        k = r.random()
        if k < 0.40:
            c = _p(r)
            if r.random() < 0.2:
                w.add(Sphere.moving(c, c + vec3(0, r.uniform(0, 0.5), 0), r.uniform(0.2, 1.0), _material(r, earth)))
            else:
                w.add(Sphere.stationary(c, r.uniform(0.2, 1.2), _material(r, earth)))
        elif k < 0.60:
            w.add(quad(_p(r), vec3(r.uniform(-2, 2), r.uniform(-2, 2), r.uniform(-2, 2)),
                       vec3(r.uniform(-2, 2), r.uniform(-2, 2), r.uniform(-2, 2)), _material(r, earth)))
        elif k < 0.78:
            a = _p(r)
            w.add(triangle(a, a + vec3(r.uniform(-2, 2), r.uniform(0, 2), r.uniform(-2, 2)),
                           a + vec3(r.uniform(-2, 2), r.uniform(0, 2), r.uniform(-2, 2)), _material(r, earth)))
        elif k < 0.88:
            a = _p(r)
            w.add(box(a, a + vec3(r.uniform(0.3, 1.5), r.uniform(0.3, 1.5), r.uniform(0.3, 1.5)),
                      _material(r, earth)))
        elif k < 0.95:
            w.add(constant_medium.from_color(Sphere.stationary(_p(r), r.uniform(0.3, 1.2), dielectric(1.5)),
                                             color(r.random(), r.random(), r.random()), r.uniform(0.1, 3.0)))
        else:
            a = _p(r)
            w.add(constant_medium.from_color(box(a, a + vec3(1, 1, 1), lambertian.from_color(color(1, 1, 1))),
                                             color(r.random(), r.random(), r.random()), r.uniform(0.1, 3.0)))
    if r.random() < 0.5:  # area light
        w.add(quad(point3(-1, 4, -1), vec3(2, 0, 0), vec3(0, 0, 2), diffuse_light.from_color(color(5, 5, 5))))
    cam = camera()
    cam.aspect_ratio = r.choice([1.0, 16.0 / 9.0, 0.75])
    cam.vfov = r.uniform(20, 70)
    cam.lookfrom = point3(r.uniform(-8, 8), r.uniform(0.5, 6), r.uniform(6, 12))
    cam.lookat = point3(r.uniform(-1, 1), r.uniform(0, 1.5), r.uniform(-1, 1))
    cam.vup = vec3(0, 1, 0)
    if r.random() < 0.4:
        cam.defocus_angle = r.uniform(0.1, 2.0)
        cam.focus_distance = r.uniform(5, 12)
    bg = (0.0, 0.0, 0.0) if r.random() < 0.3 else (r.random(), r.random(), r.random())
    max_depth = r.choice([3, 8, 50])
    return w, bg, max_depth, cam


def random_scene(seed, width=64):
    """(SceneArrays, camera upload dict, background, max_depth) for one seed."""
    key = (seed, width)
    if key not in _cache:
        random.seed(1000 + seed)  # the reference's compile path draws from the global stream
        w, bg, max_depth, cam = random_world(seed)
        cam.img_width = width
        cam.initialize()
        sa = sd.compile_world(_wrap(w.objects))
        _cache[key] = (sa, sd.camera_upload(cam), bg, max_depth)
    return _cache[key]
