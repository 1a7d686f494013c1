"""Scene builders for the BASELINE configurations.

Each builder constructs the same world as the reference scene function of the
same name in src/scenes.py — same objects, same global ``random`` calls in the
same order, same float64 arithmetic — and returns it instead of launching a
renderer (the reference functions end by opening a Tk viewer or rendering).
Seeded with random.seed(1234) they compile to arrays bit-identical with the
reference's (tests/test_scene_compile.py).

Returned: ``Scene(world, cam, background, max_depth)``; the camera keeps the
reference's defaults (img_width, samples_per_pixel) and can be resized before
rendering.
"""
from __future__ import annotations

import math
import os
import random
from dataclasses import dataclass

from .core import (Sphere, bvh_node, camera, color, constant_medium, dielectric, diffuse_light, hittable_list,
                   image_texture, lambertian, mesh, metal, noise_texture, point3, quad, vec3)


@dataclass
class Scene:
    world: object
    cam: object
    background: tuple
    max_depth: int = 50


def box(a, b, mat, angle=0.0):
    """Six quads of an (optionally Y-rotated) box, scenes.py:961-1025."""
    sides = hittable_list()
    lo = vec3(min(a.x, b.x), min(a.y, b.y), min(a.z, b.z))
    hi = vec3(max(a.x, b.x), max(a.y, b.y), max(a.z, b.z))
    dx = vec3(hi.x - lo.x, 0, 0)
    dy = vec3(0, hi.y - lo.y, 0)
    dz = vec3(0, 0, hi.z - lo.z)
    corners = [vec3(lo.x, lo.y, hi.z), vec3(hi.x, lo.y, hi.z), vec3(hi.x, lo.y, lo.z), vec3(lo.x, lo.y, lo.z),
               vec3(lo.x, hi.y, hi.z), vec3(lo.x, lo.y, lo.z)]
    if angle != 0.0:
        th = math.radians(angle)
        c, s = math.cos(th), math.sin(th)

        def rot(v):
            return vec3(c * v.x + s * v.z, v.y, -s * v.x + c * v.z)

        mid = (lo + hi) * 0.5
        dx, dyr, dz = rot(dx), rot(dy), rot(dz)
        corners = [rot(p - mid) + mid for p in corners]
    else:
        dyr = dy
    edges = [(dx, dyr), (-dz, dyr), (-dx, dyr), (dz, dyr), (dx, -dz), (dx, dz)]  # front right back left top bottom
    for q, (u, v) in zip(corners, edges):
        sides.add(quad(q, u, v, mat))
    return sides


def _cam(aspect, width, spp, vfov, lookfrom, lookat, vup=(0, 1, 0), defocus=0.0):
    cam = camera()
    cam.aspect_ratio = aspect
    cam.img_width = width
    cam.samples_per_pixel = spp
    cam.vfov = vfov
    cam.lookfrom = point3(*lookfrom)
    cam.lookat = point3(*lookat)
    cam.vup = vec3(*vup)
    cam.defocus_angle = defocus
    return cam


def _wrap(objects):
    bvh = bvh_node.from_objects(objects, 0, len(objects))
    w = hittable_list()
    w.add(bvh)
    return w


def wavefront_comparison():
    """scenes.py:1433-1530 (BASELINE configs[0] geometry)."""
    world = hittable_list()
    world.add(Sphere.stationary(point3(0, -1000, 0), 1000, lambertian.from_color(color(0.5, 0.5, 0.5))))
    for a in range(-3, 3):
        for b in range(-3, 3):
            choose = random.random()
            center = point3(a + 0.9 * random.random(), 0.2, b + 0.9 * random.random())
            if (center - point3(4, 0.2, 0)).length() > 0.9:
                if choose < 0.6:
                    mat = lambertian.from_color(color.random() * color.random())
                elif choose < 0.85:
                    alb = color.random(0.5, 1)
                    mat = metal(alb, random.uniform(0, 0.5))
                else:
                    mat = dielectric(1.5)
                world.add(Sphere.stationary(center, 0.2, mat))
    world.add(Sphere.stationary(point3(0, 1, 0), 1.0, dielectric(1.5)))
    world.add(Sphere.stationary(point3(-4, 1, 0), 1.0, lambertian.from_color(color(0.4, 0.2, 0.1))))
    world.add(Sphere.stationary(point3(4, 1, 0), 1.0, metal(color(0.7, 0.6, 0.5), 0.0)))
    world.add(Sphere.stationary(point3(0, 5, 0), 1.5, diffuse_light.from_color(color(4, 4, 4))))
    world = _wrap(world.objects)
    cam = _cam(16.0 / 9.0, 800, 200, 20, (13, 2, 3), (0, 0, 0))
    return Scene(world, cam, (0.70, 0.80, 1.00), 50)


def vol2_final_scene(aspect=1.0, width=1000):
    """scenes.py:1152-1247 (= vol2_final_scene_comparison geometry, :1256-1330)."""
    boxes1 = hittable_list()
    ground = lambertian.from_color(color(0.48, 0.83, 0.53))
    for i in range(20):
        for j in range(20):
            w = 100.0
            x0 = -1000.0 + i * w
            z0 = -1000.0 + j * w
            y1 = random.uniform(1, 101)
            boxes1.add(box(point3(x0, 0.0, z0), point3(x0 + w, y1, z0 + w), ground))
    world = hittable_list()
    world.add(bvh_node.from_objects(boxes1.objects, 0, len(boxes1.objects)))
    world.add(quad(point3(123, 554, 147), vec3(300, 0, 0), vec3(0, 0, 265),
                   diffuse_light.from_color(color(7, 7, 7))))
    c1 = point3(400, 400, 200)
    world.add(Sphere.moving(c1, c1 + vec3(30, 0, 0), 50, lambertian.from_color(color(0.7, 0.3, 0.1))))
    world.add(Sphere.stationary(point3(260, 150, 45), 50, dielectric(1.5)))
    world.add(Sphere.stationary(point3(0, 150, 145), 50, metal(color(0.8, 0.8, 0.9), 1.0)))
    boundary = Sphere.stationary(point3(360, 150, 145), 70, dielectric(1.5))
    world.add(boundary)
    world.add(constant_medium.from_color(boundary, color(0.2, 0.4, 0.9), 0.2))
    fog = Sphere.stationary(point3(0, 0, 0), 5000, dielectric(1.5))
    world.add(constant_medium.from_color(fog, color(1, 1, 1), 0.0001))
    world.add(Sphere.stationary(point3(400, 200, 400), 100,
                                lambertian.from_texture(image_texture('assets/images/earthmap.jpg'))))
    world.add(Sphere.stationary(point3(220, 280, 300), 80, lambertian.from_texture(noise_texture(0.2))))
    boxes2 = hittable_list()
    white = lambertian.from_color(color(0.73, 0.73, 0.73))
    offset = vec3(-100, 270, 395)
    for _ in range(1000):
        boxes2.add(Sphere.stationary(point3.random(0, 165) + offset, 10, white))
    world.add(bvh_node.from_objects(boxes2.objects, 0, len(boxes2.objects)))
    world = _wrap(world.objects)
    cam = _cam(aspect, width, 10000, 40, (478, 278, -600), (278, 278, 0))
    return Scene(world, cam, (0.0, 0.0, 0.0), 50)


def vol2_final_scene_comparison():
    """Same geometry; BASELINE configs[4] renders it at 3840x2160 (aspect 16/9)."""
    return vol2_final_scene(aspect=16.0 / 9.0, width=3840)


def _cornell_walls(light_q, light_u, light_v, light_emit, walls):
    red = lambertian.from_color(color(0.65, 0.05, 0.05))
    white = lambertian.from_color(color(0.73, 0.73, 0.73))
    green = lambertian.from_color(color(0.12, 0.45, 0.15))
    light = diffuse_light.from_color(color(*light_emit))
    mats = {'green': green, 'red': red, 'white': white, 'light': light}
    world = hittable_list()
    for q, u, v, m in walls(light_q, light_u, light_v):
        world.add(quad(point3(*q), vec3(*u), vec3(*v), mats[m]))
    return world, white


def cornell_box():
    """scenes.py:1028-1059."""
    def walls(lq, lu, lv):
        return [((555, 0, 0), (0, 0, 555), (0, 555, 0), 'green'), ((0, 0, 0), (0, 555, 0), (0, 0, 555), 'red'),
                (lq, lu, lv, 'light'), ((0, 0, 0), (0, 0, 555), (555, 0, 0), 'white'),
                ((555, 555, 555), (-555, 0, 0), (0, 0, -555), 'white'),
                ((0, 0, 555), (0, 555, 0), (555, 0, 0), 'white')]
    world, white = _cornell_walls((343, 554, 332), (-130, 0, 0), (0, 0, -105), (15, 15, 15), walls)
    world.add(box(point3(130, 0, 65), point3(295, 165, 230), white, -18))
    world.add(box(point3(265, 0, 295), point3(430, 330, 460), white, 15))
    world = _wrap(world.objects)
    return Scene(world, _cam(1.0, 800, 500, 40, (278, 278, -800), (278, 278, 0)), (0.0, 0.0, 0.0), 50)


def _cornell_smoke_walls(lq, lu, lv):
    return [((555, 0, 0), (0, 555, 0), (0, 0, 555), 'green'), ((0, 0, 0), (0, 555, 0), (0, 0, 555), 'red'),
            (lq, lu, lv, 'light'), ((0, 555, 0), (555, 0, 0), (0, 0, 555), 'white'),
            ((0, 0, 0), (555, 0, 0), (0, 0, 555), 'white'), ((0, 0, 555), (555, 0, 0), (0, 555, 0), 'white')]


def cornell_smoke():
    """scenes.py:1094-1149: Cornell box with two smoke boxes."""
    world, white = _cornell_walls((113, 554, 127), (330, 0, 0), (0, 0, 305), (7, 7, 7), _cornell_smoke_walls)
    box1 = box(point3(265, 0, 295), point3(430, 330, 460), white, 15)
    box2 = box(point3(130, 0, 65), point3(295, 165, 230), white, -18)
    world.add(constant_medium.from_color(box1, color(0, 0, 0), 0.01))
    world.add(constant_medium.from_color(box2, color(1, 1, 1), 0.01))
    world = _wrap(world.objects)
    return Scene(world, _cam(1.0, 800, 1000, 40, (278, 278, -800), (278, 278, 0)), (0.0, 0.0, 0.0), 50)


_MESH_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')


def cornell_mesh_fog(obj_path=None, width=1024):
    """BASELINE configs[3] (build-supplied; the reference has no such scene):
    the cornell_smoke room with an OBJ triangle mesh on the floor and a
    global constant-medium fog volume (box of density 0.002)."""
    world, white = _cornell_walls((113, 554, 127), (330, 0, 0), (0, 0, 305), (7, 7, 7), _cornell_smoke_walls)
    path = obj_path or os.path.join(_MESH_DIR, 'torus.obj')
    metal_mat = metal(color(0.8, 0.85, 0.88), 0.05)
    world.add(mesh(path, metal_mat, scale=120.0, offset=point3(278, 140, 278)))
    world.add(box(point3(130, 0, 65), point3(295, 165, 230), white, -18))
    fog_box = box(point3(1, 1, 1), point3(554, 553, 554), white)
    world.add(constant_medium.from_color(fog_box, color(1, 1, 1), 0.002))
    world = _wrap(world.objects)
    return Scene(world, _cam(1.0, width, 512, 40, (278, 278, -800), (278, 278, 0)), (0.0, 0.0, 0.0), 50)


SCENES = {'wavefront_comparison': wavefront_comparison, 'vol2_final_scene': vol2_final_scene,
          'vol2_final_scene_comparison': vol2_final_scene_comparison, 'cornell_box': cornell_box,
          'cornell_smoke': cornell_smoke, 'cornell_mesh_fog': cornell_mesh_fog}
