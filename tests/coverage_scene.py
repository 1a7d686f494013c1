"""A small parity scene that exercises every shading branch the BASELINE
scenes leave out: checker textures on a sphere and a quad (kernels.py:965-975),
an image texture on a quad (magenta, Q8), triangles with metal / dielectric /
noise materials (kernels.py:252-307, Q3), a triangle mesh, a moving sphere
(Q22), a sphere medium and a quad-box medium, an area light, and a defocus
camera (random_in_unit_disk, kernels.py:188-195). Test infrastructure only."""
import os

from ptmi import scene_data as sd
from ptmi.core import (Sphere, camera, checker_texture, color, constant_medium, dielectric, diffuse_light,
                       hittable_list, image_texture, lambertian, mesh, metal, noise_texture, point3, quad,
                       triangle, vec3)
from ptmi.scenes import Scene, _wrap, box

TORUS = os.path.join(os.path.dirname(sd.__file__), 'assets', 'torus.obj')


def coverage_scene(width=160):
    earth = image_texture(sd.load_earthmap())
    w = hittable_list()
    w.add(Sphere.stationary(point3(0, -1000, 0), 1000,
                            lambertian.from_texture(checker_texture.from_colors(0.32, color(.2, .3, .1),
                                                                               color(.9, .9, .9)))))
    w.add(quad(point3(-3.5, 0, -2.5), vec3(2, 0, 0), vec3(0, 2, 0),
               lambertian.from_texture(checker_texture.from_colors(0.5, color(1, 0, 0), color(0, 0, 1)))))
    w.add(quad(point3(1.5, 0, -2.5), vec3(2, 0, 0), vec3(0, 2, 0), lambertian.from_texture(earth)))
    w.add(Sphere.stationary(point3(0, 1, -0.5), 1.0, lambertian.from_texture(earth)))
    w.add(Sphere.stationary(point3(-2.3, 0.7, 1.0), 0.7, dielectric(1.5)))
    w.add(Sphere.stationary(point3(2.3, 0.7, 1.0), 0.7, metal(color(.8, .6, .2), 0.3)))
    w.add(Sphere.moving(point3(0, 0.4, 2.2), point3(0, 0.7, 2.2), 0.4, lambertian.from_texture(noise_texture(4.0))))
    w.add(triangle(point3(0.8, 0.0, 0.4), point3(1.8, 0.0, 0.4), point3(1.3, 1.2, 0.4), metal(color(.9, .9, .9), 0.0)))
    w.add(triangle(point3(-1.8, 0.0, 0.4), point3(-0.8, 0.0, 0.4), point3(-1.3, 1.2, 0.4), dielectric(1.5)))
    w.add(mesh(TORUS, lambertian.from_texture(noise_texture(2.0)), scale=0.45, offset=point3(-0.2, 1.9, -0.5)))
    w.add(quad(point3(-1, 3.5, -1), vec3(2, 0, 0), vec3(0, 0, 2), diffuse_light.from_color(color(4, 4, 4))))
    w.add(constant_medium.from_color(Sphere.stationary(point3(1.2, 0.45, 2.4), 0.45, dielectric(1.5)),
                                     color(.2, .4, .9), 0.8))
    w.add(constant_medium.from_color(box(point3(-2.0, 0.0, 2.0), point3(-1.2, 0.8, 2.8),
                                         lambertian.from_color(color(1, 1, 1))), color(.9, .9, .9), 1.5))
    world = _wrap(w.objects)
    cam = camera()
    cam.aspect_ratio = 16.0 / 9.0
    cam.img_width = width
    cam.samples_per_pixel = 4
    cam.vfov = 30
    cam.lookfrom = point3(0, 2.5, 9)
    cam.lookat = point3(0, 0.6, 0)
    cam.vup = vec3(0, 1, 0)
    cam.defocus_angle = 0.8
    cam.focus_distance = 8.5
    return Scene(world, cam, (0.7, 0.8, 1.0), 50)
