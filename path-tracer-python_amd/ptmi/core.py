"""Scene object model consumed by the scene compiler.

Construction-side counterpart of the reference's ``src/core`` + ``src/util``
(vec3.py, aabb.py, interval.py, sphere.py, quad.py, triangle.py, mesh.py,
bvh_node.py, hittable_list.py, constant_medium.py, material.py, texture.py,
perlin.py, camera.py): same class names, constructors and derived fields,
evaluated in float64 with the reference's operation order, because those
values are what ``compile_scene`` packs into f32 arrays and what decides the
primitive order (``bvh_node.from_objects`` sorts in place, bvh_node.py:41).
Only construction is modelled; ray intersection/shading lives on the GPU
(the reference's CPU ``hit``/``scatter`` have different semantics).

Scenes built from these classes compile to arrays bit-identical with the
reference's (tests/test_scene_compile.py). The compiler also accepts the
reference's own ``core`` objects (it dispatches on class names).
"""
from __future__ import annotations

import math
import os
import random

import numpy as np


# ---------------------------------------------------------------- vectors
class vec3:
    """float64 3-vector (util/vec3.py); operators keep the reference's order."""
    __slots__ = ('x', 'y', 'z')

    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __add__(self, o):
        return vec3(self.x + o.x, self.y + o.y, self.z + o.z)

    def __sub__(self, o):
        return vec3(self.x - o.x, self.y - o.y, self.z - o.z)

    def __mul__(self, s):
        if isinstance(s, vec3):
            return vec3(self.x * s.x, self.y * s.y, self.z * s.z)
        return vec3(self.x * s, self.y * s, self.z * s)

    __rmul__ = __mul__

    def __truediv__(self, s):
        return vec3(self.x / s, self.y / s, self.z / s)

    def __neg__(self):
        return vec3(-self.x, -self.y, -self.z)

    def __repr__(self):
        return f'vec3({self.x}, {self.y}, {self.z})'

    def dot(self, o):
        return self.x * o.x + self.y * o.y + self.z * o.z

    def cross(self, o):
        return vec3(self.y * o.z - self.z * o.y, self.z * o.x - self.x * o.z, self.x * o.y - self.y * o.x)

    def length_squared(self):
        return self.x ** 2 + self.y ** 2 + self.z ** 2

    def length(self):
        return math.sqrt(self.length_squared())

    def unit_vector(self):
        n = self.length()
        if n == 0:
            raise ZeroDivisionError('Cannot normalize zero vector')
        return self / n

    normalize = normalized = unit_vector

    def copy(self):
        return vec3(self.x, self.y, self.z)

    def to_list(self):
        return [self.x, self.y, self.z]

    @staticmethod
    def random(lo=0.0, hi=1.0):
        return vec3(random.uniform(lo, hi), random.uniform(lo, hi), random.uniform(lo, hi))


point3 = color = vec3


def dot(a, b):
    return a.dot(b)


def cross(a, b):
    return a.cross(b)


def normalize(v):
    return v.unit_vector()


def degrees_to_radians(deg):
    return deg * math.pi / 180.0


# ---------------------------------------------------------------- boxes
class interval:
    __slots__ = ('min', 'max')

    def __init__(self, lo=math.inf, hi=-math.inf):
        self.min, self.max = lo, hi

    @classmethod
    def from_floats(cls, lo=math.inf, hi=-math.inf):
        return cls(lo, hi)

    @classmethod
    def from_intervals(cls, a, b):
        return cls(a.min if a.min < b.min else b.min, a.max if a.max > b.max else b.max)

    def size(self):
        return self.max - self.min

    def expand(self, delta):
        pad = delta / 2
        return interval(self.min - pad, self.max + pad)


interval.empty = interval(math.inf, -math.inf)
interval.universe = interval(-math.inf, math.inf)


class aabb:
    __slots__ = ('x', 'y', 'z')

    def __init__(self, x=None, y=None, z=None):
        self.x, self.y, self.z = x, y, z

    @classmethod
    def from_intervals(cls, x, y, z):
        return cls(x, y, z)

    @classmethod
    def from_points(cls, a, b):
        def iv(p, q):
            return interval(p, q) if p < q else interval(q, p)
        return cls(iv(a.x, b.x), iv(a.y, b.y), iv(a.z, b.z))

    @classmethod
    def from_aabbs(cls, a, b):
        return cls(interval.from_intervals(a.x, b.x), interval.from_intervals(a.y, b.y),
                   interval.from_intervals(a.z, b.z))

    def axis_interval(self, n):
        return (self.x, self.y, self.z)[n]

    def longest_axis(self):
        sx, sy, sz = self.x.size(), self.y.size(), self.z.size()
        if sx >= sy:
            return 0 if sx >= sz else 2
        return 1 if sy >= sz else 2

    def _pad_to_minimums(self):
        delta = 0.0001
        if self.x.size() < delta:
            self.x = self.x.expand(delta)
        if self.y.size() < delta:
            self.y = self.y.expand(delta)
        if self.z.size() < delta:
            self.z = self.z.expand(delta)


# ---------------------------------------------------------------- textures
class texture:
    pass


class solid_color(texture):
    def __init__(self, albedo=None):
        self.albedo = albedo if albedo is not None else color(0, 0, 0)

    @classmethod
    def from_color(cls, albedo):
        return cls(albedo)

    @classmethod
    def from_rgb(cls, r, g, b):
        return cls(color(r, g, b))

    def value(self, u, v, p):
        return self.albedo


class checker_texture(texture):
    def __init__(self, scale=1.0, even=None, odd=None):
        self.inv_scale = 1.0 / scale
        self.even, self.odd = even, odd

    @classmethod
    def from_textures(cls, scale, even, odd):
        return cls(scale, even, odd)

    @classmethod
    def from_colors(cls, scale, c1, c2):
        return cls(scale, solid_color(c1), solid_color(c2))


class image_data:
    """Decoded RGB8 image; ``fdata`` = u8/255 in f32 like util/rtw_image.py:66."""

    def __init__(self, u8):
        self.u8 = np.ascontiguousarray(u8, dtype=np.uint8)
        self.fdata = self.u8.astype(np.float32) / np.float32(255.0)
        self.image_height, self.image_width = self.u8.shape[:2]


_ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')


def load_image_u8(filename):
    """RGB8 pixels of an image file; the reference's earthmap ships pre-decoded
    (PIL decode pinned once)."""
    base = os.path.basename(filename)
    if base == 'earthmap.jpg':
        return np.load(os.path.join(_ASSETS, 'earthmap_u8.npz'))['earthmap']
    from PIL import Image
    return np.array(Image.open(filename).convert('RGB'), dtype=np.uint8)


class image_texture(texture):
    def __init__(self, filename_or_u8):
        u8 = load_image_u8(filename_or_u8) if isinstance(filename_or_u8, str) else filename_or_u8
        self.image = image_data(u8)


class perlin:
    """Perlin tables (core/perlin.py): consumes the global ``random`` stream in
    the reference's order (256 x vec3.random(-1, 1), then 3 Fisher-Yates
    permutations with randint)."""
    point_count = 256

    def __init__(self):
        self.randvec = [vec3.random(-1, 1) for _ in range(self.point_count)]
        self.perm_x = self._perm()
        self.perm_y = self._perm()
        self.perm_z = self._perm()

    @classmethod
    def _perm(cls):
        p = list(range(cls.point_count))
        for i in range(cls.point_count - 1, 0, -1):
            t = random.randint(0, i)
            p[i], p[t] = p[t], p[i]
        return p

    def tables(self):
        return {'perlin_randvec': np.array([[v.x, v.y, v.z] for v in self.randvec], np.float32),
                'perlin_perm_x': np.array(self.perm_x, np.int32),
                'perlin_perm_y': np.array(self.perm_y, np.int32),
                'perlin_perm_z': np.array(self.perm_z, np.int32)}


class noise_texture(texture):
    def __init__(self, scale=1.0):
        self.noise = perlin()  # consumes `random` exactly like texture.py:79-81
        self.scale = scale


# ---------------------------------------------------------------- materials
class material:
    pass


class lambertian(material):
    def __init__(self, tex=None):
        self.tex = tex

    @classmethod
    def from_color(cls, albedo):
        return cls(solid_color(albedo))

    @classmethod
    def from_texture(cls, tex):
        return cls(tex)


class metal(material):
    def __init__(self, albedo, fuzz):
        self.albedo = albedo
        self.fuzz = fuzz if fuzz < 1.0 else 1.0


class dielectric(material):
    def __init__(self, index_of_refraction):
        self.ir = index_of_refraction


class diffuse_light(material):
    def __init__(self, tex=None):
        self.tex = tex

    @classmethod
    def from_color(cls, c):
        return cls(solid_color(c))

    @classmethod
    def from_texture(cls, tex):
        return cls(tex)


class isotropic(material):
    def __init__(self, tex=None):
        self.tex = tex

    @classmethod
    def from_color(cls, c):
        return cls(solid_color(c))

    @classmethod
    def from_texture(cls, tex):
        return cls(tex)


# ---------------------------------------------------------------- geometry
class hittable:
    def bounding_box(self):
        return self.bbox


class _center:
    """Ray(center1, center2 - center1) as used for a sphere centre (sphere.py:18-32)."""
    __slots__ = ('origin', 'direction')

    def __init__(self, origin, direction):
        self.origin, self.direction = origin, direction

    def at(self, t):
        return self.origin + t * self.direction


class Sphere(hittable):
    @classmethod
    def stationary(cls, static_center, radius, mat):
        s = cls.__new__(cls)
        s.center = _center(static_center, vec3(0, 0, 0))
        s.radius = max(0.0, radius)
        s.material = mat
        rv = vec3(radius, radius, radius)
        s.bbox = aabb.from_points(static_center - rv, static_center + rv)
        return s

    @classmethod
    def moving(cls, center1, center2, radius, mat):
        s = cls.__new__(cls)
        s.center = _center(center1, center2 - center1)
        s.radius = max(0.0, radius)
        s.material = mat
        rv = vec3(radius, radius, radius)
        b1 = aabb.from_points(s.center.at(0.0) - rv, s.center.at(0.0) + rv)
        b2 = aabb.from_points(s.center.at(1.0) - rv, s.center.at(1.0) + rv)
        s.bbox = aabb.from_aabbs(b1, b2)
        return s


class quad(hittable):
    def __init__(self, Q, u, v, mat):
        self.Q, self.u, self.v, self.mat = Q, u, v, mat
        n = u.cross(v)
        self.normal = n.unit_vector()
        self.D = self.normal.dot(Q)
        self.w = n / n.dot(n)
        d1 = aabb.from_points(Q, Q + u + v)
        d2 = aabb.from_points(Q + u, Q + v)
        self.bbox = aabb.from_aabbs(d1, d2)
        self.bbox._pad_to_minimums()


class triangle(hittable):
    def __init__(self, v0, v1, v2, mat):
        self.v0, self.v1, self.v2, self.mat = v0, v1, v2, mat
        self.edge1 = v1 - v0
        self.edge2 = v2 - v0
        self.normal = self.edge1.cross(self.edge2).unit_vector()
        lo = point3(min(v0.x, v1.x, v2.x), min(v0.y, v1.y, v2.y), min(v0.z, v1.z, v2.z))
        hi = point3(max(v0.x, v1.x, v2.x), max(v0.y, v1.y, v2.y), max(v0.z, v1.z, v2.z))
        self.bbox = aabb.from_points(lo, hi)
        self.bbox._pad_to_minimums()


class hittable_list(hittable):
    def __init__(self):
        self.objects = []
        self.bbox = aabb(interval.empty, interval.empty, interval.empty)

    def add(self, obj):
        self.objects.append(obj)
        self.bbox = aabb.from_aabbs(self.bbox, obj.bounding_box())

    def clear(self):
        self.objects = []


class bvh_node(hittable):
    """CPU median-split BVH over objects (bvh_node.py:14-47). Only its effect
    on primitive order matters to the compiler: spans of > 2 objects are
    stable-sorted in place by bbox min on the longest axis."""

    @classmethod
    def from_objects(cls, objects, start, end):
        node = cls.__new__(cls)
        bbox = objects[start].bounding_box()
        for k in range(start + 1, end):
            bbox = aabb.from_aabbs(bbox, objects[k].bounding_box())
        node.bbox = bbox
        axis = bbox.longest_axis()
        span = end - start
        if span == 1:
            node.left = node.right = objects[start]
        elif span == 2:
            node.left, node.right = objects[start], objects[start + 1]
        else:
            objects[start:end] = sorted(objects[start:end], key=lambda o: o.bounding_box().axis_interval(axis).min)
            mid = start + span // 2
            node.left = cls.from_objects(objects, start, mid)
            node.right = cls.from_objects(objects, mid, end)
        return node


class constant_medium(hittable):
    @classmethod
    def from_color(cls, boundary, c, density):
        m = cls.__new__(cls)
        m.boundary = boundary
        m.phase_function = isotropic.from_color(c)
        m.neg_inv_density = -1 / density
        return m

    @classmethod
    def from_texture(cls, boundary, tex, density):
        m = cls.__new__(cls)
        m.boundary = boundary
        m.phase_function = isotropic.from_texture(tex)
        m.neg_inv_density = -1 / density
        return m

    def bounding_box(self):
        return self.boundary.bounding_box()


class mesh(hittable):
    """Triangle mesh from a Wavefront OBJ file (replaces the pywavefront-based
    core/mesh.py:93-173): fan triangulation of each face, vertices scaled then
    offset, triangles with |cross(e1, e2)|^2 < 1e-10 skipped."""

    def __init__(self, model_path, mat, scale=1.0, offset=None, obj_filename=None, use_bvh=True):
        self.model_path, self.mat, self.scale = model_path, mat, scale
        self.offset = offset if offset is not None else point3(0, 0, 0)
        path = model_path if os.path.isfile(model_path) else self._find_obj(model_path, obj_filename)
        verts, faces = read_obj(path)
        self.triangles = []
        for f in faces:
            for i in range(1, len(f) - 1):
                a, b, c = (self._vertex(verts[j]) for j in (f[0], f[i], f[i + 1]))
                e = (b - a).cross(c - a)
                if e.length_squared() < 1e-10:
                    continue
                self.triangles.append(triangle(a, b, c, mat))
        if not self.triangles:
            raise ValueError('No valid triangles created from OBJ file')
        bb = self.triangles[0].bounding_box()
        for t in self.triangles[1:]:
            bb = aabb.from_aabbs(bb, t.bounding_box())
        self.bbox = bb

    @staticmethod
    def _find_obj(folder, name):
        if name:
            return os.path.join(folder, name)
        for root, _, files in os.walk(folder):
            for f in sorted(files):
                if f.lower().endswith('.obj'):
                    return os.path.join(root, f)
        raise FileNotFoundError(f'No OBJ files found in {folder}')

    def _vertex(self, p):
        return point3(p[0] * self.scale, p[1] * self.scale, p[2] * self.scale) + self.offset


def read_obj(path):
    """Positions and polygon vertex indices (0-based) of an OBJ file."""
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            parts = line.split()
            if not parts:
                continue
            if parts[0] == 'v':
                verts.append(tuple(float(x) for x in parts[1:4]))
            elif parts[0] == 'f':
                idx = []
                for tok in parts[1:]:
                    k = int(tok.split('/')[0])
                    idx.append(k - 1 if k > 0 else len(verts) + k)
                if len(idx) >= 3:
                    faces.append(idx)
    return verts, faces


# ---------------------------------------------------------------- camera
class camera:
    """Pinhole/thin-lens camera (core/camera.py:20-72); initialize() derives the
    ray-generation basis the renderer uploads (renderer.py:230-247)."""
    aspect_ratio = 1.0
    img_width = 100
    samples_per_pixel = 10
    vfov = 90
    lookfrom = point3(0, 0, 0)
    lookat = point3(0, 0, -1)
    vup = vec3(0, 1, 0)
    defocus_angle = 0.0
    focus_distance = 10.0

    def initialize(self):
        h_img = int(self.img_width / self.aspect_ratio)
        self.img_height = 1 if h_img < 1 else h_img
        self.pixel_samples_scale = 1.0 / self.samples_per_pixel
        self.center = self.lookfrom
        theta = degrees_to_radians(self.vfov)
        h = math.tan(theta / 2)
        vh = 2.0 * h * self.focus_distance
        vw = vh * (self.img_width / self.img_height)
        w = (self.lookfrom - self.lookat).unit_vector()
        u = self.vup.cross(w).unit_vector()
        v = w.cross(u)
        vu = vw * u
        vv = vh * -v
        self.delta_u = vu / self.img_width
        self.delta_v = vv / self.img_height
        upper_left = self.center - (self.focus_distance * w) - vu / 2 - vv / 2
        self.pixel00_loc = upper_left + 0.5 * (self.delta_u + self.delta_v)
        r = self.focus_distance * math.tan(degrees_to_radians(self.defocus_angle) / 2)
        self.defocus_disk_u = r * u
        self.defocus_disk_v = r * v

    def upload_values(self):
        """f32 values renderer.py:_upload_camera writes to the camera fields."""
        f = lambda p: np.array([p.x, p.y, p.z], np.float64).astype(np.float32)  # noqa: E731
        return {'center': f(self.center), 'pixel00': f(self.pixel00_loc), 'delta_u': f(self.delta_u),
                'delta_v': f(self.delta_v), 'defocus_u': f(self.defocus_disk_u),
                'defocus_v': f(self.defocus_disk_v), 'defocus_angle': float(np.float32(self.defocus_angle)),
                'width': self.img_width, 'height': self.img_height}
