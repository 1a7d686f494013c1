"""Scene compile surface (reference: src/render_server/taichi_renderer/scene_compiler.py).

``compile_scene(world)`` returns the reference's 11-tuple (scene_compiler.py:
931-965): sphere geometry/materials/list, quad geometry/materials/list,
triangle geometry/materials/list, image-texture registry and image list, with
identical array names, dtypes and values (pinned by tests/test_scene_compile.py
against arrays captured from the reference). The walk dispatches on class
names, so worlds built from the reference's own ``core`` classes and from
``ptmi.core`` compile alike.

Walk semantics kept from the reference: primitives are deduplicated by
identity in depth-first order through hittable_list / bvh_node (left then
right) / constant_medium (its boundary) / mesh (its triangles), so the
in-place sort of bvh_node.from_objects fixes the primitive order; any
primitive reachable from a constant_medium's boundary is flagged as a medium
with density -1/neg_inv_density (0.01 if neg_inv_density == 0) and albedo
phase_function.tex.value(0, 0, (0, 0, 0)) (:854-928), even where the same
object is also placed in the world as a surface (Q10).
"""
from __future__ import annotations

import numpy as np

PRIM_SPHERE, PRIM_TRIANGLE, PRIM_QUAD = 0, 1, 2
MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_EMISSIVE, MAT_ISOTROPIC = 0, 1, 2, 3, 4
TEX_SOLID, TEX_CHECKER, TEX_IMAGE, TEX_NOISE = 0, 1, 2, 3


def _kind(obj):
    return type(obj).__name__


def _children(obj):
    """Objects a container exposes to the compiler's depth-first walk."""
    k = _kind(obj)
    if k == 'hittable_list':
        return list(obj.objects)
    if k == 'bvh_node':
        return [c for c in (getattr(obj, 'left', None), getattr(obj, 'right', None)) if c is not None]
    return []


def _collect(world, leaf_kinds, into_medium=True, into_mesh=False):
    seen, out = set(), []

    def visit(obj):
        k = _kind(obj)
        if k == 'constant_medium':
            if into_medium:
                visit(obj.boundary)
        elif k == 'mesh' and into_mesh:
            for t in obj.triangles:
                if id(t) not in seen:
                    seen.add(id(t))
                    out.append(t)
        elif k in leaf_kinds:
            if id(obj) not in seen:
                seen.add(id(obj))
                out.append(obj)
        else:
            for c in _children(obj):
                visit(c)

    visit(world)
    return out


def extract_spheres(world):
    return _collect(world, ('Sphere',))


def extract_quads(world):
    return _collect(world, ('quad',))


def extract_triangles(world):
    return _collect(world, ('triangle',), into_mesh=True)


def build_image_texture_registry(world):
    """(id(texture) -> index, [textures]) in first-seen order (:812-851).
    Does not look inside constant_medium boundaries, like the reference."""
    found = {}

    def visit(obj):
        k = _kind(obj)
        if k in ('Sphere', 'quad', 'triangle'):
            mat = getattr(obj, 'material', None) if hasattr(obj, 'material') else getattr(obj, 'mat', None)
            tex = getattr(mat, 'tex', None)
            if tex is not None and _kind(tex) == 'image_texture':
                found[id(tex)] = tex
        elif k in ('hittable_list', 'bvh_node'):
            for c in _children(obj):
                visit(c)

    visit(world)
    texs = list(found.values())
    return {id(t): i for i, t in enumerate(texs)}, texs


def _boundary_prims(obj):
    k = _kind(obj)
    if k in ('Sphere', 'quad', 'triangle'):
        return [obj]
    out = []
    for c in _children(obj):
        out += _boundary_prims(c)
    return out


def build_constant_medium_registry(world):
    reg = {}

    def visit(obj):
        k = _kind(obj)
        if k == 'constant_medium':
            nid = obj.neg_inv_density
            density = -1.0 / nid if nid != 0 else 0.01
            albedo = (1.0, 1.0, 1.0)
            tex = getattr(obj.phase_function, 'tex', None)
            if tex is not None:
                try:
                    c = tex.value(0, 0, _Origin)
                    albedo = (c.x, c.y, c.z)
                except Exception:  # the reference swallows texture errors here (:905-906)
                    pass
            for p in _boundary_prims(obj.boundary):
                reg[id(p)] = {'density': density, 'albedo': albedo}
        elif k in ('hittable_list', 'bvh_node'):
            for c in _children(obj):
                visit(c)

    visit(world)
    return reg


class _P:
    x = y = z = 0.0


_Origin = _P()


def _rgb(c):
    return [c.x, c.y, c.z]


def _material_row(mat, ref_point, img_reg):
    """One primitive's material/texture record (the per-class branches of
    compile_materials, :301-417)."""
    r = {'material_type': MAT_LAMBERTIAN, 'material_albedo': [0.0, 0.0, 0.0], 'material_fuzz': 0.0,
         'material_ir': 0.0, 'material_emit_color': [0.0, 0.0, 0.0], 'texture_type': TEX_SOLID,
         'texture_scale': 1.0, 'texture_color1': [0.0, 0.0, 0.0], 'texture_color2': [0.0, 0.0, 0.0],
         'texture_image_idx': -1}
    kind = _kind(mat)
    if kind == 'lambertian':
        tex = mat.tex
        tk = _kind(tex)
        if tk == 'checker_texture':
            r.update(texture_type=TEX_CHECKER, texture_scale=1.0 / tex.inv_scale,
                     texture_color1=_rgb(tex.even.value(0, 0, ref_point)),
                     texture_color2=_rgb(tex.odd.value(0, 0, ref_point)), material_albedo=[1.0, 1.0, 1.0])
        elif tk == 'image_texture':
            r.update(texture_type=TEX_IMAGE, texture_image_idx=img_reg.get(id(tex), -1),
                     material_albedo=[1.0, 1.0, 1.0], texture_color1=[1.0, 1.0, 1.0],
                     texture_color2=[1.0, 1.0, 1.0])
        elif tk == 'noise_texture':
            r.update(texture_type=TEX_NOISE, texture_scale=tex.scale, texture_color1=[0.5, 0.5, 0.5],
                     texture_color2=[0.5, 0.5, 0.5], material_albedo=[1.0, 1.0, 1.0])
        else:
            try:
                c = _rgb(tex.value(0, 0, ref_point))
            except Exception:  # :353-356
                c = [0.8, 0.8, 0.8]
            r.update(material_albedo=c, texture_color1=c, texture_color2=c)
        r['material_ir'] = 1.0
    elif kind == 'metal':
        a = _rgb(mat.albedo)
        r.update(material_type=MAT_METAL, material_albedo=a, material_fuzz=mat.fuzz, material_ir=1.0,
                 texture_color1=a, texture_color2=a)
    elif kind == 'dielectric':
        one = [1.0, 1.0, 1.0]
        r.update(material_type=MAT_DIELECTRIC, material_albedo=one, material_ir=mat.ir, texture_color1=one,
                 texture_color2=one)
    elif kind == 'diffuse_light':
        try:
            e = _rgb(mat.tex.value(0, 0, ref_point))
        except Exception:  # :392-393
            e = [1.0, 1.0, 1.0]
        r.update(material_type=MAT_EMISSIVE, material_emit_color=e, material_ir=1.0)
    else:  # unsupported -> Lambertian 0.8 grey (:406-417)
        g = [0.8, 0.8, 0.8]
        r.update(material_albedo=g, material_ir=1.0, texture_color1=g, texture_color2=g)
    return r


def _compile_materials(prims, get_mat, get_ref, img_reg, med_reg):
    n = len(prims)
    out = {
        'material_type': np.zeros(n, np.int32), 'material_albedo': np.zeros((n, 3), np.float32),
        'material_fuzz': np.zeros(n, np.float32), 'material_ir': np.zeros(n, np.float32),
        'material_emit_color': np.zeros((n, 3), np.float32), 'texture_type': np.zeros(n, np.int32),
        'texture_scale': np.ones(n, np.float32), 'texture_color1': np.zeros((n, 3), np.float32),
        'texture_color2': np.zeros((n, 3), np.float32), 'texture_image_idx': np.full(n, -1, np.int32),
        'is_constant_medium': np.zeros(n, np.int32), 'medium_density': np.zeros(n, np.float32),
        'medium_albedo': np.zeros((n, 3), np.float32),
    }
    for i, p in enumerate(prims):
        row = _material_row(get_mat(p), get_ref(p), img_reg)
        for k, v in row.items():
            out[k][i] = v
        m = med_reg.get(id(p))
        if m is not None:
            out['is_constant_medium'][i] = 1
            out['medium_density'][i] = m['density']
            out['medium_albedo'][i] = m['albedo']
    return out


def compile_materials(spheres, image_texture_registry=None, medium_registry=None):
    return _compile_materials(spheres, lambda s: s.material, lambda s: s.center.at(0.0),
                              image_texture_registry or {}, medium_registry or {})


def compile_quad_materials(quads, image_texture_registry=None, medium_registry=None):
    return _compile_materials(quads, lambda q: q.mat, lambda q: q.Q, image_texture_registry or {},
                              medium_registry or {})


def compile_triangle_materials(triangles, image_texture_registry=None, medium_registry=None):
    return _compile_materials(triangles, lambda t: t.mat, lambda t: t.v0, image_texture_registry or {},
                              medium_registry or {})


def compile_geometry(spheres):
    sd = np.zeros((len(spheres), 4), np.float32)
    for i, s in enumerate(spheres):
        c = s.center.at(0.0)  # moving spheres use their t = 0 centre (Q22)
        sd[i] = [c.x, c.y, c.z, s.radius]
    return {'sphere_data': sd, 'num_spheres': len(spheres)}


def compile_quad_geometry(quads):
    n = len(quads)
    g = {k: np.zeros((n, 3), np.float32) for k in ('quad_Q', 'quad_u', 'quad_v', 'quad_normal', 'quad_w')}
    g['quad_D'] = np.zeros(n, np.float32)
    for i, q in enumerate(quads):
        g['quad_Q'][i] = _rgb(q.Q)
        g['quad_u'][i] = _rgb(q.u)
        g['quad_v'][i] = _rgb(q.v)
        g['quad_normal'][i] = _rgb(q.normal)
        g['quad_D'][i] = q.D
        g['quad_w'][i] = _rgb(q.w)
    g['num_quads'] = n
    return g


def compile_triangle_geometry(triangles):
    n = len(triangles)
    keys = ('triangle_v0', 'triangle_v1', 'triangle_v2', 'triangle_edge1', 'triangle_edge2', 'triangle_normal')
    attrs = ('v0', 'v1', 'v2', 'edge1', 'edge2', 'normal')
    g = {k: np.zeros((n, 3), np.float32) for k in keys}
    for i, t in enumerate(triangles):
        for k, a in zip(keys, attrs):
            g[k][i] = _rgb(getattr(t, a))
    g['num_triangles'] = n
    return g


def compile_scene(world):
    """The reference's 11-tuple (scene_compiler.py:931-965)."""
    img_reg, img_list = build_image_texture_registry(world)
    med_reg = build_constant_medium_registry(world)
    spheres = extract_spheres(world)
    quads = extract_quads(world)
    tris = extract_triangles(world)
    return (compile_geometry(spheres), compile_materials(spheres, img_reg, med_reg), spheres,
            compile_quad_geometry(quads), compile_quad_materials(quads, img_reg, med_reg), quads,
            compile_triangle_geometry(tris), compile_triangle_materials(tris, img_reg, med_reg), tris,
            img_reg, img_list)


def image_u8(tex):
    """RGB8 payload of an image texture: ptmi.core stores it; the reference's
    rtw_image keeps fdata = u8/255 (f32), inverted exactly by rounding."""
    img = tex.image
    u8 = getattr(img, 'u8', None)
    if u8 is not None:
        return u8
    fd = np.asarray(img.fdata, np.float32)
    return np.rint(fd * np.float32(255.0)).astype(np.uint8)
