"""Compiled-scene container in the reference's array layout, and the packer
that turns it into the MI355X device layout of include/ptmi.h.

The reference compiles a scene into per-primitive-type numpy arrays
(src/render_server/taichi_renderer/scene_compiler.py:931-965) and a flattened
SAH BVH (bvh_compiler.py:132-168, sah_bvh_builder.py:338-418) and then
uploads them field by field (renderer.py:102-228). ``SceneArrays`` keeps
exactly those arrays (same names, dtypes and shapes) so fixtures captured from
the reference compare array-for-array; ``pack_device`` produces the packed
GPU layout (child-box BVH2 nodes, 16-float quads, 20-float materials, RGBA8
texels) documented in include/ptmi.h.
"""
from __future__ import annotations

import collections
import json
import os
from dataclasses import dataclass, field

import numpy as np

PRIM_SPHERE, PRIM_TRIANGLE, PRIM_QUAD = 0, 1, 2  # scene_compiler.py:10-12
MAX_IMAGES = 16

# per-type material array names (compile_materials, scene_compiler.py:425-439)
MAT_KEYS = ('material_type', 'material_albedo', 'material_fuzz', 'material_ir', 'material_emit_color',
            'texture_type', 'texture_scale', 'texture_color1', 'texture_color2', 'texture_image_idx',
            'is_constant_medium', 'medium_density', 'medium_albedo')
BVH_KEYS = ('bvh_bbox_min', 'bvh_bbox_max', 'bvh_left_child', 'bvh_right_child', 'bvh_parent',
            'bvh_prim_type', 'bvh_prim_idx')
QUAD_KEYS = ('quad_Q', 'quad_u', 'quad_v', 'quad_normal', 'quad_D', 'quad_w')
TRI_KEYS = ('triangle_v0', 'triangle_v1', 'triangle_v2', 'triangle_edge1', 'triangle_edge2', 'triangle_normal')
PERLIN_KEYS = ('perlin_randvec', 'perlin_perm_x', 'perlin_perm_y', 'perlin_perm_z')

_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'tests', 'golden')


def _empty_mats(n):
    return {
        'material_type': np.zeros(n, np.int32), 'material_albedo': np.zeros((n, 3), np.float32),
        'material_fuzz': np.zeros(n, np.float32), 'material_ir': np.zeros(n, np.float32),
        'material_emit_color': np.zeros((n, 3), np.float32), 'texture_type': np.zeros(n, np.int32),
        'texture_scale': np.ones(n, np.float32), 'texture_color1': np.zeros((n, 3), np.float32),
        'texture_color2': np.zeros((n, 3), np.float32), 'texture_image_idx': np.full(n, -1, np.int32),
        'is_constant_medium': np.zeros(n, np.int32), 'medium_density': np.zeros(n, np.float32),
        'medium_albedo': np.zeros((n, 3), np.float32),
    }


@dataclass
class SceneArrays:
    """Reference-layout compiled scene (geometry, materials, BVH, Perlin, images)."""
    sphere_data: np.ndarray
    sphere_mats: dict
    quads: dict
    quad_mats: dict
    tris: dict
    tri_mats: dict
    bvh: dict
    perlin: dict
    images: list = field(default_factory=list)  # (H, W, 3) uint8 each

    @property
    def num_spheres(self):
        return int(self.sphere_data.shape[0])

    @property
    def num_quads(self):
        return int(self.quads['quad_Q'].shape[0])

    @property
    def num_triangles(self):
        return int(self.tris['triangle_v0'].shape[0])

    @property
    def num_bvh_nodes(self):
        return int(self.bvh['bvh_bbox_min'].shape[0])

    def mats(self, prim_type):
        return {PRIM_SPHERE: self.sphere_mats, PRIM_TRIANGLE: self.tri_mats, PRIM_QUAD: self.quad_mats}[prim_type]

    # ------------------------------------------------------------ constructors
    @classmethod
    def from_compiled(cls, geometry, materials, quad_geometry, quad_materials, tri_geometry, tri_materials,
                      bvh, perlin, images):
        """From compile_scene()/compile_bvh() outputs (reference or ptmi)."""
        ns = int(geometry['num_spheres'])
        nq = int(quad_geometry['num_quads'])
        nt = int(tri_geometry['num_triangles'])
        sd = np.asarray(geometry['sphere_data'], np.float32).reshape(ns, 4)
        q = {k: np.asarray(quad_geometry[k], np.float32).reshape((nq,) if k == 'quad_D' else (nq, 3))
             for k in QUAD_KEYS}
        t = {k: np.asarray(tri_geometry[k], np.float32).reshape(nt, 3) for k in TRI_KEYS}

        def fix(m, n):
            out = _empty_mats(n)
            for k in MAT_KEYS:
                if k in m:
                    out[k] = np.asarray(m[k], out[k].dtype).reshape(out[k].shape)
            return out

        b = {k: np.asarray(bvh[k], np.float32 if 'bbox' in k else np.int32) for k in BVH_KEYS}
        b['bvh_bbox_min'] = b['bvh_bbox_min'].reshape(-1, 3)
        b['bvh_bbox_max'] = b['bvh_bbox_max'].reshape(-1, 3)
        p = {'perlin_randvec': np.asarray(perlin['perlin_randvec'], np.float32).reshape(256, 3)}
        for k in PERLIN_KEYS[1:]:
            p[k] = np.asarray(perlin[k], np.int32).reshape(256)
        return cls(sd, fix(materials, ns), q, fix(quad_materials, nq), t, fix(tri_materials, nt), b, p,
                   [np.ascontiguousarray(im, dtype=np.uint8) for im in images])

    @classmethod
    def from_npz(cls, path, images=None):
        """Load a tests/golden/<scene>.npz fixture (see gen_fixtures.py)."""
        z = np.load(path)
        geom = {'sphere_data': z['sph_sphere_data'], 'num_spheres': z['sph_sphere_data'].shape[0]}
        mats = {k: z['sphm_' + k] for k in MAT_KEYS}
        qg = {k: z[k] for k in QUAD_KEYS}
        qg['num_quads'] = z['quad_Q'].shape[0]
        qm = {k: z['quadm_' + k] for k in MAT_KEYS}
        tg = {k: z[k] for k in TRI_KEYS}
        tg['num_triangles'] = z['triangle_v0'].shape[0]
        tm = {k: z['trim_' + k] for k in MAT_KEYS}
        bvh = {k: z[k] for k in BVH_KEYS}
        per = {k: z[k] for k in PERLIN_KEYS}
        if images is None:
            used = max(int(np.max(z['sphm_texture_image_idx'], initial=-1)),
                       int(np.max(z['quadm_texture_image_idx'], initial=-1)),
                       int(np.max(z['trim_texture_image_idx'], initial=-1)))
            images = [load_earthmap()] if used >= 0 else []
        return cls.from_compiled(geom, mats, qg, qm, tg, tm, bvh, per, images)


def golden_dir():
    return os.path.normpath(_GOLDEN)


def load_earthmap():
    """Decoded RGB8 earthmap (the only image texture the BASELINE scenes use)."""
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets', 'earthmap_u8.npz'))['earthmap']


def load_fixture(name):
    return SceneArrays.from_npz(os.path.join(golden_dir(), name + '.npz'))


def fixture_camera(name, width):
    """f32 camera upload values captured from the reference (renderer.py:230-247)."""
    z = np.load(os.path.join(golden_dir(), name + '.npz'))
    tag = f'cam{width}_'
    cam = {k: np.asarray(z[tag + k], np.float32) for k in
           ('center', 'pixel00', 'delta_u', 'delta_v', 'defocus_u', 'defocus_v')}
    cam['defocus_angle'] = float(z[tag + 'defocus_angle'])
    cam['width'], cam['height'] = (int(v) for v in z[tag + 'size'])
    return cam


def camera_upload(cam):
    """f32 camera upload values (renderer.py:230-247) of an initialized camera
    object (ptmi.core.camera or the reference's), in fixture_camera's format."""
    def vec(p):
        return np.array([p.x, p.y, p.z], np.float64).astype(np.float32)
    return {'center': vec(cam.center), 'pixel00': vec(cam.pixel00_loc), 'delta_u': vec(cam.delta_u),
            'delta_v': vec(cam.delta_v), 'defocus_u': vec(cam.defocus_disk_u),
            'defocus_v': vec(cam.defocus_disk_v), 'defocus_angle': float(cam.defocus_angle),
            'width': int(cam.img_width), 'height': int(cam.img_height)}


def fixture_manifest():
    with open(os.path.join(golden_dir(), 'manifest.json')) as f:
        return json.load(f)


# ---------------------------------------------------------------- packing
LEAF_FLAG = np.int64(0x80000000)
LEAF_INDEX_BITS = 25  # leaf code: flag | type << 28 | material class << 25 | primitive index
MAX_PRIMS_PER_TYPE = 1 << LEAF_INDEX_BITS

# Material class of a leaf (include/ptmi.h PTMI_CLASS_*): which of the
# wavefront's shading lists a hit on it goes to, decided once per primitive
# from its material flags instead of by a dependent load after every traversal.
CLASS_LAMBERTIAN, CLASS_GLOSSY, CLASS_DIELECTRIC, CLASS_MEDIUM, CLASS_NOISE, CLASS_EMISSIVE = range(6)


NODE_FLOATS = 20  # 80-B internal node (include/ptmi.h)
NODE_BYTES = 4 * NODE_FLOATS  # an internal child ref is the child's byte offset in the node array
# Internal nodes sit in the node array in the reference's preorder. (A/B,
# rounds 1, 4 and 5, not kept: a 64-B stride without the stored x / y centres,
# breadth-first and depth-first sibling-pair placements; profiles/HISTORY.md §9d.)


def leaf_code(prim_type, prim_idx, mat_class=0):
    code = LEAF_FLAG | (np.int64(prim_type) << 28) | (np.int64(mat_class) << LEAF_INDEX_BITS) | np.int64(prim_idx)
    return np.int32(np.int64(code) - (1 << 32))  # as signed int32 bits


def material_class(flags):
    """Class of packed material flags (mt | tex << 4 | medium << 8 | ...):
    medium boundary; Perlin-textured Lambertian or isotropic (noise); then by
    material type: Lambertian 0, dielectric 2, emissive 3, else glossy (metal
    1, isotropic 4, unknown: scatter() decides)."""
    flags = np.asarray(flags, np.uint32).astype(np.int64)
    mt, tt, med = flags & 0xf, (flags >> 4) & 0xf, (flags >> 8) & 1
    cls = np.full(flags.shape, CLASS_GLOSSY, np.int64)
    cls[mt == 0] = CLASS_LAMBERTIAN
    cls[mt == 2] = CLASS_DIELECTRIC
    cls[mt == 3] = CLASS_EMISSIVE
    cls[(tt == 3) & ((mt == 0) | (mt == 4))] = CLASS_NOISE
    cls[med == 1] = CLASS_MEDIUM
    return cls


@dataclass
class DeviceLayout:
    """Host-side arrays in the device layout of include/ptmi.h."""
    nodes: np.ndarray       # (n_inner, node_bytes / 4) f32
    root_ref: int
    root_min: np.ndarray
    root_max: np.ndarray
    max_leaf_depth: int
    spheres: np.ndarray     # (ns, 4) f32
    quads: np.ndarray       # (nq, 16) f32
    tris: np.ndarray        # (nt, 12) f32
    mats: np.ndarray        # (ns+nq+nt, 20) f32
    texels: np.ndarray      # (sum H*W,) u32 RGBA8
    img_offset: list
    img_w: list
    img_h: list
    perlin_vec: np.ndarray  # (256, 4) f32
    perlin_perm: np.ndarray  # (768,) i32
    num_spheres: int
    num_quads: int
    num_triangles: int
    # device primitive k of type t is the reference's primitive prim_perm[t][k]
    # (types indexed sphere 0, triangle 1, quad 2; identity unless leaf_order)
    prim_perm: tuple = ()
    # the reference's own nodes for the stackless traversal (include/ptmi.h
    # ref_nodes): (num_bvh_nodes, 12) f32
    ref_nodes: np.ndarray = None

    @property
    def num_bvh_nodes(self):
        return 0 if self.ref_nodes is None else int(self.ref_nodes.shape[0])

    # internal nodes (the node array may hold unused padding rows besides)
    n_internal: int = None

    @property
    def n_inner(self):
        return int(self.nodes.shape[0]) if self.n_internal is None else int(self.n_internal)

    def nbytes(self):
        return sum(int(a.nbytes) for a in (self.nodes, self.spheres, self.quads, self.tris, self.mats,
                                              self.texels, self.perlin_vec, self.perlin_perm)
                   if a is not None) + (0 if self.ref_nodes is None else int(self.ref_nodes.nbytes))


def _pack_mats(m, n):
    out = np.zeros((n, 20), np.float32)
    out[:, 0:3] = m['material_albedo']
    out[:, 3] = m['material_fuzz']
    out[:, 4:7] = m['material_emit_color']
    out[:, 7] = m['material_ir']
    out[:, 8:11] = m['texture_color1']
    out[:, 11] = m['texture_scale']
    out[:, 12:15] = m['texture_color2']
    out[:, 15] = m['medium_density']
    out[:, 16:19] = m['medium_albedo']
    mt = m['material_type'].astype(np.int64)
    tt = m['texture_type'].astype(np.int64)
    if n and (mt.min() < 0 or mt.max() > 15 or tt.min() < 0 or tt.max() > 15):
        raise ValueError('material/texture type codes must be in [0, 15]')
    med = (m['is_constant_medium'] > 0).astype(np.int64)
    img = m['texture_image_idx'].astype(np.int64) + 1
    if n and (img.min() < 0 or img.max() > 0xffff):
        raise ValueError('texture image index out of range')
    flags = (mt | (tt << 4) | (med << 8) | (img << 16)).astype(np.uint32)
    out[:, 19] = flags.view(np.float32)
    return out


def leaf_depths(bvh):
    """Depth of every node (root = 0) of a preorder flattened BVH.

    The depths size the kernels' traversal stack, which has no overflow check,
    so a BVH whose children do not follow their parent (not the preorder
    flatten() of sah_bvh_builder.py:338-418 writes) is refused here rather
    than reported with too small a depth."""
    left, right = bvh['bvh_left_child'], bvh['bvh_right_child']
    n = left.shape[0]
    idx = np.arange(n)
    for name, ch in (('left', left), ('right', right)):
        has = ch >= 0
        if np.any(ch[has] >= n) or np.any(ch[has] <= idx[has]):
            raise ValueError(f'BVH is not in preorder: a {name} child does not follow its parent')
    depth = np.zeros(n, np.int32)
    for i in range(n):  # preorder: parents precede children
        if left[i] >= 0:
            depth[left[i]] = depth[i] + 1
        if right[i] >= 0:
            depth[right[i]] = depth[i] + 1
    return depth


def leaf_order_perm(bvh, counts):
    """Per primitive type, the reference's primitive indices in the order the
    preorder flattened BVH reaches their leaves (index order is preorder,
    sah_bvh_builder.py:338-418). Laying the device primitives and materials
    out in this order puts primitives that share a subtree, and are therefore
    tested by the same rays one after the other, on the same cache lines; the
    reference's compile order (scene_compiler.py:931) follows scene
    construction, which for vol2's 1000 randomly placed spheres is spatially
    random."""
    ptype, pidx = bvh['bvh_prim_type'], bvh['bvh_prim_idx']
    leaves = np.nonzero(pidx >= 0)[0]
    perm = []
    for t, n in enumerate(counts):
        order = pidx[leaves[ptype[leaves] == t]].astype(np.int64)
        if order.shape[0] != n or (n and not np.array_equal(np.sort(order), np.arange(n))):
            raise ValueError(f'BVH leaves of type {t} are not a permutation of the {n} primitives')
        perm.append(order)
    return tuple(perm)


def ref_layout_nodes(bvh, codes):
    """The reference's flattened nodes (fields.py:52-63, in its preorder) for
    the stackless traversal (traverse_bvh_stackless, kernels.py:453-597):
    12 f32 per node {min.xyz, left | max.xyz, right | parent, leaf code, side,
    0} (i32 bits). ``codes``: the device leaf code of every leaf (0 for
    internal nodes). ``side`` precomputes the reference's climb test
    ``0 if parent_node.left_child == node_idx else 1`` (kernels.py:506-507)."""
    left, right, parent = bvh['bvh_left_child'], bvh['bvh_right_child'], bvh['bvh_parent']
    n = left.shape[0]
    out = np.zeros((n, 12), np.float32)
    if n == 0:
        return out
    if np.any(parent[1:] < 0) or np.any(parent >= n) or parent[0] >= 0:
        raise ValueError('BVH parent pointers: only the root (node 0) may lack a parent')
    side = np.zeros(n, np.int32)
    has = parent >= 0
    side[has] = (left[parent[has]] != np.nonzero(has)[0]).astype(np.int32)
    out[:, 0:3] = bvh['bvh_bbox_min']
    out[:, 3] = left.astype(np.int32).view(np.float32)
    out[:, 4:7] = bvh['bvh_bbox_max']
    out[:, 7] = right.astype(np.int32).view(np.float32)
    out[:, 8] = parent.astype(np.int32).view(np.float32)
    out[:, 9] = np.asarray(codes, np.int32).view(np.float32)
    out[:, 10] = side.view(np.float32)
    return out


def node_slots(left, right, is_leaf):
    """Slot (row of the node array) of every internal node, by reference node
    index (-1 for leaves), in the reference's preorder, and the number of rows."""
    slot = np.full(left.shape[0], -1, np.int64)
    idx = np.nonzero(~is_leaf)[0]
    slot[idx] = np.arange(idx.shape[0])
    return slot, int(idx.shape[0])


def pack_device(sa: SceneArrays, node_bytes: int = NODE_BYTES, leaf_order: bool = True) -> DeviceLayout:
    """Reference-layout arrays -> include/ptmi.h device layout. ``node_bytes``
    is the library's node stride (ptmi_node_bytes(): 80, one child record
    per internal node). Each leaf code carries its primitive's material
    class (material_class). ``leaf_order`` renumbers each primitive type in BVH leaf order
    (leaf_order_perm); leaf codes, primitive and material rows are permuted
    together, so every lookup the kernels make finds the same data and the
    traversal visits the same leaves in the same order: results are
    unchanged bit for bit."""
    ns, nq, nt = sa.num_spheres, sa.num_quads, sa.num_triangles
    b = sa.bvh
    bmin, bmax = b['bvh_bbox_min'], b['bvh_bbox_max']
    left, right = b['bvh_left_child'], b['bvh_right_child']
    ptype, pidx = b['bvh_prim_type'], b['bvh_prim_idx']
    n = bmin.shape[0]
    if n != (2 * (ns + nq + nt) - 1 if (ns + nq + nt) else 0):
        raise ValueError(f'BVH has {n} nodes for {ns + nq + nt} primitives (expected 2N-1)')
    is_leaf = pidx >= 0
    internal = np.nonzero(~is_leaf)[0]
    if np.any(left[internal] < 0) or np.any(right[internal] < 0):
        raise ValueError('internal BVH node with a missing child')
    cidx = np.full(n, -1, np.int64)
    cidx[internal] = np.arange(internal.shape[0])
    counts = (ns, nt, nq)  # by prim type code: sphere 0, triangle 1, quad 2
    if leaf_order and n:
        perm = leaf_order_perm(b, counts)
    else:
        perm = tuple(np.arange(c, dtype=np.int64) for c in counts)
    new_idx = pidx.astype(np.int64).copy()
    for t in range(3):
        inv = np.empty(counts[t], np.int64)
        inv[perm[t]] = np.arange(counts[t])
        sel = is_leaf & (ptype == t)
        new_idx[sel] = inv[pidx[sel]]
    if max(counts) > MAX_PRIMS_PER_TYPE:
        raise ValueError(f'at most {MAX_PRIMS_PER_TYPE} primitives of one type (25-bit leaf index)')
    ps, pt, pq = perm
    mats = np.concatenate([_pack_mats(sa.sphere_mats, ns)[ps], _pack_mats(sa.quad_mats, nq)[pq],
                           _pack_mats(sa.tri_mats, nt)[pt]], axis=0)
    mat_base = np.array([0, ns + nq, ns], np.int64)  # mats rows: spheres | quads | triangles, by type code
    cls = np.zeros(n, np.int64)
    if n:
        rows = mat_base[np.where(is_leaf, ptype, 0)] + np.where(is_leaf, new_idx, 0)
        cls = np.where(is_leaf, material_class(mats[rows, 19].view(np.uint32)) if len(mats) else 0, 0)
    codes = ((LEAF_FLAG | (ptype.astype(np.int64) << 28) | (cls << LEAF_INDEX_BITS) | new_idx)
             - (1 << 32)).astype(np.int32)
    if node_bytes != NODE_BYTES:
        raise ValueError(f'unsupported node stride {node_bytes} (the library reads {NODE_BYTES}-B nodes)')
    cidx, nrows = node_slots(left, right, is_leaf)
    if nrows * node_bytes > 0x7fffffff:
        raise ValueError(f'{nrows} BVH node rows: byte offsets exceed int32')
    refs = np.where(is_leaf, codes, (cidx * node_bytes).astype(np.int32)).astype(np.int32)
    nodes = np.zeros((nrows, node_bytes // 4), np.float32)
    if internal.size:  # children interleaved per component (include/ptmi.h)
        l, r = left[internal], right[internal]
        rows = cidx[internal]
        nodes[rows, 0:12:2] = np.concatenate([bmin[l], bmax[l]], axis=1)
        nodes[rows, 1:12:2] = np.concatenate([bmin[r], bmax[r]], axis=1)
        nodes[rows, 12] = refs[l].view(np.float32)
        nodes[rows, 13] = refs[r].view(np.float32)
        # box centres (min + max) * 0.5 in f32 — the same rounding as the
        # kernels' (kernels.py:707-710), so precomputing them changes nothing
        cl = (bmin[l] + bmax[l]) * np.float32(0.5)
        cr = (bmin[r] + bmax[r]) * np.float32(0.5)
        nodes[rows, 14], nodes[rows, 15] = cl[:, 2], cr[:, 2]
        nodes[rows, 16], nodes[rows, 17] = cl[:, 0], cr[:, 0]
        nodes[rows, 18], nodes[rows, 19] = cl[:, 1], cr[:, 1]
    ref_nodes = ref_layout_nodes(b, np.where(is_leaf, codes, 0).astype(np.int32))
    if n:
        root_ref = int(refs[0])
        root_min, root_max = bmin[0].copy(), bmax[0].copy()
        max_leaf_depth = int(leaf_depths(b).max())
    else:
        root_ref, root_min, root_max, max_leaf_depth = 0, np.zeros(3, np.float32), np.zeros(3, np.float32), 0
    spheres = np.ascontiguousarray(np.asarray(sa.sphere_data, np.float32).reshape(ns, 4)[ps])
    q = sa.quads
    quads = np.zeros((nq, 16), np.float32)
    quads[:, 0:3] = q['quad_normal']
    quads[:, 3] = q['quad_D']
    quads[:, 4:7] = q['quad_Q']
    quads[:, 7:10] = q['quad_u']
    quads[:, 10:13] = q['quad_v']
    quads[:, 13:16] = q['quad_w']
    t = sa.tris
    tris = np.zeros((nt, 12), np.float32)
    tris[:, 0:3] = t['triangle_v0']
    tris[:, 3:6] = t['triangle_edge1']
    tris[:, 6:9] = t['triangle_edge2']
    tris[:, 9:12] = t['triangle_normal']
    quads, tris = quads[pq], tris[pt]
    if len(sa.images) > MAX_IMAGES:
        raise ValueError(f'at most {MAX_IMAGES} image textures')
    texels, offs, ws, hs, off = [], [], [], [], 0
    for im in sa.images:
        h, w, _ = im.shape
        rgba = np.zeros((h, w, 4), np.uint8)
        rgba[..., :3] = im
        texels.append(rgba.reshape(-1).view(np.uint32))
        offs.append(off)
        ws.append(w)
        hs.append(h)
        off += h * w
    texels = np.concatenate(texels) if texels else np.zeros(1, np.uint32)
    pv = np.zeros((256, 4), np.float32)
    pv[:, :3] = sa.perlin['perlin_randvec']
    pperm = np.concatenate([sa.perlin['perlin_perm_x'], sa.perlin['perlin_perm_y'],
                            sa.perlin['perlin_perm_z']]).astype(np.int32)
    if pperm.min() < 0 or pperm.max() > 255:
        raise ValueError('Perlin permutation out of range')
    return DeviceLayout(nodes, root_ref, root_min, root_max, max_leaf_depth, spheres, quads, tris, mats,
                        texels, offs, ws, hs, pv, pperm, ns, nq, nt, perm, ref_nodes, int(internal.shape[0]))


def compile_world(world, perlin_tables=None):
    """World -> SceneArrays the way the renderer does it (renderer.py:65-100):
    Perlin tables from a perlin() created after the scene (it draws from the
    global `random` stream), compile_scene, native SAH BVH, RGB8 images."""
    from . import bvh as bvh_mod, core, scene_compiler
    if perlin_tables is None:
        perlin_tables = core.perlin().tables()
    (geom, mats, spheres, qgeom, qmats, quads, tgeom, tmats, tris, _reg,
     img_list) = scene_compiler.compile_scene(world)
    bvh = bvh_mod.compile_bvh(world, spheres, quads, tris)
    return SceneArrays.from_compiled(geom, mats, qgeom, qmats, tgeom, tmats, bvh, perlin_tables,
                                     [scene_compiler.image_u8(t) for t in img_list])
