#!/usr/bin/env python3
"""Generate golden fixtures from the reference's own pure-Python scene-compile path.

TEST INFRASTRUCTURE ONLY. Run in the build container (where /root/reference
exists); never at test time and never on the GPU box. It imports the
reference's importable modules read-only (no bytecode is written) and saves
*data only* (.npz / .json) under tests/golden/:

  * <scene>.npz   — every array `compile_scene` returns
                    (reference: src/render_server/taichi_renderer/scene_compiler.py:931-965),
                    the 7 flattened SAH-BVH arrays
                    (sah_bvh_builder.py:338-418 via bvh_compiler.py:132-168),
                    the f32 camera upload values (renderer.py:230-247 after
                    camera.initialize, core/camera.py:34-72) for the BASELINE
                    resolutions, and the Perlin tables the renderer uploads
                    (renderer.py:78-80 -> fields.py:304-318), created after the
                    scene exactly as the reference orders it.
  * earthmap_u8.npz — the decoded RGB8 earthmap (assets/images/earthmap.jpg),
                    decoded with PIL like util/rtw_image.py:58-66; the renderer
                    uses u8/255 in f32 (checked below).
  * sah_cases.npz — synthetic inputs + reference SAH outputs for edge cases
                    (coincident centroids, thin quads, triangle soups).

Scene RNG: random.seed(1234) before each scene function (the reference never
seeds; SURVEY.md §8d fixes 1234). numpy version is recorded: the SAH builder is
NEP-50 sensitive.
"""
import json
import os
import random
import sys
import types

import numpy as np

REF_SRC = '/root/reference/src'
OUT = os.path.dirname(os.path.abspath(__file__))


class _Captured(Exception):
    def __init__(self, world, cam):
        super().__init__('captured')
        self.world, self.cam = world, cam


def _install_stubs():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    # core/__init__.py -> mesh.py imports pywavefront (absent here); only the
    # OBJ loader needs it, and no BASELINE scene uses a mesh.
    sys.modules.setdefault('pywavefront', types.ModuleType('pywavefront'))
    # Skip render_server/__init__ side effects and taichi_renderer/__init__
    # (which would `import taichi`): namespace stubs with the real paths.
    for name, path in (('render_server', 'render_server'),
                       ('render_server.taichi_renderer', 'render_server/taichi_renderer')):
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(REF_SRC, path)]
        sys.modules[name] = m

    class CapFactory:
        @staticmethod
        def create(kind, world, cam, path, **kw):
            raise _Captured(world, cam)

    class CapViewer:
        def __init__(self, world, cam, path):
            raise _Captured(world, cam)

    rf = types.ModuleType('render_server.renderer_factory')
    rf.RendererFactory = CapFactory
    iv = types.ModuleType('render_server.interactive_viewer')
    iv.InteractiveViewer = CapViewer
    sys.modules['render_server.renderer_factory'] = rf
    sys.modules['render_server.interactive_viewer'] = iv


def _capture(scenes_mod, fn_name, seed):
    random.seed(seed)
    try:
        getattr(scenes_mod, fn_name)()
    except _Captured as c:
        return c.world, c.cam
    raise RuntimeError(f'{fn_name} did not reach a renderer')


def _camera_f32(cam, width, aspect=None):
    if aspect is not None:
        cam.aspect_ratio = aspect
    cam.img_width = width
    cam.initialize()
    v = lambda p: [p.x, p.y, p.z]
    rec64 = {
        'center': v(cam.center), 'pixel00': v(cam.pixel00_loc),
        'delta_u': v(cam.delta_u), 'delta_v': v(cam.delta_v),
        'defocus_u': v(cam.defocus_disk_u), 'defocus_v': v(cam.defocus_disk_v),
    }
    out = {k: np.array(x, dtype=np.float32) for k, x in rec64.items()}
    out['defocus_angle'] = np.float32(cam.defocus_angle)
    out['size'] = np.array([cam.img_width, cam.img_height], dtype=np.int32)
    out64 = {k: np.array(x, dtype=np.float64) for k, x in rec64.items()}
    return out, out64


def _pack_scene(world, cam, widths, perlin_cls, scene_compiler, bvh_compiler):
    # renderer.py:65-84 order: cam.initialize, allocate, perlin() (consumes the
    # global `random` stream), then compile_scene.
    per = perlin_cls()
    (geom, mats, spheres, qgeom, qmats, quads, tgeom, tmats, tris,
     img_reg, img_list) = scene_compiler.compile_scene(world)
    bvh = bvh_compiler.compile_bvh(world, spheres, quads, tris)
    arrs = {}
    for k, x in geom.items():
        if isinstance(x, np.ndarray):
            arrs['sph_' + k] = x
    for k, x in mats.items():
        arrs['sphm_' + k] = x
    for k, x in qgeom.items():
        if isinstance(x, np.ndarray):
            arrs[k] = x
    for k, x in qmats.items():
        arrs['quadm_' + k] = x
    for k, x in tgeom.items():
        if isinstance(x, np.ndarray):
            arrs[k] = x
    for k, x in tmats.items():
        arrs['trim_' + k] = x
    for k, x in bvh.items():
        if isinstance(x, np.ndarray):
            arrs[k] = x
    arrs['perlin_randvec'] = np.array([[p.x, p.y, p.z] for p in per.randvec], dtype=np.float32)
    arrs['perlin_perm_x'] = np.array(per.perm_x, dtype=np.int32)
    arrs['perlin_perm_y'] = np.array(per.perm_y, dtype=np.int32)
    arrs['perlin_perm_z'] = np.array(per.perm_z, dtype=np.int32)
    images = []
    for t in img_list:
        fd = t.image.fdata
        images.append({'shape': list(fd.shape)})
    for w, aspect in widths:
        c32, c64 = _camera_f32(cam, w, aspect)
        tag = f'cam{w}'
        for k, x in c32.items():
            arrs[f'{tag}_{k}'] = np.asarray(x)
        for k, x in c64.items():
            arrs[f'{tag}_f64_{k}'] = x
    meta = {
        'num_spheres': int(geom['num_spheres']), 'num_quads': int(qgeom['num_quads']),
        'num_triangles': int(tgeom['num_triangles']), 'num_bvh_nodes': int(bvh['num_bvh_nodes']),
        'images': images, 'camera_widths': [w for w, _ in widths],
        'cam_settings': {
            'aspect_ratio': cam.aspect_ratio, 'vfov': cam.vfov,
            'lookfrom': [cam.lookfrom.x, cam.lookfrom.y, cam.lookfrom.z],
            'lookat': [cam.lookat.x, cam.lookat.y, cam.lookat.z],
            'vup': [cam.vup.x, cam.vup.y, cam.vup.z],
            'defocus_angle': cam.defocus_angle, 'focus_distance': cam.focus_distance,
        },
    }
    return arrs, meta, img_list


def _sah_cases(sah):
    """Synthetic SAH inputs exercising the builder's edge paths."""
    NS = types.SimpleNamespace

    def P(x, y, z):
        return NS(x=float(x), y=float(y), z=float(z))

    def sphere(c, r):
        return NS(center=NS(at=lambda t, c=c: P(*c)), radius=float(r))

    cases = {}
    rng = np.random.default_rng(7)
    # 1) random spheres
    sp = [sphere(rng.uniform(-50, 50, 3), rng.uniform(0.1, 5)) for _ in range(300)]
    cases['spheres300'] = (sp, [], [])
    # 2) coincident centroids (median / inf-cost fallbacks)
    sp2 = [sphere((1.0, 2.0, 3.0), 0.5 + 0.01 * i) for i in range(9)]
    sp2 += [sphere((1.0, 2.0, 3.0 + (i % 2) * 1e-12), 1.0) for i in range(4)]
    cases['coincident'] = (sp2, [], [])
    # 3) axis-aligned quads (thin boxes -> pad_to_minimums) + spheres
    qd = []
    for i in range(120):
        Q = rng.uniform(-20, 20, 3)
        ax = i % 3
        u = np.zeros(3); v = np.zeros(3)
        u[(ax + 1) % 3] = rng.uniform(0.5, 4)
        v[(ax + 2) % 3] = rng.uniform(0.5, 4)
        qd.append(NS(Q=P(*Q), u=P(*u), v=P(*v)))
    cases['quads_mixed'] = (sp[:40], qd, [])
    # 4) triangle soup (OBJ-like meshes for config C4)
    tr = []
    for i in range(500):
        c = rng.uniform(-10, 10, 3)
        v0 = c + rng.uniform(-1, 1, 3)
        v1 = c + rng.uniform(-1, 1, 3)
        v2 = c + rng.uniform(-1, 1, 3)
        if i % 7 == 0:
            v2 = v0.copy(); v2[1] += 1.0; v1 = v0.copy(); v1[0] += 1.0; v1[1] = v0[1]; v2[2] = v0[2]
        tr.append(NS(v0=P(*v0), v1=P(*v1), v2=P(*v2)))
    cases['tris500'] = ([], [], tr)
    # 5) two prims / single prim
    cases['two'] = ([sphere((0, 0, 0), 1), sphere((3, 0, 0), 1)], [], [])
    cases['one'] = ([], [qd[0]], [])

    out = {}
    for name, (s, q, t) in cases.items():
        if s or t or q:
            res = sah.build_sah_bvh_from_primitives(s, q, t) if (q or t) else sah.build_sah_bvh_from_spheres(s)
        out[f'{name}__sph'] = np.array([[o.center.at(0).x, o.center.at(0).y, o.center.at(0).z, o.radius]
                                         for o in s], dtype=np.float64).reshape(-1, 4)
        out[f'{name}__quad'] = np.array([[o.Q.x, o.Q.y, o.Q.z, o.u.x, o.u.y, o.u.z, o.v.x, o.v.y, o.v.z]
                                          for o in q], dtype=np.float64).reshape(-1, 9)
        out[f'{name}__tri'] = np.array([[o.v0.x, o.v0.y, o.v0.z, o.v1.x, o.v1.y, o.v1.z, o.v2.x, o.v2.y, o.v2.z]
                                         for o in t], dtype=np.float64).reshape(-1, 9)
        for k, x in res.items():
            if isinstance(x, np.ndarray):
                out[f'{name}__{k}'] = x
    return out


def crosscheck_ptmi(scenes_mod, scene_compiler, bvh_compiler, plan, seed):
    """Drop-in check of the boundary: worlds built by the reference's own
    scenes.py / core classes go through ptmi.scene_compiler.compile_scene and
    ptmi.bvh.compile_bvh (native SAH builder), and every array must equal the
    reference's compile_scene / compile_bvh output on the same world object.
    Writes tests/golden/ptmi_crosscheck.json (data only)."""
    sys.path.insert(0, os.path.join(OUT, '..', '..', 'path-tracer-python_amd'))
    from ptmi import scene_compiler as pc, bvh as pb
    result = {}
    for name, (fn, _) in plan.items():
        world, _cam = _capture(scenes_mod, fn, seed)
        ref = scene_compiler.compile_scene(world)
        ours = pc.compile_scene(world)
        bad = []
        for i in (0, 1, 3, 4, 6, 7):
            for k, x in ref[i].items():
                y = ours[i][k]
                if isinstance(x, np.ndarray) and not (x.dtype == y.dtype and np.array_equal(x, y)):
                    bad.append(f'{i}:{k}')
                elif not isinstance(x, np.ndarray) and x != y:
                    bad.append(f'{i}:{k}')
        same_prims = all(a is b for i in (2, 5, 8) for a, b in zip(ref[i], ours[i])) and \
            all(len(ref[i]) == len(ours[i]) for i in (2, 5, 8))
        rb = bvh_compiler.compile_bvh(world, ref[2], ref[5], ref[8])
        ob = pb.compile_bvh(world, ours[2], ours[5], ours[8])
        for k, x in rb.items():
            if isinstance(x, np.ndarray) and not np.array_equal(x, np.asarray(ob[k])):
                bad.append(f'bvh:{k}')
        result[name] = {'arrays_equal': not bad, 'mismatches': bad, 'same_primitive_objects': same_prims,
                        'images': len(ours[10])}
        print(name, result[name])
    with open(os.path.join(OUT, 'ptmi_crosscheck.json'), 'w') as f:
        json.dump({'numpy': np.__version__, 'seed': seed, 'scenes': result}, f, indent=1, sort_keys=True)


def main():
    _install_stubs()
    os.chdir(REF_SRC)  # image_texture("assets/images/earthmap.jpg") is cwd-relative
    import scenes  # noqa: E402
    from core.perlin import perlin  # noqa: E402
    from render_server.taichi_renderer import scene_compiler, bvh_compiler, sah_bvh_builder  # noqa: E402

    seed = 1234
    plan = {
        # name: (scene fn, [(img_width, aspect override)])
        'wavefront_comparison': ('wavefront_comparison', [(400, None), (800, None)]),
        'vol2_final_scene': ('vol2_final_scene', [(800, None), (1000, None), (64, None)]),
        'cornell_smoke': ('cornell_smoke', [(800, None), (1024, None)]),
        'vol2_final_scene_comparison': ('vol2_final_scene_comparison', [(3840, 16.0 / 9.0)]),
    }
    if '--crosscheck-ptmi' in sys.argv:
        crosscheck_ptmi(scenes, scene_compiler, bvh_compiler, plan, seed)
        return
    manifest = {'numpy': np.__version__, 'seed': seed, 'scenes': {}}
    earth = None
    for name, (fn, widths) in plan.items():
        world, cam = _capture(scenes, fn, seed)
        arrs, meta, imgs = _pack_scene(world, cam, widths, perlin, scene_compiler, bvh_compiler)
        for t in imgs:
            from PIL import Image
            u8 = np.array(Image.open('assets/images/earthmap.jpg').convert('RGB'), dtype=np.uint8)
            assert np.array_equal((u8.astype(np.float32) / np.float32(255.0)), t.image.fdata)
            earth = u8
        np.savez_compressed(os.path.join(OUT, f'{name}.npz'), **arrs)
        manifest['scenes'][name] = meta
        print(name, meta['num_spheres'], meta['num_quads'], meta['num_triangles'], meta['num_bvh_nodes'])
    if earth is not None:
        np.savez_compressed(os.path.join(OUT, '..', '..', 'path-tracer-python_amd', 'ptmi', 'assets', 'earthmap_u8.npz'), earthmap=earth)
    np.savez_compressed(os.path.join(OUT, 'sah_cases.npz'), **_sah_cases(sah_bvh_builder))
    with open(os.path.join(OUT, 'manifest.json'), 'w') as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
