"""CPU: ptmi's scene builders + compile_scene + native SAH reproduce, bit for
bit, every array the reference's own compile path produced (tests/golden,
random.seed(1234)), the f32 camera upload values and the Perlin tables."""
import random

import numpy as np
import pytest

from ptmi import bvh, core, scene_compiler, scene_data as sd, scenes

CASES = [('wavefront_comparison', [400, 800]), ('vol2_final_scene', [800, 1000, 64]), ('cornell_smoke', [800, 1024])]


def compile_like_renderer(scene):
    """renderer.py:65-89 order: camera init, perlin() after the scene, compile, BVH."""
    per = core.perlin()
    out = scene_compiler.compile_scene(scene.world)
    b = bvh.compile_bvh(scene.world, out[2], out[5], out[8])
    return out, b, per


@pytest.mark.parametrize('name,widths', CASES)
def test_scene_arrays_bit_exact_vs_reference(name, widths):
    random.seed(1234)
    scene = getattr(scenes, name)()
    (geom, mats, spheres, qg, qm, quads, tg, tm, tris, img_reg, img_list), b, per = compile_like_renderer(scene)
    z = np.load(f'{sd.golden_dir()}/{name}.npz')
    assert np.array_equal(geom['sphere_data'], z['sph_sphere_data'])
    for k in sd.MAT_KEYS:
        assert np.array_equal(mats[k], z['sphm_' + k]), k
        assert np.array_equal(qm[k], z['quadm_' + k]), k
        assert np.array_equal(tm[k], z['trim_' + k]), k
    for k in sd.QUAD_KEYS:
        assert np.array_equal(qg[k], z[k]), k
    for k in sd.TRI_KEYS:
        assert np.array_equal(tg[k], z[k]), k
    for k in sd.BVH_KEYS:
        assert np.array_equal(b[k], z[k]), k
    for k, v in per.tables().items():
        assert np.array_equal(v, z[k]), k
    for w in widths:
        scene.cam.img_width = w
        scene.cam.initialize()
        up = scene.cam.upload_values()
        for k in ('center', 'pixel00', 'delta_u', 'delta_v', 'defocus_u', 'defocus_v'):
            assert np.array_equal(up[k], z[f'cam{w}_{k}']), (w, k)
        assert [up['width'], up['height']] == z[f'cam{w}_size'].tolist()
    if name == 'vol2_final_scene':
        assert len(img_list) == 1
        assert np.array_equal(scene_compiler.image_u8(img_list[0]), sd.load_earthmap())


def test_vol2_comparison_camera_4k():
    random.seed(1234)
    scene = scenes.vol2_final_scene_comparison()
    scene.cam.initialize()
    z = np.load(f'{sd.golden_dir()}/vol2_final_scene_comparison.npz')
    up = scene.cam.upload_values()
    assert [up['width'], up['height']] == [3840, 2160]
    for k in ('center', 'pixel00', 'delta_u', 'delta_v'):
        assert np.array_equal(up[k], z[f'cam3840_{k}'])


def test_mesh_scene_compiles():
    random.seed(1234)
    scene = scenes.cornell_mesh_fog()
    (geom, mats, spheres, qg, qm, quads, tg, tm, tris, _, _), b, _ = compile_like_renderer(scene)
    assert tg['num_triangles'] == 3000  # 60x25 quads fan-triangulated
    assert qm['is_constant_medium'].sum() == 6  # fog box
    n = geom['num_spheres'] + qg['num_quads'] + tg['num_triangles']
    assert b['num_bvh_nodes'] == 2 * n - 1
    assert sd.leaf_depths(b).max() <= 62


def test_leaf_depths_refuses_non_preorder_bvh():
    # the stack size comes from these depths and the kernels push without a
    # bound check, so a BVH whose children precede their parent is refused
    b = {'bvh_left_child': np.array([-1, -1, 0], np.int32), 'bvh_right_child': np.array([-1, -1, 1], np.int32)}
    import pytest
    with pytest.raises(ValueError, match='preorder'):
        sd.leaf_depths(b)
    ok = {'bvh_left_child': np.array([1, -1, -1], np.int32), 'bvh_right_child': np.array([2, -1, -1], np.int32)}
    assert sd.leaf_depths(ok).tolist() == [0, 1, 1]
