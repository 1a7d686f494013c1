"""CPU: the parity fuzz worlds (tests/random_scenes.py) compile into valid
reference-layout BVHs (sah_bvh_builder.py:338-418: preorder, left child at
i + 1, parents, node box = union of the children's boxes, every primitive in
exactly one leaf) and the oracle renders them to finite, non-negative
radiance in both integrator variants."""
import numpy as np
import pytest

from ptmi import scene_data as sd
from random_scenes import random_scene

SEEDS = list(range(24))


def _check_bvh(sa):
    b = sa.bvh
    n = sa.num_bvh_nodes
    nprims = sa.num_spheres + sa.num_quads + sa.num_triangles
    assert n == (2 * nprims - 1 if nprims else 0)
    if n == 0:
        return
    lo, hi = np.asarray(b['bvh_bbox_min']), np.asarray(b['bvh_bbox_max'])
    left, right = np.asarray(b['bvh_left_child']), np.asarray(b['bvh_right_child'])
    parent, ptype, pidx = np.asarray(b['bvh_parent']), np.asarray(b['bvh_prim_type']), np.asarray(b['bvh_prim_idx'])
    assert parent[0] == -1
    seen = set()
    for i in range(n):
        if pidx[i] >= 0:  # leaf
            assert left[i] == -1 and right[i] == -1
            seen.add((int(ptype[i]), int(pidx[i])))
        else:
            l, r = left[i], right[i]
            assert l == i + 1 and i < r < n
            assert parent[l] == i and parent[r] == i
            assert np.array_equal(lo[i], np.minimum(lo[l], lo[r]))
            assert np.array_equal(hi[i], np.maximum(hi[l], hi[r]))
    counts = {sd.PRIM_SPHERE: sa.num_spheres, sd.PRIM_QUAD: sa.num_quads, sd.PRIM_TRIANGLE: sa.num_triangles}
    assert seen == {(t, k) for t, c in counts.items() for k in range(c)}


@pytest.mark.parametrize('seed', SEEDS)
def test_random_world_compiles_and_renders(seed):
    import oracle
    sa, cam, bg, max_depth = random_scene(seed)
    _check_bvh(sa)
    W, H = cam['width'], cam['height']
    fr = oracle.make_frame(cam, bg, max_depth, seed, W, H)
    for variant in ('mk', 'wf'):
        acc = np.zeros((H, W, 3), np.float32)
        oracle.render(oracle.OracleScene(sa), fr, variant, acc, (0, 0, W, H), 0, 2, 0)
        assert np.isfinite(acc).all() and (acc >= 0).all()
