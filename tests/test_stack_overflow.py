"""The reference's stack overflow (kernels.py:719-740) is part of its result.

traverse_bvh_legacy keeps a 64-entry stack and silently drops a push once it
holds 64 entries. For leaf depth <= 62 that never happens; the edge scene
`chainx70` (a linear BVH of leaf depth 69, seen along the chain so that one
far leaf stays on the stack per level, tests/edge_scenes.py) makes it happen.
The oracle reproduces the drop (pt_oracle.c traverse_bvh); this CPU test
checks that the scene really overflows — the oracle rebuilt with a 256-entry
stack renders a different image — so that the GPU edge test
(test_gpu_edge.py::test_stack_overflow_drops_match_the_oracle) compares the
integrators on the drop itself.
"""
import os
import subprocess

import numpy as np

import oracle
from edge_scenes import edge_scene
from ptmi import scene_data as sd


def _render(name, lib=None, variant='mk'):
    sa, cam, bg = edge_scene(name, 64)
    W, H = cam['width'], cam['height']
    fr = oracle.make_frame(cam, bg, 50, 0, W, H)
    acc = np.zeros((H, W, 3), np.float32)
    oracle.render(oracle.OracleScene(sa), fr, variant, acc, (0, 0, W, H), 0, 2, lib=lib)
    return acc


def test_chainx70_overflows_the_reference_stack(tmp_path):
    assert sd.pack_device(edge_scene('chainx70', 64)[0]).max_leaf_depth == 69
    src = os.path.join(os.path.dirname(oracle.__file__), 'pt_oracle.c')
    so = str(tmp_path / 'libptoracle_stack256.so')
    subprocess.run(['gcc', '-O2', '-std=c11', '-fPIC', '-shared', '-ffp-contract=off', '-fno-fast-math',
                    '-DOR_STACK_SLOTS=256', '-o', so, src, '-lm'], check=True)
    big = oracle.load_variant(so)
    for variant in ('mk', 'wf'):
        ref64 = _render('chainx70', None, variant)
        ref256 = _render('chainx70', big, variant)
        differ = np.any(ref64 != ref256, axis=2).mean()
        assert differ > 0.01, f'{variant}: the 64-entry stack dropped nothing visible ({differ:.4f})'
    # no overflow below leaf depth 63: identical with either stack
    assert np.array_equal(_render('chainx52', None), _render('chainx52', big))
