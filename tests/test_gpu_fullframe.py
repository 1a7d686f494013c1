"""GPU parity on whole frames at the BASELINE configs' resolutions (the window
tests in test_gpu_parity cover full spp on 64x64 windows; these cover every
pixel of the real frame at a few spp): HIP integrator through the C-ABI vs the
CPU oracle on the box's host threads. Same bar: per-pixel L-inf <= 1e-4 of
accum/spp and >= 99.9 % bit-identical pixels. Also checks the path, segment and
medium-traversal counts against the oracle's."""
import os

import numpy as np
import pytest

from parity_helpers import compare, gpu_render, oracle_render

pytestmark = pytest.mark.gpu

LINF_TOL = 1e-4
CASES = [
    # scene, width, integrator, spp (BASELINE configs[1], [2], [3], [4])
    ('vol2_final_scene', 800, 'mk', 4),
    ('vol2_final_scene', 800, 'wf', 4),
    ('cornell_mesh_fog', 1024, 'mk', 2),
    ('vol2_final_scene_comparison', 3840, 'mk', 1),
    # the 4K frame (8.3 M pixels) through the wavefront's 2^22 rays per iteration
    ('vol2_final_scene_comparison', 3840, 'wf', 1),
]


@pytest.mark.parametrize('case', CASES, ids=lambda c: f'{c[0]}-{c[1]}-{c[2]}')
def test_full_frame_parity(case):
    name, width, variant, spp = case
    threads = min(16, os.cpu_count() or 1)
    g, gst, _ = gpu_render(name, width, variant, None, 0, spp)
    H, W = g.shape[:2]
    o, ost = oracle_render(name, width, variant, (0, 0, W, H), 0, spp, threads=threads)
    linf, exact = compare(g, o, spp)
    print(f'{name} {W}x{H} {variant} spp={spp}: L-inf={linf:.3g} identical={exact:.6f} gpu={gst} oracle={ost}')
    assert linf <= LINF_TOL
    assert exact >= 0.999
    assert gst['paths'] == W * H * spp == ost['paths']
    # same paths, segment for segment: the device's traversal, Russian-roulette
    # and depth-budget counters equal the oracle's
    assert gst == ost
