"""GPU parity fuzz: seeded random worlds (tests/random_scenes.py) rendered by
the HIP integrators through the C-ABI and by the CPU oracle on identical
inputs. Same bar as test_gpu_parity: per-pixel L-inf <= 1e-4 of accum/spp and
>= 99.9 % bit-identical pixels."""
import numpy as np
import pytest

from parity_helpers import compare
from random_scenes import random_scene

pytestmark = pytest.mark.gpu

LINF_TOL = 1e-4
SEEDS = list(range(24))
SPP = 3


def _oracle(sa, cam, bg, variant, spp, max_depth, seed):
    import oracle
    W, H = cam['width'], cam['height']
    fr = oracle.make_frame(cam, bg, max_depth, seed, W, H)
    acc = np.zeros((H, W, 3), np.float32)
    oracle.render(oracle.OracleScene(sa), fr, variant, acc, (0, 0, W, H), 0, spp, 0)
    return acc


@pytest.mark.parametrize('variant', ['mk', 'wf'])
@pytest.mark.parametrize('seed', SEEDS)
def test_random_world_parity(seed, variant):
    import torch
    from ptmi import device
    sa, cam, bg, max_depth = random_scene(seed)
    W, H = cam['width'], cam['height']
    ref = _oracle(sa, cam, bg, variant, SPP, max_depth, seed)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, max_depth, seed, W, H)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    (integ.render_mk if variant == 'mk' else integ.render_wf)(fr, acc, 0, SPP)
    torch.cuda.synchronize()
    linf, exact = compare(acc.cpu().numpy(), ref, SPP)
    print(f'seed {seed} {variant} prims={sa.num_spheres}/{sa.num_quads}/{sa.num_triangles} '
          f'max_depth={max_depth}: L-inf={linf:.3g} identical={exact:.5f}')
    assert linf <= LINF_TOL
    assert exact >= 0.999
