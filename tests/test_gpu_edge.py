"""GPU parity on edge cases the BASELINE scenes do not reach (through the
C-ABI, against the CPU oracle, same bar as test_gpu_parity: per-pixel L-inf
<= 1e-4 of accum/spp, and bit-exact in practice):

* an empty scene and a one-sphere scene (the BVH root is a leaf);
* linear BVHs 21, 28 and 51 levels deep, which select the 24-, 32- and
  64-slot traversal kernels (the reference's 64-slot stack, kernels.py:719);
* a linear BVH 69 levels deep whose walk overflows the reference's 64-entry
  stack, so pushes are dropped (kernels.py:719-740): the reference-stack walk;
* max_depth 1 and 2 (kernels.py:1139-1141 / 1383);
* a zero-sample call, which must leave the accumulator untouched;
* 1x1, 3x1 and 13x7 frames (smaller than a wave or the pipes' work, ragged 8x8 squares);
* a scene of noise-textured surfaces, so the megakernel's shading rounds
  evaluate the turbulence of many lanes at once.
"""
import numpy as np
import pytest

from edge_scenes import edge_scene
from parity_helpers import compare

pytestmark = pytest.mark.gpu

LINF_TOL = 1e-4


def _oracle(sa, cam, bg, variant, spp, max_depth=50, seed=3):
    import oracle
    W, H = cam['width'], cam['height']
    fr = oracle.make_frame(cam, bg, max_depth, seed, W, H)
    acc = np.zeros((H, W, 3), np.float32)
    oracle.render(oracle.OracleScene(sa), fr, variant, acc, (0, 0, W, H), 0, spp, 0)
    return acc


def _gpu(sa, cam, bg, variant, spp, max_depth=50, seed=3, acc=None):
    import torch
    from ptmi import device
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, max_depth, seed, W, H)
    if acc is None:
        acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    (integ.render_mk if variant == 'mk' else integ.render_wf)(fr, acc, 0, spp)
    torch.cuda.synchronize()
    return acc.cpu().numpy()


def _check(name, variant, spp, max_depth=50):
    sa, cam, bg = edge_scene(name)
    ref = _oracle(sa, cam, bg, variant, spp, max_depth)
    got = _gpu(sa, cam, bg, variant, spp, max_depth)
    linf, exact = compare(got, ref, spp)
    print(f'{name} {variant} spp={spp} max_depth={max_depth}: L-inf={linf:.3g} identical={exact:.5f}')
    assert linf <= LINF_TOL
    assert exact >= 0.999
    return got


@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_empty_scene_is_background(variant):
    got = _check('empty', variant, 3)
    bg = np.float32(3) * np.asarray(edge_scene('empty')[2], np.float32)
    assert np.array_equal(got, np.broadcast_to(bg, got.shape))


@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_single_primitive_root_leaf(variant):
    got = _check('single', variant, 4)
    assert not np.allclose(got, got[0, 0])  # the sphere is in view


@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_noise_textured_scene(variant):
    """perlin_turb3_wave: 2..64 Perlin lanes per shading round, bit-identical to the oracle."""
    _check('marble', variant, 4)


@pytest.mark.parametrize('name', ['chain22', 'chain29', 'chain52'])
@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_deep_bvh_uses_wider_stacks(name, variant):
    from ptmi import scene_data as sd
    depth = sd.pack_device(edge_scene(name)[0]).max_leaf_depth
    assert depth + 1 > 20  # beyond the 16/20-slot kernels
    _check(name, variant, 4)


@pytest.mark.parametrize('spp', [1, 4])
@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_stack_overflow_drops_match_the_oracle(variant, spp):
    """Leaf depth 69 (chainx70): the reference's 64-entry stack drops pushes
    (kernels.py:719-740; tests/test_stack_overflow.py shows the drop changes
    the image); both integrators run its exact walk (TravRS) and match the
    oracle, direct (1 spp) and staged / wavefront (4 spp), counters included."""
    import torch
    from ptmi import device
    from parity_helpers import compare
    import oracle
    sa, cam, bg = edge_scene('chainx70')
    W, H = cam['width'], cam['height']
    fr = oracle.make_frame(cam, bg, 50, 3, W, H)
    ref = np.zeros((H, W, 3), np.float32)
    ost = oracle.render(oracle.OracleScene(sa), fr, variant, ref, (0, 0, W, H), 0, spp, 0)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    (integ.render_mk if variant == 'mk' else integ.render_wf)(device.make_frame(cam, bg, 50, 3, W, H), acc, 0, spp)
    torch.cuda.synchronize()
    linf, exact = compare(acc.cpu().numpy(), ref, spp)
    assert linf <= LINF_TOL and exact >= 0.999
    assert integ.read_counters() == ost


@pytest.mark.parametrize('name', ['chain17', 'chain18', 'chain19', 'chain20'])
@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_leaf_depth_16_to_19_exact_slot_kernels(name, variant):
    # leaf depth 16-18: the staged megakernel's 17-, 18- and 19-slot kernels
    # (exact-stack kernels 17-19); 19: its 20-slot kernel; the wavefront's 20-slot ones
    from ptmi import scene_data as sd
    depth = sd.pack_device(edge_scene(name)[0]).max_leaf_depth
    assert depth == int(name[5:]) - 1
    _check(name, variant, 4)


@pytest.mark.parametrize('max_depth', [1, 2])
@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_small_max_depth(variant, max_depth):
    _check('chain22', variant, 4, max_depth)


@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_zero_samples_leave_accumulator_untouched(variant):
    import torch
    sa, cam, bg = edge_scene('single')
    W, H = cam['width'], cam['height']
    acc = torch.full((H, W, 3), 0.25, dtype=torch.float32, device='cuda')
    got = _gpu(sa, cam, bg, variant, 0, acc=acc)
    assert np.all(got == np.float32(0.25))


@pytest.mark.parametrize('width', [1, 3, 13])
@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_tiny_and_ragged_frames(variant, width):
    """Frames far smaller than a wave, a tile or the wavefront's four pipes (most pipes get no
    work and drain at once), and widths that are not multiples of the 8x8 work squares."""
    sa, cam, bg = edge_scene('single', width)
    W, H = cam['width'], cam['height']
    ref = _oracle(sa, cam, bg, variant, 5)
    got = _gpu(sa, cam, bg, variant, 5)
    linf, exact = compare(got, ref, 5)
    print(f'{W}x{H} {variant}: L-inf={linf:.3g} identical={exact:.5f}')
    assert linf <= LINF_TOL
    assert exact >= 0.999


def test_library_loaded_before_torch_still_renders():
    """Compiling a scene first loads libptmi (native SAH builder) before torch; the GPU path must
    still work in that order (one HIP runtime per process, ptmi/_lib.py load())."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = '''
import sys
sys.path[:0] = [{pkg!r}, {tests!r}]
from edge_scenes import edge_scene
sa, cam, bg = edge_scene('single', 16)          # native SAH builder: libptmi loads here
import torch
from ptmi import device
integ = device.Integrator(device.DeviceScene.from_arrays(sa))
fr = device.make_frame(cam, bg, 50, 3, cam['width'], cam['height'])
acc = torch.zeros((cam['height'], cam['width'], 3), dtype=torch.float32, device='cuda')
integ.render_mk(fr, acc, 0, 2)
integ.render_wf(fr, acc, 2, 2)
torch.cuda.synchronize()
print('render ok', float(acc.sum()))
'''.format(pkg=os.path.join(root, 'path-tracer-python_amd'), tests=os.path.join(root, 'tests'))
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and 'render ok' in r.stdout, r.stdout + r.stderr
