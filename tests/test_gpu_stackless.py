"""GPU parity of the reference's stackless traversal (traverse_bvh_stackless,
kernels.py:453-597, switched on by USE_STACKLESS_TRAVERSAL, kernels.py:746):
the HIP integrators with frame.traversal = PTMI_TRAV_STACKLESS against the CPU
oracle's restatement of the same function, same bar as test_gpu_parity
(per-pixel L-inf <= 1e-4 of accum/spp, >= 99.9 % bit-identical pixels).

The stackless walk visits leaves left child first instead of front to back,
so it reaches the same closest hit by a different route; these tests pin the
route (the oracle's per-path segment and medium counts must match too) on the
parity windows, the edge scenes (empty world, root leaf, 52-level chain) and
both the direct and the staged megakernel.
"""
import numpy as np
import pytest

from edge_scenes import edge_scene
from parity_helpers import compare, gpu_render, oracle_render

pytestmark = pytest.mark.gpu

LINF_TOL = 1e-4

CASES = [
    ('wavefront_comparison', 400, (0, 0, 400, 225), 2),
    ('vol2_final_scene', 800, (368, 368, 64, 64), 4),
    ('vol2_final_scene', 800, (96, 560, 64, 48), 4),
    ('cornell_smoke', 800, (300, 300, 64, 64), 4),
    ('coverage', 160, (0, 0, 160, 90), 8),
    ('cornell_mesh_fog', 96, (0, 0, 96, 96), 4),
]


@pytest.mark.parametrize('variant', ['mk', 'wf'])
@pytest.mark.parametrize('case', CASES, ids=lambda c: f'{c[0]}-{c[1]}-{c[2][0]}_{c[2][1]}')
def test_stackless_parity(case, variant):
    name, width, window, spp = case
    g, gst, _ = gpu_render(name, width, variant, window, 0, spp, traversal='stackless')
    o, ost = oracle_render(name, width, variant, window, 0, spp, traversal='stackless')
    x0, y0, w, h = window
    linf, exact = compare(g[y0:y0 + h, x0:x0 + w], o[y0:y0 + h, x0:x0 + w], spp)
    print(f'stackless {name} {variant} {window}: Linf={linf:.3g} exact={exact:.5f} gpu={gst} oracle={ost}')
    assert linf <= LINF_TOL
    assert exact >= 0.999
    assert gst == ost


def test_stackless_direct_megakernel():
    """One sample per call takes the direct (unstaged) megakernel."""
    win = (368, 368, 64, 64)
    g, gst, _ = gpu_render('vol2_final_scene', 800, 'mk', win, 5, 1, chunks=[(5, 1), (6, 1)], traversal='stackless')
    o, ost = oracle_render('vol2_final_scene', 800, 'mk', win, 5, 2, traversal='stackless')
    linf, exact = compare(g, o, 2)
    assert linf <= LINF_TOL and exact >= 0.999


def _edge(name, variant, spp):
    import oracle
    import torch
    from ptmi import device
    sa, cam, bg = edge_scene(name)
    W, H = cam['width'], cam['height']
    ofr = oracle.make_frame(cam, bg, 50, 3, W, H, 'stackless')
    ref = np.zeros((H, W, 3), np.float32)
    oracle.render(oracle.OracleScene(sa), ofr, variant, ref, (0, 0, W, H), 0, spp, 0)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 3, W, H, traversal='stackless')
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    (integ.render_mk if variant == 'mk' else integ.render_wf)(fr, acc, 0, spp)
    torch.cuda.synchronize()
    got = acc.cpu().numpy()
    linf, exact = compare(got, ref, spp)
    print(f'stackless {name} {variant}: L-inf={linf:.3g} identical={exact:.5f}')
    assert linf <= LINF_TOL and exact >= 0.999
    return got


@pytest.mark.parametrize('name', ['empty', 'single', 'chain52'])
@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_stackless_edge_scenes(name, variant):
    got = _edge(name, variant, 3)
    if name == 'empty':
        bg = np.float32(3) * np.asarray(edge_scene('empty')[2], np.float32)
        assert np.array_equal(got, np.broadcast_to(bg, got.shape))


def test_stackless_needs_reference_nodes():
    """A scene view without ref_nodes cannot run the stackless traversal: the
    call fails with PTMI_EINVAL instead of reading a NULL node array."""
    import torch
    from ptmi import _lib, device
    from parity_helpers import scene_inputs
    sa, cam, bg = scene_inputs('wavefront_comparison', 400)
    ds = device.DeviceScene.from_arrays(sa)
    ds.view.ref_nodes = None
    integ = device.Integrator(ds)
    fr = device.make_frame(cam, bg, 50, 0, cam['width'], cam['height'], traversal='stackless')
    acc = torch.zeros((cam['height'], cam['width'], 3), dtype=torch.float32, device='cuda')
    for f in (integ.render_mk, integ.render_wf):
        with pytest.raises(_lib.PtmiError, match='ref_nodes'):
            f(fr, acc, 0, 2)
