"""GPU parity: the HIP integrator (through the C-ABI) against the CPU oracle
on the same fixture scenes, camera, seed and samples.

Tolerance (north star): per-pixel L-inf of accum/spp <= 1e-4. The arithmetic
and random-stream contract (include/ptmi_math.h, ptmi_rng.h) is shared, so the
expected result is bit-exact; the test also requires >= 99.9 % of pixels to
be bit-identical and reports the fraction.
"""
import numpy as np
import pytest

from parity_helpers import compare, gpu_render, oracle_render

pytestmark = pytest.mark.gpu

LINF_TOL = 1e-4

CASES = [
    # name, camera width, window (x0, y0, w, h), samples
    ('wavefront_comparison', 400, (0, 0, 400, 225), 2),          # BASELINE config 1 geometry, full frame
    ('vol2_final_scene', 800, (368, 368, 64, 64), 4),            # centre window (spheres, medium, glass)
    ('vol2_final_scene', 800, (96, 560, 64, 48), 4),             # ground boxes (quads)
    ('vol2_final_scene', 800, (560, 200, 48, 48), 4),            # earth / noise spheres region
    ('cornell_smoke', 800, (300, 300, 64, 64), 4),               # smoke volumes (quad media)
    ('vol2_final_scene', 64, (0, 0, 64, 64), 8),                 # small full frame
    ('coverage', 160, (0, 0, 160, 90), 8),                       # checker/image-on-quad/triangles/defocus
    ('cornell_mesh_fog', 1024, (448, 448, 64, 64), 4),           # BASELINE configs[3]: OBJ torus + fog
    ('cornell_mesh_fog', 96, (0, 0, 96, 96), 4),                 # same scene, small full frame
]


@pytest.mark.parametrize('variant', ['mk', 'wf'])
@pytest.mark.parametrize('case', CASES, ids=lambda c: f'{c[0]}-{c[1]}-{c[2][0]}_{c[2][1]}')
def test_parity(case, variant):
    name, width, window, spp = case
    g, gst, _ = gpu_render(name, width, variant, window, 0, spp)
    o, ost = oracle_render(name, width, variant, window, 0, spp)
    x0, y0, w, h = window
    linf, exact = compare(g[y0:y0 + h, x0:x0 + w], o[y0:y0 + h, x0:x0 + w], spp)
    print(f'{name} {variant} {window}: Linf={linf:.3g} exact={exact:.5f} gpu={gst} oracle={ost}')
    assert linf <= LINF_TOL
    assert exact >= 0.999
    # pixels outside the window untouched
    mask = np.ones(g.shape[:2], bool)
    mask[y0:y0 + h, x0:x0 + w] = False
    assert not np.any(g[mask])
    assert gst['paths'] == w * h * spp == ost['paths']
    assert gst == ost  # segments, medium exits, Russian-roulette and depth-budget ends too


@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_sample_chunking_is_exact(variant):
    """Rendering samples in several launches == one launch (accumulation order kept)."""
    win = (200, 300, 64, 32)
    a, _, integ = gpu_render('vol2_final_scene', 800, variant, win, 0, 6)
    b, _, _ = gpu_render('vol2_final_scene', 800, variant, win, 0, 6, chunks=[(0, 1), (1, 3), (4, 2)], integ=integ)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize('variant', ['mk', 'wf'])
def test_band_sharding_is_bit_identical(variant):
    """Row-band tile sharding (multi-GPU partition) reproduces the full render exactly."""
    win = (0, 0, 64, 64)
    full, _, integ = gpu_render('vol2_final_scene', 64, variant, win, 0, 4)
    parts = np.zeros_like(full)
    for r in range(3):
        p, _, _ = gpu_render('vol2_final_scene', 64, variant, win, 0, 4, band=(8, 3, r), integ=integ)
        assert not np.any(parts[p != 0])  # bands are disjoint
        parts += p
    assert np.array_equal(parts, full, equal_nan=True)


def test_tonemap_matches_reference_formula():
    import torch
    from ptmi import device, scene_data as sd
    from parity_helpers import fixture
    integ = device.Integrator(device.DeviceScene.from_arrays(fixture('cornell_smoke')))
    rng = np.random.default_rng(3)
    acc = (rng.random((37, 53, 3), dtype=np.float32) * 40.0 - 2.0).astype(np.float32)
    acc[0, 0] = [0.0, -0.0, 1e30]
    for spp in (1, 7, 1024):
        out = integ.tonemap(torch.from_numpy(acc).cuda(), spp).cpu().numpy()
        # LivePreview.buffer_to_image, preview.py:129-132 (numpy, NEP 50)
        scale = 1.0 / max(1, spp)
        ref = np.clip(np.sqrt(np.maximum(0, acc * scale)) * 255.999, 0, 255).astype(np.uint8)
        assert np.array_equal(out, ref)


@pytest.mark.parametrize('band', [(1, 1, 0), (8, 2, 1)])
def test_staged_megakernel_equals_direct(band):
    """ptmi_mk_render_ws (tile x sample-chunk units, staged colours, ordered
    resolve) is bit-identical to ptmi_mk_render (per-thread accumulation)."""
    import torch
    from ptmi import device
    from parity_helpers import scene_inputs
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, 800, 800, (96, 200, 200, 136), band)
    out = []
    for staged in (False, True):
        acc = torch.zeros((800, 800, 3), dtype=torch.float32, device='cuda')
        acc[:] = 0.25  # accumulate onto a non-zero image
        integ.render_mk(fr, acc, 3, 37, staged=staged)
        integ.render_mk(fr, acc, 40, 5, staged=staged)
        torch.cuda.synchronize()
        out.append(acc.cpu().numpy())
    assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize('traversal', ['stack', 'stackless'])
def test_overlapped_megakernel_is_bit_identical(traversal):
    """render_mk(overlap=True): traces on two side streams into two workspaces,
    resolves in call order on the caller's stream (ptmi_mk_trace_ws /
    ptmi_mk_resolve_ws) == the plain staged calls, bit for bit, counters too."""
    import torch
    from ptmi import device
    from parity_helpers import scene_inputs
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, 800, 800, (96, 200, 200, 136), traversal=traversal)
    out, cnt = [], []
    for overlap in (False, True):
        acc = torch.zeros((800, 800, 3), dtype=torch.float32, device='cuda')
        acc[:] = 0.25
        integ.reset_counters()
        for s0, n in ((0, 5), (5, 1), (6, 7), (13, 3), (16, 2)):
            integ.render_mk(fr, acc, s0, n, overlap=overlap)
        torch.cuda.synchronize()
        out.append(acc.cpu().numpy())
        cnt.append(integ.read_counters())
    assert np.array_equal(out[0], out[1])
    assert cnt[0] == cnt[1]
