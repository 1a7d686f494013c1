"""Shared helpers for parity tests: render a fixture scene window with the HIP
integrator and with the CPU oracle on identical inputs and compare."""
from __future__ import annotations

import numpy as np

from ptmi import scene_data as sd

BG = {'wavefront_comparison': (0.7, 0.8, 1.0), 'vol2_final_scene': (0.0, 0.0, 0.0),
      'cornell_smoke': (0.0, 0.0, 0.0), 'vol2_final_scene_comparison': (0.0, 0.0, 0.0)}

# Scenes compiled here (not captured from the reference): the build-supplied
# BASELINE configs[3] scene and the branch-coverage scene.
BUILT = ('cornell_mesh_fog', 'coverage')

_cache = {}


def _built(name, width):
    import random
    key = (name, width)
    if key not in _cache:
        if name == 'coverage':
            from coverage_scene import coverage_scene
            random.seed(1234)
            sc = coverage_scene(width)
        else:
            from ptmi import scenes
            random.seed(1234)
            sc = scenes.SCENES[name]()
            sc.cam.img_width = width
        sc.cam.initialize()
        sa = sd.compile_world(sc.world)
        _cache[key] = (sa, sd.camera_upload(sc.cam), tuple(sc.background))
    return _cache[key]


def fixture(name, width=None):
    if name in BUILT:
        return _built(name, width)[0]
    if name not in _cache:
        _cache[name] = sd.load_fixture(name)
    return _cache[name]


def scene_inputs(name, width):
    """(SceneArrays, camera upload dict, background) of a parity scene."""
    if name in BUILT:
        return _built(name, width)
    return fixture(name), sd.fixture_camera(name, width), BG[name]


def oracle_render(name, width, variant, window, s_begin, s_count, seed=0, max_depth=50, threads=0, acc=None,
                  traversal='stack'):
    import oracle
    sa, cam, bg = scene_inputs(name, width)
    W, H = cam['width'], cam['height']
    fr = oracle.make_frame(cam, bg, max_depth, seed, W, H, traversal)
    if acc is None:
        acc = np.zeros((H, W, 3), np.float32)
    stats = oracle.render(oracle.OracleScene(sa), fr, variant, acc, window, s_begin, s_count, threads)
    return acc, stats


def gpu_render(name, width, variant, window, s_begin, s_count, seed=0, max_depth=50, band=(1, 1, 0),
               chunks=None, integ=None, traversal='stack'):
    import torch
    from ptmi import device
    sa, cam, bg = scene_inputs(name, width)
    W, H = cam['width'], cam['height']
    if integ is None:
        integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, max_depth, seed, W, H, window, band, traversal=traversal)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    chunks = chunks or [(s_begin, s_count)]
    for b, c in chunks:
        (integ.render_mk if variant == 'mk' else integ.render_wf)(fr, acc, b, c)
    torch.cuda.synchronize()
    return acc.cpu().numpy(), integ.read_counters(), integ


def compare(a, b, spp):
    """Per-pixel L-inf of accum/spp, NaN == NaN; returns (linf, exact_fraction)."""
    x = a / np.float32(spp)
    y = b / np.float32(spp)
    both_nan = np.isnan(x) & np.isnan(y)
    d = np.where(both_nan, 0.0, np.abs(x.astype(np.float64) - y.astype(np.float64)))
    d = np.where(np.isnan(d), np.inf, d)
    exact = np.mean(np.all((a == b) | (np.isnan(a) & np.isnan(b)), axis=-1))
    return float(d.max()) if d.size else 0.0, float(exact)
