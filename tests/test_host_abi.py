"""CPU tests of the host side: the C-ABI library loads and exports every
symbol include/ptmi.h declares, validates its arguments without a GPU, and
the frame / shard bookkeeping partitions pixels and samples exactly."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from ptmi import _lib, device
from ptmi.distributed import Shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, 'include', 'ptmi.h')) as f:
        txt = f.read()
    return sorted(set(re.findall(r'\b(ptmi_[a-z_0-9]+)\s*\(', txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert set(syms) == set(_lib.EXPORTS)
    for s in syms:
        assert hasattr(lib, s), s
    with open(os.path.join(ROOT, 'include', 'ptmi.h')) as f:
        ver = int(re.search(r'#define PTMI_ABI_VERSION (\d+)', f.read()).group(1))
    assert lib.ptmi_version() == ver == _lib.ABI_VERSION


def test_struct_layouts_match_header():
    # offsets the C side sees (x86-64 SysV): spot-check the ctypes mirrors
    assert C.sizeof(_lib.Camera) == 19 * 4
    assert _lib.Frame.band_offset.offset == C.sizeof(_lib.Camera) + 4 * (3 + 1 + 1 + 2 + 4 + 2)
    assert _lib.SceneView.perlin_perm.offset > _lib.SceneView.img_h.offset
    # ABI v5 additions sit at the ends of both structs
    assert _lib.Frame.traversal.offset == _lib.Frame.band_offset.offset + 4
    assert _lib.SceneView.num_bvh_nodes.offset == _lib.SceneView.ref_nodes.offset + 8
    assert C.sizeof(_lib.SceneView) == _lib.SceneView.num_bvh_nodes.offset + 8  # padded to 8


def make_frame(**kw):
    cam = {k: np.zeros(3, np.float32) for k in ('center', 'pixel00', 'delta_u', 'delta_v', 'defocus_u', 'defocus_v')}
    cam['defocus_angle'] = 0.0
    args = dict(cam=cam, bg=(0, 0, 0), max_depth=50, seed=0, width=16, height=8)
    args.update(kw)
    return device.make_frame(**args)


@pytest.mark.parametrize('kw,msg', [
    (dict(window=(0, 0, 17, 8)), 'bad window'),
    (dict(window=(4, 4, 4, 5)), 'bad window'),
    (dict(band=(0, 1, 0)), 'band'),
    (dict(band=(2, 2, 2)), 'band'),
    (dict(max_depth=300), 'max_depth'),
])
def test_frame_validation_errors(kw, msg):
    lib = _lib.load()
    f = make_frame(**kw)
    rc = lib.ptmi_clear(C.byref(f), C.c_void_p(16), None)
    assert rc == _lib.PTMI_EINVAL
    assert msg in lib.ptmi_last_error().decode()


def test_unknown_traversal_is_rejected():
    lib = _lib.load()
    f = make_frame()
    f.traversal = 2
    assert lib.ptmi_clear(C.byref(f), C.c_void_p(16), None) == _lib.PTMI_EINVAL
    assert 'traversal' in lib.ptmi_last_error().decode()
    with pytest.raises(_lib.PtmiError):
        make_frame(traversal='restart-trail')
    assert make_frame(traversal='stackless').traversal == 1 and make_frame().traversal == 0


def test_scene_validation_errors():
    lib = _lib.load()
    v = _lib.SceneView()
    v.num_spheres = 3
    v.n_inner = 1  # needs prims - 1 = 2
    rc = lib.ptmi_scene_check(C.byref(v))
    assert rc == _lib.PTMI_EINVAL and 'n_inner' in lib.ptmi_last_error().decode()
    v.n_inner = 2
    v.max_leaf_depth = 63
    v.nodes = v.spheres = v.mats = v.perlin_vec = v.perlin_perm = 16
    v.num_bvh_nodes = 5
    # leaf depth > 62 runs the reference's own 64-entry stack walk (its silent
    # drops, kernels.py:719-740) on the reference-layout nodes: they must be bound
    assert lib.ptmi_scene_check(C.byref(v)) == _lib.PTMI_EINVAL
    assert 'ref_nodes' in lib.ptmi_last_error().decode()
    v.ref_nodes = 32
    assert lib.ptmi_scene_check(C.byref(v)) == _lib.PTMI_OK
    v.ref_nodes = None
    v.max_leaf_depth = 2
    v.num_bvh_nodes = 4  # 3 primitives: 2N - 1 = 5 nodes
    assert lib.ptmi_scene_check(C.byref(v)) == _lib.PTMI_EINVAL
    assert 'num_bvh_nodes' in lib.ptmi_last_error().decode()
    v.num_bvh_nodes = 5
    v.ref_nodes = 24  # not 16-byte aligned
    assert lib.ptmi_scene_check(C.byref(v)) == _lib.PTMI_EINVAL
    v.ref_nodes = None  # optional: only the stackless traversal reads it
    assert lib.ptmi_scene_check(C.byref(v)) == _lib.PTMI_OK


def test_render_rejects_bad_arguments_before_touching_device():
    lib = _lib.load()
    f = make_frame()
    v = _lib.SceneView()
    v.perlin_vec = v.perlin_perm = 16
    rc = lib.ptmi_mk_render(C.byref(v), C.byref(f), None, 0, 1, None, None)
    assert rc == _lib.PTMI_EINVAL and 'accum' in lib.ptmi_last_error().decode()
    rc = lib.ptmi_wf_render(C.byref(v), C.byref(f), None, 0, C.c_void_p(16), 0, 1, None, None)
    assert rc == _lib.PTMI_EINVAL and 'workspace' in lib.ptmi_last_error().decode()
    assert lib.ptmi_wf_workspace_bytes(C.byref(f), 1) >= 16 * 8 * (108 + 12)
    assert lib.ptmi_wf_workspace_bytes(C.byref(f), 4) - lib.ptmi_wf_workspace_bytes(C.byref(f), 1) >= 3 * 16 * 8 * 12
    assert lib.ptmi_wf_workspace_bytes(C.byref(f), 0) == 0
    # staged megakernel: workspace = 12 B per (sample, pixel), 256-B rounded
    rc = lib.ptmi_mk_render_ws(C.byref(v), C.byref(f), None, 0, C.c_void_p(16), 0, 2, None, None)
    assert rc == _lib.PTMI_EINVAL and 'workspace' in lib.ptmi_last_error().decode()
    rc = lib.ptmi_mk_render_ws(C.byref(v), C.byref(f), C.c_void_p(256), 64, C.c_void_p(16), 0, 2, None, None)
    assert rc == _lib.PTMI_EINVAL and 'workspace' in lib.ptmi_last_error().decode()
    rc = lib.ptmi_mk_render_ws(C.byref(v), C.byref(f), C.c_void_p(256), 1 << 20, None, 0, 2, None, None)
    assert rc == _lib.PTMI_EINVAL and 'accum' in lib.ptmi_last_error().decode()
    assert lib.ptmi_mk_workspace_bytes(C.byref(f), 1) == 16 * 8 * 12 + (-(16 * 8 * 12) % 256) + 2048  # + 8 counter lines
    assert lib.ptmi_mk_workspace_bytes(C.byref(f), 10) == 16 * 8 * 12 * 10 + 2048
    assert lib.ptmi_mk_workspace_bytes(C.byref(f), 0) == 0


def test_device_entry_points_fail_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(_lib.PtmiError):
        device.require_gpu()


@pytest.mark.parametrize('h,band_rows,world', [(800, 8, 2), (800, 8, 3), (225, 8, 8), (37, 4, 5), (10, 16, 4)])
def test_tile_bands_partition_rows(h, band_rows, world):
    rows = []
    for r in range(world):
        sh = Shard(r, world, 'tiles', band_rows)
        f = make_frame(height=h, band=sh.band())
        got = device.frame_pixel_rows(f).tolist()
        assert got == sh.rows(h)
        rows += got
    assert sorted(rows) == list(range(h))


@pytest.mark.parametrize('h,band_rows,world', [(800, 4, 8), (800, 8, 3), (225, 8, 8), (37, 4, 5), (2160, 8, 8)])
def test_library_counts_the_same_band_rows(h, band_rows, world):
    """The library's row count for a banded frame (seen through the staged
    workspace size, no GPU needed) is the Python partition's."""
    lib = _lib.load()
    for r in range(world):
        sh = Shard(r, world, 'tiles', band_rows)
        f = make_frame(height=h, band=sh.band())
        npix = f.w * len(sh.rows(h))
        assert lib.ptmi_mk_workspace_bytes(C.byref(f), 4) == (npix * 48 + 255) // 256 * 256 + 2048


def test_sample_shards_are_disjoint_and_complete():
    world, steps, sps = 4, 5, 3
    seen = []
    for r in range(world):
        sh = Shard(r, world, 'samples')
        for k in range(steps):
            b, c = sh.sample_range(k, sps)
            seen += list(range(b, b + c))
    assert sorted(seen) == list(range(world * steps * sps))


def test_tonemap_scale_matches_numpy_promotion():
    # preview.py:129: scale = 1.0 / max(1, spp) is a Python float; NEP 50 casts it to f32
    for spp in (1, 3, 7, 1000, 1024):
        assert np.float32(1.0 / spp) == (np.ones(1, np.float32) * (1.0 / spp))[0]
