"""ctypes binding of libptmi.so (the C-ABI declared in include/ptmi.h).

The library is built in-tree (``make -C path-tracer-python_amd/csrc`` or
``__graft_entry__.build()``) and loaded from ``ptmi/_lib/libptmi.so``. There is
no fallback: if the library is missing every render entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('PTMI_LIB') or os.path.join(_HERE, '_lib', 'libptmi.so')  # PTMI_LIB: A/B builds
ABI_VERSION = 7  # PTMI_ABI_VERSION of include/ptmi.h
MAX_IMAGES = 16
NUM_COUNTERS = 6
COUNTER_TAIL_SEGMENTS = 5  # wavefront segments traced in the tail launch (wf_drain), part of [0]

PTMI_OK, PTMI_EINVAL, PTMI_ECAPACITY, PTMI_EHIP, PTMI_ENODEV = 0, -1, -2, -3, -4

f3 = C.c_float * 3


class SceneView(C.Structure):
    _fields_ = [
        ('nodes', C.c_void_p), ('n_inner', C.c_int32), ('root_ref', C.c_int32),
        ('root_min', f3), ('root_max', f3), ('max_leaf_depth', C.c_int32),
        ('spheres', C.c_void_p), ('quads', C.c_void_p), ('tris', C.c_void_p), ('mats', C.c_void_p),
        ('num_spheres', C.c_int32), ('num_quads', C.c_int32), ('num_triangles', C.c_int32),
        ('texels', C.c_void_p), ('num_images', C.c_int32),
        ('img_offset', C.c_int32 * MAX_IMAGES), ('img_w', C.c_int32 * MAX_IMAGES),
        ('img_h', C.c_int32 * MAX_IMAGES),
        ('perlin_vec', C.c_void_p), ('perlin_perm', C.c_void_p),
        ('ref_nodes', C.c_void_p), ('num_bvh_nodes', C.c_int32),
    ]


class Camera(C.Structure):
    _fields_ = [('center', f3), ('pixel00', f3), ('delta_u', f3), ('delta_v', f3),
                ('defocus_u', f3), ('defocus_v', f3), ('defocus_angle', C.c_float)]


class Frame(C.Structure):
    _fields_ = [('cam', Camera), ('bg', f3), ('max_depth', C.c_int32), ('seed', C.c_uint32),
                ('width', C.c_int32), ('height', C.c_int32),
                ('x0', C.c_int32), ('y0', C.c_int32), ('w', C.c_int32), ('h', C.c_int32),
                ('band_rows', C.c_int32), ('band_stride', C.c_int32), ('band_offset', C.c_int32),
                ('traversal', C.c_int32)]


# BVH traversal of a frame (ptmi_frame.traversal): the reference's
# traverse_bvh_legacy (default) or traverse_bvh_stackless, switched in the
# reference by USE_STACKLESS_TRAVERSAL (kernels.py:746)
TRAVERSALS = {'stack': 0, 'stackless': 1}


EXPORTS = ('ptmi_version', 'ptmi_last_error', 'ptmi_scene_check', 'ptmi_mk_render', 'ptmi_mk_workspace_bytes',
           'ptmi_mk_render_ws', 'ptmi_mk_trace_ws', 'ptmi_mk_max_batch', 'ptmi_mk_resolve_ws', 'ptmi_wf_workspace_bytes',
           'ptmi_wf_render', 'ptmi_clear', 'ptmi_tonemap', 'ptmi_bvh_build_sah', 'ptmi_prof_start',
           'ptmi_prof_stop', 'ptmi_prof_stop_busy', 'ptmi_node_bytes', 'ptmi_wf_set_drain_at')
PROF_KINDS = ('megakernel', 'wf_generate', 'wf_intersect', 'wf_drain', 'wf_scatter', 'wf_resolve', 'mk_resolve')

_lib = None


class PtmiError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libptmi.so once; raises PtmiError (no silent fallback) if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise PtmiError(f'libptmi.so not built ({path}); run `make -C path-tracer-python_amd/csrc` '
                        'or __graft_entry__.build()')
    # One HIP runtime per process: torch's wheel carries its own libamdhip64
    # (soname libamdhip64.so.7, the same as /opt/rocm's). Loaded after torch,
    # libptmi binds to that copy; loaded first, it pulls in /opt/rocm's and
    # torch then maps a second runtime, under which ptmi's launches find no
    # device. So torch goes first whenever it is importable (the scene
    # compiler reaches this loader for the native SAH builder before any
    # device code runs).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    P = C.c_void_p
    lib.ptmi_version.restype = C.c_int
    lib.ptmi_node_bytes.restype = C.c_int
    lib.ptmi_last_error.restype = C.c_char_p
    lib.ptmi_scene_check.argtypes = [C.POINTER(SceneView)]
    lib.ptmi_mk_render.argtypes = [C.POINTER(SceneView), C.POINTER(Frame), P, C.c_int32, C.c_int32, P, P]
    lib.ptmi_mk_workspace_bytes.argtypes = [C.POINTER(Frame), C.c_int32]
    lib.ptmi_mk_workspace_bytes.restype = C.c_size_t
    lib.ptmi_mk_max_batch.argtypes = [C.POINTER(Frame)]
    lib.ptmi_mk_max_batch.restype = C.c_int64
    lib.ptmi_mk_render_ws.argtypes = [C.POINTER(SceneView), C.POINTER(Frame), P, C.c_size_t, P, C.c_int32,
                                      C.c_int32, P, P]
    lib.ptmi_mk_trace_ws.argtypes = [C.POINTER(SceneView), C.POINTER(Frame), P, C.c_size_t, C.c_int32, C.c_int32,
                                     P, P]
    lib.ptmi_mk_resolve_ws.argtypes = [C.POINTER(Frame), P, C.c_size_t, P, C.c_int32, P]
    lib.ptmi_wf_workspace_bytes.argtypes = [C.POINTER(Frame), C.c_int32]
    lib.ptmi_wf_workspace_bytes.restype = C.c_size_t
    lib.ptmi_wf_render.argtypes = [C.POINTER(SceneView), C.POINTER(Frame), P, C.c_size_t, P, C.c_int32,
                                   C.c_int32, P, P]
    lib.ptmi_wf_set_drain_at.argtypes = [C.c_int32]
    lib.ptmi_clear.argtypes = [C.POINTER(Frame), P, P]
    lib.ptmi_tonemap.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, P]
    lib.ptmi_bvh_build_sah.argtypes = [P, C.c_int32, P, C.c_int32, P, C.c_int32, P, P, P, P, P, P, P,
                                       C.POINTER(C.c_int32)]
    lib.ptmi_prof_start.argtypes = [C.c_int32]
    lib.ptmi_prof_stop.argtypes = [P, P, C.c_int32]
    lib.ptmi_prof_stop_busy.argtypes = [P, P, P, C.c_int32]
    if lib.ptmi_version() != ABI_VERSION:
        raise PtmiError(f'libptmi ABI version {lib.ptmi_version()} != {ABI_VERSION} (rebuild libptmi.so)')
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != PTMI_OK:
        msg = load().ptmi_last_error().decode(errors='replace')
        raise PtmiError(f'{what} failed ({rc}): {msg}')
    return rc


class KernelTimer:
    """Per-kernel device time of libptmi's own launches (ptmi_prof_start/stop)."""

    def __init__(self, max_launches=200000):
        self.max_launches = int(max_launches)

    def __enter__(self):
        check(load().ptmi_prof_start(self.max_launches), 'ptmi_prof_start')
        self.result = None
        return self

    def __exit__(self, *exc):
        import numpy as np
        ms = np.zeros(len(PROF_KINDS), np.float64)
        busy = np.zeros(len(PROF_KINDS), np.float64)
        n = np.zeros(len(PROF_KINDS), np.uint64)
        rc = load().ptmi_prof_stop_busy(C.c_void_p(ms.ctypes.data), C.c_void_p(busy.ctypes.data),
                                        C.c_void_p(n.ctypes.data), len(PROF_KINDS))
        self.truncated = rc == PTMI_ECAPACITY  # more launches than events: totals cover the first ones
        if not self.truncated:
            check(rc, 'ptmi_prof_stop_busy')
        # ms: summed launch durations; busy_ms: union of the launches' intervals
        self.result = {k: {'ms': float(ms[i]), 'busy_ms': float(busy[i]), 'launches': int(n[i])}
                       for i, k in enumerate(PROF_KINDS)}
        return False
