"""Device residency of a packed scene and thin wrappers over the C-ABI.

PyTorch is used only as the device allocator / stream provider: every array
of the packed layout (scene_data.DeviceLayout) becomes one torch tensor on
the GPU and the C-ABI receives raw pointers (include/ptmi.h). This replaces
the reference's module-global Taichi fields (fields.py) with a per-device
object, so several scenes can coexist in one process.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from .scene_data import DeviceLayout, SceneArrays, camera_upload, pack_device


def _stream_ptr(stream=None, device=None):
    if stream is None:
        stream = torch.cuda.current_stream(device)
    elif device is not None and stream.device != device:
        raise _lib.PtmiError(f'stream is on {stream.device}, the scene on {device}')
    return C.c_void_p(stream.cuda_stream)


def require_gpu():
    if not torch.cuda.is_available():
        raise _lib.PtmiError('no GPU visible: the MI355X integrator has no CPU fallback')
    _lib.load()


class DeviceScene:
    """A packed scene resident in HBM plus its ptmi_scene_view."""

    def __init__(self, scene, device=None):
        require_gpu()
        node_bytes = int(_lib.load().ptmi_node_bytes())
        # PTMI_PACK_LEAF_ORDER=0: compile-order primitives (A/B timing only: same results)
        leaf_order = os.environ.get('PTMI_PACK_LEAF_ORDER', '1') != '0'
        layout = scene if isinstance(scene, DeviceLayout) else pack_device(scene, node_bytes, leaf_order)
        if layout.n_inner and layout.nodes.shape[1] * 4 != node_bytes:
            raise _lib.PtmiError(f'scene packed with {layout.nodes.shape[1] * 4}-B nodes, '
                                 f'libptmi expects {node_bytes}')
        self.layout = layout
        dev = torch.device(device if device is not None else 'cuda')
        if dev.type != 'cuda':
            raise _lib.PtmiError(f'DeviceScene needs a cuda device, got {dev}')
        # a bare 'cuda' means the current device; fixed here so every later
        # launch goes to the device that holds the scene (the C-ABI launches on
        # the current HIP device)
        self.device = torch.device('cuda', dev.index if dev.index is not None else torch.cuda.current_device())

        def up(a):
            a = np.ascontiguousarray(a)
            if a.size == 0:
                a = np.zeros(4, dtype=a.dtype)  # keep a valid 16-B aligned pointer
            return torch.from_numpy(a.reshape(-1).copy()).to(self.device)

        self.t_nodes = up(layout.nodes)
        self.t_spheres = up(layout.spheres)
        self.t_quads = up(layout.quads)
        self.t_tris = up(layout.tris)
        self.t_mats = up(layout.mats)
        self.t_texels = up(layout.texels.view(np.int32))
        self.t_pvec = up(layout.perlin_vec)
        self.t_perm = up(layout.perlin_perm)
        self.t_ref_nodes = up(layout.ref_nodes) if layout.ref_nodes is not None else None
        v = _lib.SceneView()
        v.nodes = self.t_nodes.data_ptr()
        v.n_inner = layout.n_inner
        v.root_ref = layout.root_ref
        for k in range(3):
            v.root_min[k] = float(layout.root_min[k])
            v.root_max[k] = float(layout.root_max[k])
        v.max_leaf_depth = layout.max_leaf_depth
        v.spheres = self.t_spheres.data_ptr()
        v.quads = self.t_quads.data_ptr()
        v.tris = self.t_tris.data_ptr()
        v.mats = self.t_mats.data_ptr()
        v.num_spheres, v.num_quads, v.num_triangles = layout.num_spheres, layout.num_quads, layout.num_triangles
        v.texels = self.t_texels.data_ptr()
        v.num_images = len(layout.img_w)
        for k in range(len(layout.img_w)):
            v.img_offset[k] = layout.img_offset[k]
            v.img_w[k] = layout.img_w[k]
            v.img_h[k] = layout.img_h[k]
        v.perlin_vec = self.t_pvec.data_ptr()
        v.perlin_perm = self.t_perm.data_ptr()
        if self.t_ref_nodes is not None:
            v.ref_nodes = self.t_ref_nodes.data_ptr()
        v.num_bvh_nodes = layout.num_bvh_nodes if layout.ref_nodes is not None else \
            (2 * (layout.n_inner + 1) - 1 if layout.num_spheres + layout.num_quads + layout.num_triangles else 0)
        self.view = v
        _lib.check(_lib.load().ptmi_scene_check(C.byref(v)), 'ptmi_scene_check')

    @classmethod
    def from_arrays(cls, sa: SceneArrays, device=None):
        return cls(sa, device)


def make_frame(cam, bg, max_depth, seed, width, height, window=None, band=(1, 1, 0), traversal='stack'):
    """ptmi_frame from camera upload values (dict of f32 3-vectors or an
    object with the reference camera's attributes). ``traversal``: 'stack'
    (traverse_bvh_legacy, the reference's default) or 'stackless'
    (traverse_bvh_stackless, its USE_STACKLESS_TRAVERSAL = True)."""
    f = _lib.Frame()
    if traversal not in _lib.TRAVERSALS:
        raise _lib.PtmiError(f'unknown traversal {traversal!r} (one of {sorted(_lib.TRAVERSALS)})')
    f.traversal = _lib.TRAVERSALS[traversal]
    vals = cam if isinstance(cam, dict) else camera_upload(cam)
    get = vals.__getitem__
    for k, fld in (('center', 'center'), ('pixel00', 'pixel00'), ('delta_u', 'delta_u'), ('delta_v', 'delta_v'),
                   ('defocus_u', 'defocus_u'), ('defocus_v', 'defocus_v')):
        arr = np.asarray(get(k), np.float32)
        for i in range(3):
            getattr(f.cam, fld)[i] = float(arr[i])
    f.cam.defocus_angle = float(np.float32(get('defocus_angle')))
    bgv = np.asarray([bg.x, bg.y, bg.z] if hasattr(bg, 'x') else bg, np.float64).astype(np.float32)
    for i in range(3):
        f.bg[i] = float(bgv[i])
    f.max_depth = int(max_depth)
    f.seed = int(seed) & 0xffffffff
    f.width, f.height = int(width), int(height)
    x0, y0, w, h = window if window is not None else (0, 0, width, height)
    f.x0, f.y0, f.w, f.h = int(x0), int(y0), int(w), int(h)
    f.band_rows, f.band_stride, f.band_offset = (int(b) for b in band)
    return f


def frame_pixel_rows(frame):
    """Image rows owned by a frame (window + band filter), as the kernels see them."""
    rows = [frame.y0 + r for r in range(frame.h)
            if (r // frame.band_rows) % frame.band_stride == frame.band_offset]
    return np.asarray(rows, np.int64)


class Integrator:
    """Launch wrapper: megakernel / wavefront / clear / tonemap on one stream."""

    def __init__(self, dscene: DeviceScene, with_counters=True):
        self.scene = dscene
        self.lib = _lib.load()
        self.counters = torch.zeros(_lib.NUM_COUNTERS, dtype=torch.int64, device=dscene.device) \
            if with_counters else None
        self._ws = None
        self._ws_bytes = 0
        self._reset_event = None  # counter reset the next overlapped trace must wait for

    def _cnt(self):
        return C.c_void_p(self.counters.data_ptr()) if self.counters is not None else None

    def _dev(self):
        """Context that makes the scene's device current for a C-ABI call."""
        return torch.cuda.device(self.scene.device)

    def _stream(self, stream):
        return _stream_ptr(stream, self.scene.device)

    # multi-sample megakernel calls run as (tile, sample chunk) work units with
    # staged colours (ptmi_mk_render_ws); single samples accumulate directly
    MK_STAGED_MIN_SAMPLES = 2

    def render_mk(self, frame, accum, sample_begin, sample_count, stream=None, staged=None, overlap=False):
        """Megakernel render of samples [sample_begin, sample_begin + sample_count)
        added into accum in sample order. overlap=True: consecutive calls
        pipeline (see render_mk_overlapped)."""
        _check_accum(accum, frame, self.scene.device)
        if overlap:
            return self.render_mk_overlapped(frame, accum, sample_begin, sample_count, stream)
        if staged is None:
            staged = int(sample_count) >= self.MK_STAGED_MIN_SAMPLES
        with self._dev():
            if staged:
                ws = self.workspace(frame, sample_count, 'mk')
                _lib.check(self.lib.ptmi_mk_render_ws(C.byref(self.scene.view), C.byref(frame),
                                                      C.c_void_p(ws.data_ptr()), self._ws_bytes,
                                                      C.c_void_p(accum.data_ptr()), int(sample_begin),
                                                      int(sample_count), self._cnt(), self._stream(stream)),
                           'ptmi_mk_render_ws')
                return
            _lib.check(self.lib.ptmi_mk_render(C.byref(self.scene.view), C.byref(frame),
                                               C.c_void_p(accum.data_ptr()), int(sample_begin), int(sample_count),
                                               self._cnt(), self._stream(stream)),
                       'ptmi_mk_render')

    # Staging budget for the per-(sample, pixel) colour slots of one batch:
    # 2 GiB keeps a whole 16-spp 4K call (1.6 GB) in one batch. A/B on MI355X
    # (PTMI_STAGING_BYTES, A/B only): C5 3757 (1 GiB: 10 + 6 spp batches) ->
    # 3788 Msamples/s, C2 unchanged, 4 GiB no further change
    # (profiles/r03/ab/ab_staging_bytes.log).
    STAGING_BYTES = int(os.environ.get('PTMI_STAGING_BYTES', str(2 << 30)))
    # Overlapped megakernel calls: traces in flight, one workspace and side
    # stream each. Round 3 measured two in flight for whole-frame calls and
    # three for small calls (vol2 800x800, 64 spp per call: the full frame,
    # 41 M samples per call, 2851 (2) vs 2762 (3) Msamples/s; an 8-GPU tile
    # shard, 5.1 M samples per call, 2380-2487 (2) vs 2450-2565 (3); 4 slower
    # than both; profiles/r03/overlap_depth_and_bands.log). Since draining
    # waves traverse at the lowest priority (pt_megakernel.hip,
    # PTMI_MK_PRIO_DRAIN) three are as fast on whole frames too: C2 3314 vs
    # 3312, C5 4306 vs 4314, C4 1786 vs 1760; the shard 3085 (3) vs 2985 (2)
    # vs 3092 (4) (profiles/r05/overlap_depth_r05.log), so three always.
    # PTMI_OVERLAP_DEPTH fixes the depth (A/B only).
    OVERLAP_DEPTH_MAX = 3

    def render_mk_overlapped(self, frame, accum, sample_begin, sample_count, stream=None):
        """Megakernel calls whose launches overlap: each batch is traced
        (ptmi_mk_trace_ws) on one of two side streams into one of two
        workspaces, alternately, and resolved (ptmi_mk_resolve_ws) on the
        caller's stream in call order, so the next call's megakernel fills
        the chip while the previous one's last long paths drain (~1.5 ms of a
        17-ms vol2 launch otherwise leaves most of the chip idle). Results
        are bit-identical to render_mk: the resolves add the same staged
        colours in the same sample order.

        Ordering, whatever stream each call passes:
        * a trace into workspace half h waits for the resolve that last read
          half h (an event recorded on the stream that ran that resolve), and
          for every counter reset issued before it (reset_counters makes
          every side stream wait on its event; the reset and read_counters in
          turn wait for the traces still adding to the counters, whatever
          stream they run on);
        * a resolve waits for its own trace and for the previous resolve, so
          the accumulator sees the batches in call order;
        * a trace does not wait for other work the caller queued after the
          previous call: the scene must not change between overlapped calls,
          and work on the caller's stream after this call sees the resolved
          accumulator as usual."""
        import torch
        dev = self.scene.device
        caller = stream if stream is not None else torch.cuda.current_stream(dev)
        npix = frame.w * len(frame_pixel_rows(frame))
        if npix == 0 or sample_count <= 0:
            return
        max_batch = int(self.lib.ptmi_mk_max_batch(C.byref(frame)))
        if max_batch < 1:
            _lib.check(-1, 'ptmi_mk_max_batch')
        per = max(1, min(int(sample_count), self.STAGING_BYTES // max(1, 12 * npix), max_batch))
        with self._dev():
            if getattr(self, '_ov', None) is None:
                D = self.OVERLAP_DEPTH_MAX
                self._ov = {'streams': [torch.cuda.Stream(dev) for _ in range(D)], 'ws': [None] * D,
                            'k': 0, 'resolved': [None] * D, 'last_resolved': None, 'traced': [None] * D}
                if self._reset_event is not None:  # a reset issued before the side streams existed
                    for side in self._ov['streams']:
                        side.wait_event(self._reset_event)
            ov = self._ov
            depth = int(os.environ.get('PTMI_OVERLAP_DEPTH', '0')) or self.OVERLAP_DEPTH_MAX
            depth = max(1, min(depth, len(ov['ws'])))
            b = 0
            while b < sample_count:
                n = min(per, int(sample_count) - b)
                h = ov['k'] % depth  # any rotation is safe: each half waits for its own last reader
                ov['k'] += 1
                need = int(self.lib.ptmi_mk_workspace_bytes(C.byref(frame), n))
                if need == 0:
                    _lib.check(-1, 'ptmi_mk_workspace_bytes')
                side = ov['streams'][h]
                ws = ov['ws'][h]
                if ws is None or ws.numel() * 4 < need:
                    torch.cuda.synchronize(dev)  # the old half may still be read by a trace or a resolve
                    ws = torch.empty((need + 15) // 16 * 4, dtype=torch.float32, device=dev)
                    ov['ws'][h] = ws
                    fresh = torch.cuda.Event()
                    fresh.record(torch.cuda.current_stream(dev))  # the allocation's stream
                    side.wait_event(fresh)
                if ov['resolved'][h] is not None:
                    side.wait_event(ov['resolved'][h])
                _lib.check(self.lib.ptmi_mk_trace_ws(C.byref(self.scene.view), C.byref(frame),
                                                     C.c_void_p(ws.data_ptr()), ws.numel() * 4,
                                                     int(sample_begin) + b, n, self._cnt(),
                                                     C.c_void_p(side.cuda_stream)), 'ptmi_mk_trace_ws')
                traced = torch.cuda.Event()
                traced.record(side)
                ov['traced'][h] = traced
                caller.wait_event(traced)
                if ov['last_resolved'] is not None:
                    caller.wait_event(ov['last_resolved'])
                _lib.check(self.lib.ptmi_mk_resolve_ws(C.byref(frame), C.c_void_p(ws.data_ptr()), ws.numel() * 4,
                                                       C.c_void_p(accum.data_ptr()), n,
                                                       C.c_void_p(caller.cuda_stream)), 'ptmi_mk_resolve_ws')
                done = torch.cuda.Event()
                done.record(caller)
                ov['resolved'][h] = done
                ov['last_resolved'] = done
                b += n

    def workspace(self, frame, sample_count=1, kind='wf'):
        """Cached device workspace (torch) big enough for one batch of the call
        (shared by the megakernel's staged mode and the wavefront)."""
        npix = frame.w * len(frame_pixel_rows(frame))
        batch = max(1, min(int(sample_count), self.STAGING_BYTES // max(1, 12 * npix)))
        fn = self.lib.ptmi_wf_workspace_bytes if kind == 'wf' else self.lib.ptmi_mk_workspace_bytes
        need = int(fn(C.byref(frame), batch))
        if need == 0:
            _lib.check(-1, f'ptmi_{kind}_workspace_bytes')
        if self._ws is None or self._ws_bytes < need:
            self._ws = None
            self._ws = torch.empty((need + 15) // 16 * 4, dtype=torch.float32, device=self.scene.device)
            self._ws_bytes = self._ws.numel() * 4
        return self._ws

    def render_wf(self, frame, accum, sample_begin, sample_count, stream=None):
        _check_accum(accum, frame, self.scene.device)
        with self._dev():
            ws = self.workspace(frame, sample_count)
            _lib.check(self.lib.ptmi_wf_render(C.byref(self.scene.view), C.byref(frame), C.c_void_p(ws.data_ptr()),
                                               self._ws_bytes, C.c_void_p(accum.data_ptr()), int(sample_begin),
                                               int(sample_count), self._cnt(), self._stream(stream)),
                       'ptmi_wf_render')

    def clear(self, frame, accum, stream=None):
        _check_accum(accum, frame, self.scene.device)
        with self._dev():
            _lib.check(self.lib.ptmi_clear(C.byref(frame), C.c_void_p(accum.data_ptr()), self._stream(stream)),
                       'ptmi_clear')

    def tonemap(self, accum, spp, stream=None):
        if accum.device != self.scene.device:
            raise _lib.PtmiError(f'accum is on {accum.device}, the scene on {self.scene.device}')
        h, w, _ = accum.shape
        with self._dev():
            out = torch.empty((h, w, 3), dtype=torch.uint8, device=accum.device)
            _lib.check(self.lib.ptmi_tonemap(C.c_void_p(accum.data_ptr()), C.c_void_p(out.data_ptr()), w, h,
                                             int(spp), self._stream(stream)), 'ptmi_tonemap')
        return out

    def _after_traces(self, stream):
        """Make `stream` wait for the overlapped traces in flight: they add to
        the counters from their side streams."""
        ov = getattr(self, '_ov', None)
        if ov is not None:
            for ev in ov['traced']:
                if ev is not None:
                    stream.wait_event(ev)

    def read_counters(self):
        if self.counters is None:
            return None
        self._after_traces(torch.cuda.current_stream(self.scene.device))
        c = self.counters.cpu().numpy()
        return {'segments': int(c[0]), 'medium': int(c[1]), 'paths': int(c[2]), 'rr': int(c[3]),
                'depth_cap': int(c[4])}

    def tail_segments(self):
        """Segments the wavefront traced in its one-launch tail (wf_drain):
        part of read_counters()['segments'], counted apart so per-kernel
        rates attribute them to the launch that traced them."""
        if self.counters is None:
            return None
        self._after_traces(torch.cuda.current_stream(self.scene.device))
        return int(self.counters[_lib.COUNTER_TAIL_SEGMENTS].item())

    def reset_counters(self, stream=None):
        if self.counters is not None:
            s = stream if stream is not None else torch.cuda.current_stream(self.scene.device)
            self._after_traces(s)
            with torch.cuda.stream(s):
                self.counters.zero_()
            # overlapped traces run on side streams: every later trace, on any of
            # them, waits for this reset (a multi-batch call rotates through the
            # side streams, so waiting on the first one only is not enough)
            ev = torch.cuda.Event()
            ev.record(s)
            ov = getattr(self, '_ov', None)
            if ov is not None:
                for side in ov['streams']:
                    side.wait_event(ev)
            self._reset_event = ev  # side streams created after this reset wait on it too


def _check_accum(accum, frame, device=None):
    if not (isinstance(accum, torch.Tensor) and accum.is_cuda and accum.dtype == torch.float32
            and accum.is_contiguous() and tuple(accum.shape) == (frame.height, frame.width, 3)):
        raise _lib.PtmiError(f'accum must be a contiguous cuda float32 tensor of shape '
                             f'({frame.height}, {frame.width}, 3)')
    if device is not None and accum.device != device:
        raise _lib.PtmiError(f'accum is on {accum.device}, the scene on {device}')
