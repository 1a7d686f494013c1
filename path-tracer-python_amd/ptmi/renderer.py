"""MI355X renderer with the reference's TaichiRenderer surface.

Mirrors src/render_server/taichi_renderer/renderer.py:25-648 — constructor
``(world, cam, img_path)``, ``max_depth`` / ``background_color`` attributes
picked up at render time, ``render()`` (megakernel), ``render_wavefront()``,
the InteractiveViewer compatibility API (``render_sample``,
``clear_accumulation_buffer``, ``_upload_camera_to_gpu``, ``write_image``,
``print_statistics``, ``num_spheres``, ``num_bvh_nodes``, ``timing``,
``sample_times``, ``current_sample``) — on the HIP integrator of libptmi.

Differences by design: no Taichi JIT (``timing['taichi_init']`` stays 0),
scene arrays sized dynamically (no MAX_* capacities), each
renderer owns its device buffers (the reference's are module globals), the
random stream is keyed by (seed, pixel, sample) so ``render_sample(i)``
renders sample i deterministically, and the preview window is not opened
(Tk GUI is out of scope): ``enable_preview`` is accepted and ignored.

Checkpoint / resume (the reference has none: its progressive accumulation
lives only in accum_buffer, renderer.py:405-442):
``save_checkpoint(path)`` writes the accumulator, the next sample index and
the render state; ``load_checkpoint(path)`` followed by ``render(resume=True)``
finishes the remaining samples. Samples are keyed by (seed, pixel, sample) and
added in sample order, so the resumed image is bit-identical to an
uninterrupted render.
"""
from __future__ import annotations

import time

import numpy as np

from . import _lib, bvh as bvh_mod, core, device, scene_compiler
from .scene_data import SceneArrays

# kernels.py:746: the reference's switch between its front-to-back stack
# traversal (False, its default) and its parent-pointer stackless traversal.
# Read when a renderer uploads its camera; the per-renderer attribute
# `use_stackless_traversal` overrides it.
USE_STACKLESS_TRAVERSAL = False


class MI355XRenderer:
    def __init__(self, world, cam, img_path: str, seed: int = 0, samples_per_launch: int = 0, device_id=None):
        self.timing = {'taichi_init': 0.0, 'scene_compile': 0.0, 'bvh_compile': 0.0, 'bvh_flatten': 0.0,
                       'camera_upload': 0.0, 'gpu_upload': 0.0, 'kernel_warmup': 0.0, 'total_setup': 0.0}
        self.sample_times = []
        self.current_sample = 0
        self.render_start_time = 0.0
        t_setup = time.time()
        self.img_path = img_path
        self.cam = cam
        self.cam.initialize()
        self.max_depth = 50
        self.background_color = (0.70, 0.80, 1.00)
        self.seed = int(seed)
        self.use_stackless_traversal = USE_STACKLESS_TRAVERSAL
        # integrator whose samples the accumulator holds (checkpoint state):
        # render_sample() and render() use the megakernel
        self._integrator_label = 'megakernel'
        # periodic checkpoints during render(): every `checkpoint_every` progress chunks
        self.checkpoint_path = None
        self.checkpoint_every = 1
        self._resume_state = None
        # launches per progress report: one launch renders many samples (path regeneration)
        self.samples_per_launch = int(samples_per_launch)
        device.require_gpu()
        # renderer.py:78-80: Perlin tables from a perlin() made after the scene
        perlin = core.perlin()
        t0 = time.time()
        (geom, mats, spheres, qgeom, qmats, quads, tgeom, tmats, tris, _reg,
         img_list) = scene_compiler.compile_scene(world)
        self.timing['scene_compile'] = time.time() - t0
        t0 = time.time()
        bvh = bvh_mod.compile_bvh(world, spheres, quads, tris)
        self.timing['bvh_compile'] = self.timing['bvh_flatten'] = time.time() - t0
        t0 = time.time()
        images = [scene_compiler.image_u8(t) for t in img_list]
        self.arrays = SceneArrays.from_compiled(geom, mats, qgeom, qmats, tgeom, tmats, bvh, perlin.tables(),
                                                images)
        self.dscene = device.DeviceScene.from_arrays(self.arrays, device_id)
        self.integrator = device.Integrator(self.dscene)
        import torch
        self.accum = torch.zeros((self.cam.img_height, self.cam.img_width, 3), dtype=torch.float32,
                                 device=self.dscene.device)
        self._upload_camera()
        self.timing['gpu_upload'] = self.timing['camera_upload'] = time.time() - t0
        self.timing['total_setup'] = time.time() - t_setup

    # ------------------------------------------------------------------ state
    def _upload_camera(self):
        """renderer.py:230-247: camera + background + max_depth as f32/i32."""
        W, H = self.cam.img_width, self.cam.img_height
        self.frame = device.make_frame(self.cam, self.background_color, self.max_depth, self.seed, W, H,
                                       traversal='stackless' if self.use_stackless_traversal else 'stack')
        if tuple(self.accum.shape[:2]) != (H, W):
            import torch
            self.accum = torch.zeros((H, W, 3), dtype=torch.float32, device=self.dscene.device)

    def _upload_camera_to_gpu(self):
        self._upload_camera()

    @property
    def num_spheres(self):
        return self.arrays.num_spheres

    @property
    def num_bvh_nodes(self):
        return self.arrays.num_bvh_nodes

    def clear_accumulation_buffer(self):
        self.integrator.clear(self.frame, self.accum)

    # ---------------------------------------------------------------- renders
    def render_sample(self, sample: int):
        """One sample of every pixel (renderer.py:551-556): sample index
        ``sample`` of the counter-based stream, megakernel."""
        self._integrator_label = 'megakernel'
        self.integrator.render_mk(self.frame, self.accum, int(sample), 1)

    def _run(self, render_fn, label, resume=False):
        import torch
        self._integrator_label = label
        self._upload_camera()
        spp = int(self.cam.samples_per_pixel)
        t0 = time.time()
        if resume:  # continue a loaded checkpoint: no warm-up, keep the accumulator
            if self._resume_state is None:
                raise ValueError('render(resume=True) needs load_checkpoint() first')
            self._check_resume_state()
        else:
            render_fn(self.frame, self.accum, 0, 1)  # warm-up sample, then cleared (renderer.py:381-385)
            torch.cuda.synchronize(self.dscene.device)
            self.clear_accumulation_buffer()
            self.current_sample = 0
        self._resume_state = None
        self.integrator.reset_counters()
        torch.cuda.synchronize(self.dscene.device)
        self.timing['kernel_warmup'] = time.time() - t0
        print(f'\n{self.__class__.__name__} ({label})')
        print(f'Resolution: {self.cam.img_width}x{self.cam.img_height} | Samples: {spp} | Depth: {self.max_depth}')
        print(f'Spheres: {self.num_spheres} | BVH Nodes: {self.num_bvh_nodes}')
        per = self.samples_per_launch or max(1, spp // 20)  # ~20 progress reports, like renderer.py:402
        self.render_start_time = time.time()
        done = self.current_sample
        while done < spp:
            n = min(per, spp - done)
            t = time.time()
            render_fn(self.frame, self.accum, done, n)
            torch.cuda.synchronize(self.dscene.device)
            dt = time.time() - t
            self.sample_times += [dt / n] * n
            done += n
            self.current_sample = done
            pps = self.cam.img_width * self.cam.img_height * n / dt if dt > 0 else 0.0
            print(f'{done:5d}/{spp} ({100.0 * done / spp:5.1f}%) | {dt * 1e3 / n:7.2f} ms/sample | '
                  f'{pps / 1e6:8.2f} Msamples/s')
            if self.checkpoint_path and done < spp and (done // per) % max(1, self.checkpoint_every) == 0:
                self.save_checkpoint(self.checkpoint_path)
        self.write_image()
        self.print_statistics()

    def render(self, enable_preview: bool = True, resume: bool = False):
        """Megakernel render of cam.samples_per_pixel samples (renderer.py:361-434).
        resume=True continues from a load_checkpoint() state."""
        self._run(self.integrator.render_mk, 'megakernel', resume)

    def render_wavefront(self, enable_preview: bool = True, resume: bool = False):
        """Wavefront render (renderer.py:249-359)."""
        self._run(self.integrator.render_wf, 'wavefront', resume)

    # ------------------------------------------------------- checkpoint/resume
    # what must match for a checkpoint to continue this render exactly; the
    # integrator too: megakernel and wavefront paths differ (Q1, Q11, Q14), so
    # a render resumed with the other one would match neither uninterrupted render
    _STATE_KEYS = ('integrator', 'seed', 'max_depth', 'background', 'traversal', 'width', 'height', 'camera',
                   'scene')

    def _render_state(self):
        import hashlib
        lay = self.dscene.layout
        h = hashlib.sha256()
        for a in (lay.nodes, lay.spheres, lay.quads, lay.tris, lay.mats, lay.texels, lay.perlin_vec, lay.perlin_perm):
            h.update(np.ascontiguousarray(a).tobytes())
        f = self.frame
        cam = np.array([list(f.cam.center), list(f.cam.pixel00), list(f.cam.delta_u), list(f.cam.delta_v),
                        list(f.cam.defocus_u), list(f.cam.defocus_v), [f.cam.defocus_angle, 0.0, 0.0]], np.float32)
        return {'integrator': np.array(self._integrator_label), 'seed': np.int64(f.seed), 'max_depth': np.int64(f.max_depth),
                'background': np.array(list(f.bg), np.float32), 'traversal': np.int64(f.traversal),
                'width': np.int64(f.width), 'height': np.int64(f.height), 'camera': cam,
                'scene': np.array(h.hexdigest())}

    def save_checkpoint(self, path):
        """Write the accumulator and the next sample index (plain arrays, npz)
        to exactly ``path`` (no suffix added). The file is written next to it
        under a temporary name and renamed over it, so a crash mid-save leaves
        the previous checkpoint intact."""
        import os
        import tempfile
        import torch
        torch.cuda.synchronize(self.dscene.device)
        st = self._render_state()
        acc = self.accum.cpu().numpy()
        d = os.path.dirname(os.path.abspath(path))
        fd, tmp = tempfile.mkstemp(prefix='.ckpt-', suffix='.npz', dir=d)
        try:
            with os.fdopen(fd, 'wb') as f:
                np.savez(f, accum=acc, next_sample=np.int64(self.current_sample), **st)
            os.replace(tmp, path)
        except BaseException:
            if os.path.exists(tmp):
                os.unlink(tmp)
            raise

    def load_checkpoint(self, path):
        """Load a save_checkpoint() file into this renderer; render(resume=True)
        then renders samples next_sample .. cam.samples_per_pixel - 1. The
        render state (scene arrays, camera, seed, max_depth, background,
        traversal) is checked when the render resumes, after the
        render-time attributes have been applied."""
        import torch
        with np.load(path, allow_pickle=False) as z:
            missing = [k for k in self._STATE_KEYS if k not in z.files]
            if missing:
                raise ValueError(f'{path} is not a checkpoint of this renderer version (missing {missing})')
            state = {k: z[k].copy() for k in self._STATE_KEYS}
            acc = z['accum'].copy()
            nxt = int(z['next_sample'])
        if acc.dtype != np.float32 or acc.ndim != 3 or acc.shape[2] != 3:
            raise ValueError(f'checkpoint accumulator has shape {acc.shape} / {acc.dtype}')
        self.accum = torch.from_numpy(acc).to(self.dscene.device)
        self.current_sample = nxt
        self._resume_state = state

    def _check_resume_state(self):
        cur = self._render_state()
        for k in self._STATE_KEYS:
            if not np.array_equal(cur[k], self._resume_state[k]):
                raise ValueError(f'checkpoint was written for another render: {k} differs')
        if tuple(self.accum.shape) != (int(cur['height']), int(cur['width']), 3):
            raise ValueError('checkpoint accumulator does not match the image size')

    # ----------------------------------------------------------------- output
    def image_u8(self, sample_count=None):
        spp = self.cam.samples_per_pixel if sample_count is None else sample_count
        return self.integrator.tonemap(self.accum, spp).cpu().numpy()

    def write_image(self):
        """PNG of the tone-mapped accumulator (renderer.py:436-442, preview.py:117-132)."""
        from PIL import Image
        Image.fromarray(self.image_u8(), mode='RGB').save(self.img_path)
        print(f'\nImage saved to {self.img_path}')

    _write_image = write_image

    def _get_rr_stats(self):
        """Russian-roulette statistics of the last render (renderer.py:481-500)
        from the device counters, with the reference's keys, value types and
        formulas, so a drop-in caller can format or add them.

        * 'killed': paths ended by RR (kernels.py:1145-1157), counted exactly
          (the reference's atomics are commented out, kernels.py:1193-1202,
          so its own 'killed' is always 0).
        * 'survived', 'avg_depth_killed', 'avg_depth_survived': 0 / 0.0, as in
          the reference: the device does not count paths that passed the RR
          test, nor depth sums. Their names are listed under 'uncounted'.
        * 'total_rr_paths' = killed + survived, as in the reference
          (renderer.py:488). 'kill_rate' is killed / paths x 100, the share of
          all traced paths that Russian roulette ended (0.0 when none were
          traced): the reference's killed / total_rr_paths would read 100 %
          whenever anything was killed, because survived is uncounted here, so
          that formula is not published.
        * Extra keys: 'paths', 'depth_cap' (paths ended by the depth / wave
          budget), 'uncounted'."""
        c = self.integrator.read_counters() or {}
        killed, survived = int(c.get('rr', 0)), 0
        total = killed + survived
        paths = int(c.get('paths', 0))
        return {'killed': killed, 'survived': survived, 'total_rr_paths': total,
                'kill_rate': 100.0 * killed / paths if paths else 0.0,
                'avg_depth_killed': 0.0, 'avg_depth_survived': 0.0,
                'paths': paths, 'depth_cap': int(c.get('depth_cap', 0)),
                'uncounted': ('survived', 'avg_depth_killed', 'avg_depth_survived')}

    def _get_average_depth(self):
        """Mean ray segments per path (renderer.py:473-479 reports the mean
        depth-loop count; a segment is one traversal of that loop)."""
        c = self.integrator.read_counters() or {}
        return c['segments'] / c['paths'] if c.get('paths') else 0.0

    def _print_depth_stats(self):
        """Depth statistics block of renderer.py:502-523."""
        c = self.integrator.read_counters() or {}
        n = c.get('paths', 0)
        if not n:
            return
        print('\nDepth Statistics:')
        print(f'  Average path segments: {c["segments"] / n:.2f} (max depth: {self.max_depth})')
        print(f'  Russian Roulette terminations: {c["rr"]:,} ({100.0 * c["rr"] / n:.1f}%)')
        print(f'  Max depth terminations: {c["depth_cap"]:,} ({100.0 * c["depth_cap"] / n:.1f}%)')
        print(f'  Total paths traced: {n:,}')

    def print_statistics(self):
        if not self.sample_times:
            return
        tot = sum(self.sample_times)
        avg = tot / len(self.sample_times)
        pps = self.cam.img_width * self.cam.img_height / avg if avg > 0 else 0.0
        c = self.integrator.read_counters() or {}
        print('\nPERFORMANCE SUMMARY')
        print(f'Total Render Time: {tot:6.2f}s')
        print(f'Throughput: {pps / 1e6:8.2f} Msamples/s')
        if c.get('paths'):
            print(f'Segments/sample: {c["segments"] / c["paths"]:.3f} | '
                  f'medium traversals/sample: {c["medium"] / c["paths"]:.3f}')
        self._print_depth_stats()

    _print_stats = print_statistics

    # -------------------------------------------------- live preview (GUI, out of scope)
    def setup_live_preview(self, update_interval_ms=500):
        """renderer.py:593-616 opens a Tk window here. The Tk GUI is out of
        scope, so this records the interval and opens nothing;
        callers such as InteractiveViewer keep working headless."""
        self.update_interval_ms = update_interval_ms
        self.preview_window = None
        self.last_preview_update = 0.0

    def update_preview_if_needed(self):
        """renderer.py:618-648: no window was opened (setup_live_preview), so
        there is nothing to refresh; use image_u8() for the current image."""
        return None


TaichiRenderer = MI355XRenderer  # drop-in name (render_server.taichi_renderer.TaichiRenderer)
