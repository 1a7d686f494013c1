"""Headless InteractiveViewer (reference: src/render_server/interactive_viewer.py:18-451).

The reference's vol2_final_scene / cornell_box / cornell_smoke entry points
(scenes.py:1068, 1144, 1242) drive the renderer through
``InteractiveViewer(world, cam, path).render_interactive()``: progressive
accumulation up to ``cam.samples_per_pixel``, orbit-camera rotation that
restarts accumulation, and the image written at the end divided by
``cam.samples_per_pixel`` (renderer.py:436-442). This class keeps that API and
those effects on the MI355X integrator. The Tk preview window is out of scope
(SURVEY.md §2), so ``render_interactive`` returns once the sample budget is
reached instead of idling in a window; the mouse handlers stay callable with
any object carrying ``.x`` / ``.y`` so a host GUI can still drive them.

Progressive sampling launches ``display_interval`` samples per call (the
reference launches one per call, :389): sample i of a pixel is keyed by
(seed, pixel, i), so the accumulated image is bit-identical however the
samples are batched.
"""
from __future__ import annotations

import math
import statistics
import time

from .renderer import MI355XRenderer


def spherical_from(lookfrom, lookat):
    """(radius, theta, phi) of lookfrom around lookat (interactive_viewer.py:52-71)."""
    off = lookfrom - lookat
    r = math.sqrt(off.x ** 2 + off.y ** 2 + off.z ** 2)
    theta = math.atan2(off.x, -off.z)
    phi = math.asin(off.y / r) if r > 0 else 0.0
    return r, theta, phi


def spherical_offset(radius, theta, phi):
    """Cartesian offset (x, y, z) of spherical coordinates (interactive_viewer.py:73-99)."""
    cp, sp = math.cos(phi), math.sin(phi)
    ct, st = math.cos(theta), math.sin(theta)
    return radius * cp * st, radius * sp, -radius * cp * ct


def orbit_step(theta, phi, delta_x, delta_y, velocity=(0.3, 0.3)):
    """New (theta, phi) after a mouse delta, phi clamped to +-89 deg (interactive_viewer.py:101-123)."""
    theta += math.radians(delta_x * velocity[0])
    phi += math.radians(delta_y * velocity[1])
    lim = math.radians(89.0)
    return theta, max(-lim, min(lim, phi))


class InteractiveViewer(MI355XRenderer):
    def __init__(self, world, cam, img_path: str, **kwargs):
        super().__init__(world, cam, img_path, **kwargs)
        self.mouse_down = False
        self.last_mouse_x = 0
        self.last_mouse_y = 0
        self.last_camera_update_time = 0
        self.camera_update_interval = 0.05
        self.rotation_velocity = (0.3, 0.3)
        self._camera_radius = 0.0
        self._camera_theta = 0.0
        self._camera_phi = 0.0
        self._initialize_spherical_coords()
        self.is_rendering_active = True
        self.preview_window = None

    # ----------------------------------------------------------- orbit camera
    def _initialize_spherical_coords(self):
        self._camera_radius, self._camera_theta, self._camera_phi = spherical_from(self.cam.lookfrom,
                                                                                   self.cam.lookat)

    def _spherical_to_cartesian(self, radius, theta, phi):
        x, y, z = spherical_offset(radius, theta, phi)
        return type(self.cam.lookfrom - self.cam.lookat)(x, y, z)

    def rotate_camera(self, delta_x, delta_y):
        self._camera_theta, self._camera_phi = orbit_step(self._camera_theta, self._camera_phi, delta_x, delta_y,
                                                          self.rotation_velocity)
        offset = self._spherical_to_cartesian(self._camera_radius, self._camera_theta, self._camera_phi)
        self.cam.lookfrom = self.cam.lookat + offset
        self.cam.initialize()
        self._upload_camera_to_gpu()

    def restart_rendering(self):
        self.current_sample = 0
        self.sample_times = []
        self.render_start_time = time.time()
        self.clear_accumulation_buffer()
        self.integrator.reset_counters()
        self.is_rendering_active = True
        print(f"\n{'─' * 60}\nCamera rotated - restarting render from sample 0\n{'─' * 60}")

    # ------------------------------------------------------- mouse handlers
    def on_mouse_down(self, event):
        self.mouse_down = True
        self.last_mouse_x, self.last_mouse_y = event.x, event.y

    def on_mouse_up(self, event):
        self.mouse_down = False

    def on_mouse_drag(self, event):
        if not self.mouse_down:
            return
        now = time.time()
        if now - self.last_camera_update_time < self.camera_update_interval:
            self.last_mouse_x, self.last_mouse_y = event.x, event.y
            return
        self.last_camera_update_time = now
        dx, dy = event.x - self.last_mouse_x, event.y - self.last_mouse_y
        self.last_mouse_x, self.last_mouse_y = event.x, event.y
        if dx == 0 and dy == 0:
            return
        self.rotate_camera(dx, dy)
        self.restart_rendering()

    def setup_interactive_preview(self, update_interval_ms=16):
        """No window here (Tk preview is out of scope); kept for API compatibility."""
        self.update_interval_ms = update_interval_ms

    def update_preview_if_needed(self):
        return None

    # ------------------------------------------------------------ rendering
    def render_interactive(self):
        """Progressive render to cam.samples_per_pixel, then write the image
        (interactive_viewer.py:327-451, headless)."""
        import torch
        spp = int(self.cam.samples_per_pixel)
        print('\nInteractiveViewer')
        print(f'Resolution: {self.cam.img_width}x{self.cam.img_height} | Max Samples: {spp} | Depth: {self.max_depth}')
        print(f'Spheres: {self.num_spheres} | BVH Nodes: {self.num_bvh_nodes}')
        self._upload_camera_to_gpu()
        t0 = time.time()
        self.render_sample(0)  # warm-up sample, cleared (interactive_viewer.py:355-359)
        torch.cuda.synchronize(self.dscene.device)
        self.clear_accumulation_buffer()
        self.integrator.reset_counters()
        print(f'  Kernel Warmup: {(time.time() - t0) * 1000:6.2f}ms')
        self.setup_interactive_preview()
        display_interval = max(1, spp // 20)
        total_pixels = self.cam.img_width * self.cam.img_height
        print(f"\nRendering Progress:\n{'─' * 60}")
        self.render_start_time = time.time()
        while self.is_rendering_active and self.current_sample < spp:
            n = min(display_interval - self.current_sample % display_interval, spp - self.current_sample)
            if self.current_sample == 0:
                n = 1  # the reference prints sample 1
            t = time.time()
            self.integrator.render_mk(self.frame, self.accum, self.current_sample, n)
            torch.cuda.synchronize(self.dscene.device)
            dt = (time.time() - t) / n
            self.sample_times += [dt] * n
            self.current_sample += n
            elapsed = time.time() - self.render_start_time
            avg = sum(self.sample_times) / len(self.sample_times)
            thr = total_pixels / avg if avg > 0 else 0.0
            print(f'{self.current_sample:4d}/{spp} ({self.current_sample / spp * 100:5.1f}%) │ {dt * 1000:5.1f}ms │ '
                  f'Elapsed: {elapsed:5.1f}s │ Throughput: {thr / 1e6:5.2f}M pix/s │ '
                  f'ETA: {(spp - self.current_sample) * avg:4.1f}s')
        if self.current_sample >= spp:
            print(f"{'─' * 60}\n✓ Reached max samples ({spp})")
            self.is_rendering_active = False
        self._print_render_summary()
        self._sync_gpu_to_cpu()
        self.write_image()

    def _sync_gpu_to_cpu(self):
        """renderer.py:566-573: nothing to copy (the accumulator stays on the GPU)."""
        return None

    def _print_render_summary(self):
        if not self.sample_times:
            return
        st = self.sample_times
        avg = statistics.mean(st)
        total_pixels = self.cam.img_width * self.cam.img_height
        c = self.integrator.read_counters() or {}
        print(f"\n{'═' * 60}\nRENDER SUMMARY\n{'═' * 60}")
        print(f'Resolution:       {self.cam.img_width} x {self.cam.img_height} ({total_pixels:,} pixels)')
        print(f'Samples:          {self.current_sample} / {self.cam.samples_per_pixel}')
        print(f'Max Ray Depth:    {self.max_depth}')
        if c.get('paths'):
            print(f'Avg Path Depth:   {c["segments"] / c["paths"]:.2f}')
        print(f'Scene Complexity: {self.num_spheres} spheres, {self.num_bvh_nodes} BVH nodes')
        print(f'Total Render Time:  {time.time() - self.render_start_time:6.2f}s')
        print(f'Sample Time: mean {avg * 1000:6.2f}ms | median {statistics.median(st) * 1000:6.2f}ms | '
              f'min {min(st) * 1000:6.2f}ms | max {max(st) * 1000:6.2f}ms')
        print(f'Pixels/sec:       {total_pixels / avg / 1e6 if avg > 0 else 0.0:6.2f} Mpix/s')
