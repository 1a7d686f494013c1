#!/usr/bin/env python3
"""Drain probe of the persistent megakernel (diagnostic build PTMI_PROBE=3, not product).

For overlapped calls of several sizes: the share of the waves' cycles spent
after the batch's units ran out for them (the drain), and the live lanes in
those cycles. usage: PTMI_LIB=.../libptmi_probe3.so drain_probe.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
import bench
from ptmi import device, _lib
from ptmi.distributed import Shard


def main():
    a = bench.parse([])
    run = bench.BenchRun(a, torch.device('cuda', 0))
    W, H = run.W, run.H
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    lib = _lib.load()
    out = (C.c_ulonglong * 16)()
    sh = Shard(0, 8, 'tiles', 4)
    cases = [('full_64spp', device.make_frame(run.cam, run.bg, 50, 0, W, H), 64),
             ('rank0_of_8_band4_64spp', device.make_frame(run.cam, run.bg, 50, 0, W, H, band=sh.band()), 64),
             ('full_8spp', device.make_frame(run.cam, run.bg, 50, 0, W, H), 8)]
    for name, fr, spp in cases:
        for k in range(2):
            run.integ.render_mk(fr, acc, k * spp, spp, overlap=True)
        torch.cuda.synchronize()
        lib.ptmi_probe_read(out, 1)
        for k in range(8):
            run.integ.render_mk(fr, acc, 1000 + k * spp, spp, overlap=True)
        torch.cuda.synchronize()
        lib.ptmi_probe_read(out, 1)
        tot, dry, lanecyc, waves = list(out)[:4]
        print(json.dumps({'case': name, 'waves': waves, 'drain_frac_of_wave_cycles': round(dry / max(1, tot), 4),
                          'drain_lane_eff': round(lanecyc / max(1, 64 * dry), 4),
                          'idle_lane_cycles_in_drain_frac': round((64 * dry - lanecyc) / max(1, 64 * tot), 4),
                          'wave_cycles_mean': round(tot / max(1, waves)), 'drain_cycles_mean': round(dry / max(1, waves))}))


if __name__ == '__main__':
    main()
