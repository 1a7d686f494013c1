#!/usr/bin/env python3
"""Drain-consolidation probe (diagnostic build PTMI_PROBE=5 with PTMI_MK_MIGRATE, not product):
retirements, records donated / claimed, keeper polls, wave exits and the call's span
(s_memrealtime, 100 MHz) for one staged megakernel call. usage: PTMI_LIB=... mig_probe.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
import bench
from ptmi import device, _lib


def main():
    a = bench.parse([])
    run = bench.BenchRun(a, torch.device('cuda', 0))
    W, H = run.W, run.H
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    lib = _lib.load()
    out = (C.c_ulonglong * 16)()
    fr = device.make_frame(run.cam, run.bg, 50, 0, W, H)
    for spp in (8, 64):
        run.integ.render_mk(fr, acc, 0, spp)
        torch.cuda.synchronize()
        lib.ptmi_probe_read(out, 1)
        run.integ.render_mk(fr, acc, 100, spp)
        torch.cuda.synchronize()
        lib.ptmi_probe_read(out, 1)
        v = list(out)
        print(json.dumps({'spp': spp, 'retired': v[0], 'donated': v[1], 'claimed': v[2], 'keeper_polls': v[3],
                          'keeper_bound_hits': v[4], 'exits': v[5], 'publish_wait_iters': v[6],
                          'span_us': (v[8] - (2 ** 64 - 1 - v[9])) / 100.0, 'last_start_us': (v[10] - (2 ** 64 - 1 - v[9])) / 100.0,
                          'wave_life_us_mean': v[11] / max(1, v[5]) / 100.0, 'keep_polls_sum': v[12],
                          'retiring_exits': v[13], 'drain_start_us_mean': v[14] / max(1, v[5]) / 100.0,
                          'retire_to_exit_us_mean': v[7] / max(1, v[13]) / 100.0,
                          'nonretiring_life_us_mean': v[15] / max(1, v[5] - v[13]) / 100.0}), flush=True)


if __name__ == '__main__':
    main()
