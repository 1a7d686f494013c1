#!/usr/bin/env python3
"""Section probe of the persistent megakernel (diagnostic build PTMI_PROBE=4, not product):
wave cycles per section of the outer loop for one staged 32-spp call.
usage: PTMI_LIB=.../libptmi_probe4.so section_probe.py [SCENE WIDTH SPP]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
import bench
from ptmi import device, _lib

NAMES = ['traversal', 'wave_turbulence', 'material_medium_scatter', 'unit_vector_scatter_end', 'epilogue_staging',
         'refill', 'segment_begin']


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else 'vol2_final_scene'
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    sa, cam, bg, _ = bench.load_workload(scene, width)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    lib = _lib.load()
    out = (C.c_ulonglong * 16)()
    integ.render_mk(fr, acc, 0, 4)
    torch.cuda.synchronize()
    lib.ptmi_probe_read(out, 1)
    integ.reset_counters()
    integ.render_mk(fr, acc, 4, spp)
    torch.cuda.synchronize()
    lib.ptmi_probe_read(out, 1)
    c = integ.read_counters()
    v = list(out)[:7]
    tot = sum(v)
    print(json.dumps({'scene': scene, 'spp': spp, 'frac': {n: round(x / max(1, tot), 4) for n, x in zip(NAMES, v)},
                      'cycles_per_sample': {n: round(x / max(1, c['paths']), 1) for n, x in zip(NAMES, v)}, **c}))


if __name__ == '__main__':
    main()
