"""Debug probe (PTMI_PROBE build): node visits, wave-uniform node visits,
wave-level node steps and their active lanes, for one megakernel render.
usage: PTMI_LIB=.../libptmi_probe.so probe.py [SCENE WIDTH SPP]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
from ptmi import device, _lib
import bench

scene = sys.argv[1] if len(sys.argv) > 1 else 'vol2_final_scene'
width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 8
sa, cam, bg, _ = bench.load_workload(scene, width)
W, H = cam['width'], cam['height']
integ = device.Integrator(device.DeviceScene.from_arrays(sa))
fr = device.make_frame(cam, bg, 50, 0, W, H)
acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
lib = _lib.load()
out = (C.c_ulonglong * 8)()
lib.ptmi_probe_read(out, 1)
integ.reset_counters()
integ.render_mk(fr, acc, 0, spp)
torch.cuda.synchronize()
lib.ptmi_probe_read(out, 1)
c = integ.read_counters()
n, u, steps, lanes, pops, culled, lsph, lother = list(out)
print(json.dumps({'scene': scene, 'spp': spp, 'node_visits': n, 'uniform_visit_frac': u / max(1, n),
                  'simd_eff_node_steps': lanes / max(1, 64 * steps), 'node_visits_per_traversal':
                  n / max(1, c['segments'] + c['medium']), 'pops_per_traversal': pops / max(1, c['segments'] + c['medium']),
                  'culled_frac': culled / max(1, pops), 'leaf_tests_per_traversal': (lsph + lother) / max(1, c['segments'] + c['medium']),
                  'sphere_leaf_frac': lsph / max(1, lsph + lother), **c}))
