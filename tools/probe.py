"""Debug probes of the megakernel (diagnostic builds, not product).
PTMI_PROBE=1: node visits, wave-uniform visits, pops, culls, leaf tests, node-step SIMD efficiency.
PTMI_PROBE=2: wave cycles in the traversal loop vs shading (s_memtime), wave steps per sample and
the share of steps that ran a sphere / quad-triangle / node branch.
usage: PTMI_LIB=.../libptmi_probeN.so probe.py [SCENE WIDTH SPP]"""
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
out = (C.c_ulonglong * 16)()
lib.ptmi_probe_read(out, 1)
integ.reset_counters()
integ.render_mk(fr, acc, 0, spp)
torch.cuda.synchronize()
lib.ptmi_probe_read(out, 1)
c = integ.read_counters()
n, u, steps, lanes, pops, culled, lsph, lother = list(out)[:8]
cyc_trav, cyc_shade, wsteps, wsph, woth, wnode, wboth, wbusy = list(out)[8:16]
print(json.dumps({'scene': scene, 'spp': spp, 'node_visits': n, 'uniform_visit_frac': u / max(1, n),
                  'simd_eff_node_steps': lanes / max(1, 64 * steps), 'node_visits_per_traversal':
                  n / max(1, c['segments'] + c['medium']), 'pops_per_traversal': pops / max(1, c['segments'] + c['medium']),
                  'culled_frac': culled / max(1, pops), 'leaf_tests_per_traversal': (lsph + lother) / max(1, c['segments'] + c['medium']),
                  'sphere_leaf_frac': lsph / max(1, lsph + lother),
                  'probe2': {'cycles_trav_frac': cyc_trav / max(1, cyc_trav + cyc_shade), 'wave_steps_per_sample':
                             wsteps / max(1, c['paths']), 'sphere_step_frac': wsph / max(1, wsteps),
                             'quadtri_step_frac': woth / max(1, wsteps), 'node_step_frac': wnode / max(1, wsteps),
                             'sphere_and_quadtri_step_frac': wboth / max(1, wsteps), 'busy_lanes_per_step': wbusy / max(1, wsteps),
                             'cycles_per_wave_step': cyc_trav / max(1, wsteps),
                             'shade_cycles_per_sample': cyc_shade / max(1, c['paths'])}, **c}))
