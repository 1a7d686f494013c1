"""Fixed per-launch cost of the staged megakernel (not product): time one
render_mk call at several sample counts (best of REPS) and fit
T(spp) = T0 + a * spp. T0 is what a launch pays besides its samples (grid
ramp-up, the drain of the last units, the resolve kernel, the counter reset).
usage: launch_fit.py [SCENE WIDTH VARIANT]"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import numpy as np
import torch
from ptmi import device
import bench


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else 'vol2_final_scene'
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    variant = sys.argv[3] if len(sys.argv) > 3 else 'mk'
    sa, cam, bg, _ = bench.load_workload(scene, width)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    f = integ.render_mk if variant == 'mk' else integ.render_wf
    f(fr, acc, 0, 8)
    torch.cuda.synchronize()
    xs, ys = [], []
    base = 8
    for spp in (8, 16, 32, 64, 128):
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            f(fr, acc, base, spp)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
            base += spp
        xs.append(spp)
        ys.append(best * 1e3)
        print(json.dumps({'spp': spp, 'ms': round(best * 1e3, 3), 'Msamples_s': round(W * H * spp / best / 1e6, 1)}),
              flush=True)
    a, t0 = np.polyfit(xs, ys, 1)
    print(json.dumps({'scene': scene, 'variant': variant, 'fit_T0_ms': round(float(t0), 3),
                      'fit_ms_per_spp': round(float(a), 4),
                      'T0_share_at_64spp': round(float(t0 / (t0 + 64 * a)), 4)}), flush=True)


if __name__ == '__main__':
    main()
