"""Throughput of a 512-spp render split into calls of n spp, with and without
overlapped megakernel launches (not product). Separates the per-launch fixed
cost that overlap hides (the drain of the last long paths) from the one it
cannot (whatever each launch pays inside its own kernel)."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
from ptmi import device
import bench


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else 'vol2_final_scene'
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    total = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    sa, cam, bg, _ = bench.load_workload(scene, width)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    for ov in (False, True):
        integ.render_mk(fr, acc, 0, 8, overlap=ov)
    torch.cuda.synchronize()
    for n in [int(x) for x in os.environ.get('PROBE_N', '8,16,32,64,128,256').split(',')]:
        for ov in (False, True):
            best = 1e9
            for _ in range(2):
                t = time.perf_counter()
                for s0 in range(0, total, n):
                    integ.render_mk(fr, acc, s0, n, overlap=ov)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t)
            print(json.dumps({'spp_per_call': n, 'overlap': ov, 'ms': round(best * 1e3, 2),
                              'Msamples_s': round(W * H * total / best / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    main()
