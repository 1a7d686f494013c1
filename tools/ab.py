"""A/B timing of one libptmi build (PTMI_LIB=...) on one workload (not product).
usage: ab.py VARIANT(mk|mkd|wf|mksl|wfsl) SPP REPS [SCENE WIDTH]  (sl: stackless traversal)"""
import os, sys, time, json
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
from ptmi import device, _lib
import bench


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else 'mk'
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    scene = sys.argv[4] if len(sys.argv) > 4 else 'vol2_final_scene'
    width = int(sys.argv[5]) if len(sys.argv) > 5 else 800
    sa, cam, bg, _ = bench.load_workload(scene, width)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H, traversal='stackless' if variant.endswith('sl') else 'stack')
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    f = {'mk': integ.render_mk, 'wf': integ.render_wf, 'mksl': integ.render_mk, 'wfsl': integ.render_wf,
         'mkd': lambda *a: integ.render_mk(*a, staged=False)}[variant]
    f(fr, acc, 0, 4); torch.cuda.synchronize()
    best = 1e9
    for r in range(reps):
        t = time.perf_counter(); f(fr, acc, 4 + r * spp, spp); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t)
    print(json.dumps({'lib': os.path.basename(_lib.LIB_PATH),
                      'variant': variant, 'scene': scene, 'width': width,
                      'spp': spp, 'Msamples_s': round(W * H * spp / best / 1e6, 1), 'ms': round(best * 1e3, 2)}),
          flush=True)


if __name__ == '__main__':
    main()
