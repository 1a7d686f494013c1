"""A/B timing of one libptmi build (PTMI_LIB=...) on vol2 800x800 (not product)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'path-tracer-python_amd'))
import torch
from ptmi import device, scene_data as sd, _lib

def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else 'mk'
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    sa = sd.load_fixture('vol2_final_scene')
    cam = sd.fixture_camera('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, (0, 0, 0), 50, 0, 800, 800)
    acc = torch.zeros((800, 800, 3), dtype=torch.float32, device='cuda')
    f = {'mk': integ.render_mk, 'wf': integ.render_wf,
         'mkd': lambda *a: integ.render_mk(*a, staged=False)}[variant]
    f(fr, acc, 0, 4); torch.cuda.synchronize()
    best = 1e9
    for r in range(reps):
        t = time.perf_counter(); f(fr, acc, 4 + r * spp, spp); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t)
    print(json.dumps({'lib': os.path.basename(_lib.LIB_PATH), 'variant': variant, 'spp': spp,
                      'Msamples_s': round(800 * 800 * spp / best / 1e6, 1), 'ms': round(best * 1e3, 2)}), flush=True)

if __name__ == '__main__':
    main()
