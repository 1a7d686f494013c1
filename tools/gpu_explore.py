"""Quick GPU throughput exploration (not part of the product)."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'path-tracer-python_amd'))
import numpy as np, torch
from ptmi import device, scene_data as sd, _lib

def run(name, width, variant, spp_per_launch, launches, bg):
    sa = sd.load_fixture(name)
    cam = sd.fixture_camera(name, width)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    f = integ.render_mk if variant == 'mk' else integ.render_wf
    f(fr, acc, 0, spp_per_launch)  # warmup
    torch.cuda.synchronize()
    integ.reset_counters()
    with _lib.KernelTimer() as kt:
        t0 = time.perf_counter()
        for i in range(launches):
            f(fr, acc, (i + 1) * spp_per_launch, spp_per_launch)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    c = integ.read_counters()
    ns = W * H * spp_per_launch * launches
    prof = {k: round(v['ms'], 2) for k, v in kt.result.items() if v['launches']}
    print(f'{name} {W}x{H} {variant} spp/launch={spp_per_launch} launches={launches}: {dt*1e3:.1f} ms '
          f'{ns/dt/1e6:.1f} Msamples/s seg/sample={c["segments"]/ns:.3f} med/sample={c["medium"]/ns:.3f} '
          f'Gseg/s={(c["segments"]+c["medium"])/dt/1e9:.3f} prof_ms={prof}', flush=True)

if __name__ == '__main__':
    for variant, spl, n in [('mk', 1, 8), ('mk', 8, 2), ('mk', 32, 1), ('wf', 1, 8)]:
        run('vol2_final_scene', 800, variant, spl, n, (0, 0, 0))
    for variant, spl, n in [('mk', 4, 2), ('wf', 1, 4)]:
        run('wavefront_comparison', 800, variant, spl, n, (0.7, 0.8, 1.0))
        run('cornell_smoke', 800, variant, spl, n, (0, 0, 0))
