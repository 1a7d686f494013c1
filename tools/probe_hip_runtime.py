"""Which HIP runtime(s) a process maps when torch and libptmi are loaded in a
given order, and whether a tiny render works (diagnostic, not product).
usage: probe_hip_runtime.py torch-first|lib-first"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT, os.path.join(ROOT, 'tests')]
order = sys.argv[1] if len(sys.argv) > 1 else 'torch-first'
if order == 'lib-first':
    from ptmi import _lib
    _lib.load()
import torch  # noqa: E402
from ptmi import device  # noqa: E402


def maps():
    with open('/proc/self/maps') as f:
        return sorted({l.split()[-1] for l in f if 'amdhip64' in l or 'hsa-runtime64' in l})


print(order, 'before render:', maps(), flush=True)
from edge_scenes import edge_scene  # noqa: E402
sa, cam, bg = edge_scene('single', 16)
integ = device.Integrator(device.DeviceScene.from_arrays(sa))
fr = device.make_frame(cam, bg, 50, 3, cam['width'], cam['height'])
acc = torch.zeros((cam['height'], cam['width'], 3), dtype=torch.float32, device='cuda')
try:
    integ.render_mk(fr, acc, 0, 2)
    torch.cuda.synchronize()
    print(order, 'render ok, sum', float(acc.sum()), flush=True)
except Exception as e:  # noqa: BLE001
    print(order, 'render FAILED:', e, flush=True)
print(order, 'after render:', maps(), flush=True)
