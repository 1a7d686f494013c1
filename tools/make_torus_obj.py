"""Writes the build-supplied OBJ mesh for BASELINE configs[3] (a torus of
quad faces; the loader fan-triangulates them): ptmi/assets/torus.obj."""
import math
import os

R, r, NU, NV = 1.0, 0.38, 60, 25
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'path-tracer-python_amd', 'ptmi', 'assets',
                   'torus.obj')
with open(out, 'w') as f:
    f.write('# torus R=1 r=0.38, 60x25 quads (build-supplied mesh for the OBJ Cornell config)\n')
    for i in range(NU):
        u = 2 * math.pi * i / NU
        for j in range(NV):
            v = 2 * math.pi * j / NV
            x = (R + r * math.cos(v)) * math.cos(u)
            z = (R + r * math.cos(v)) * math.sin(u)
            y = r * math.sin(v) + 0.15 * math.sin(3 * u)
            f.write(f'v {x:.6f} {y:.6f} {z:.6f}\n')
    for i in range(NU):
        for j in range(NV):
            a = i * NV + j + 1
            b = ((i + 1) % NU) * NV + j + 1
            c = ((i + 1) % NU) * NV + (j + 1) % NV + 1
            d = i * NV + (j + 1) % NV + 1
            f.write(f'f {a} {b} {c} {d}\n')
print(out)
