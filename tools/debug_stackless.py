"""Bisect a stackless-traversal mismatch at the bench's call shape (debug tool, not product)."""
import os, sys, json
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT, os.path.join(ROOT, 'tests')]
import numpy as np
import torch
import bench
import oracle
from ptmi import device
from parity_helpers import compare

a = bench.parse(['--traversal', 'stackless'])
run = bench.BenchRun(a, torch.device('cuda', 0))
W, H = run.W, run.H
win = (368, 368, 64, 64)
osc = oracle.OracleScene(run.sa)
ofr = oracle.make_frame(run.cam, run.bg, 50, 0, W, H, 'stackless')


def ref(s0, n):
    o = np.zeros((H, W, 3), np.float32)
    st = oracle.render(osc, ofr, 'mk', o, win, s0, n, 16)
    return o, st


def check(name, window, s0, n, per, **kw):
    fr = device.make_frame(run.cam, run.bg, 50, 0, W, H, window, traversal='stackless')
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    b = 0
    while b < n:
        m = min(per, n - b)
        run.integ.render_mk(fr, acc, s0 + b, m, **kw)
        b += m
    torch.cuda.synchronize()
    g = acc.cpu().numpy()
    o, _ = ref(s0, n)
    x0, y0, w, h = win
    linf, ex = compare(g[y0:y0+h, x0:x0+w], o[y0:y0+h, x0:x0+w], n)
    print(json.dumps({'case': name, 'linf': linf, 'identical': ex}), flush=True)


full = (0, 0, W, H)
check('win s0=0 n=4 per=4', win, 0, 4, 4)
check('win s0=1536 n=4 per=4', win, 1536, 4, 4)
check('win s0=0 n=64 per=64', win, 0, 64, 64)
check('full s0=0 n=4 per=4 staged', full, 0, 4, 4)
check('full s0=0 n=64 per=64 staged', full, 0, 64, 64)
check('full s0=0 n=8 per=1 direct', full, 0, 8, 1)
check('full s0=1536 n=64 per=64 overlap', full, 1536, 64, 64, overlap=True)
