"""Bisect (2): the bench-shape stackless test in a fresh process, with and without a
prior stack-traversal BenchRun in the same process (debug tool, not product)."""
import os, sys, json
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT, os.path.join(ROOT, 'tests')]
import numpy as np
import torch
import bench
import oracle
from parity_helpers import compare

win = (368, 368, 64, 64)


def trial(name, run):
    W, H = run.W, run.H
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    for k in (24, 25, 26):
        run.step(acc, k)
    torch.cuda.synchronize()
    g = acc.cpu().numpy()
    o = np.zeros((H, W, 3), np.float32)
    ofr = oracle.make_frame(run.cam, run.bg, 50, 0, W, H, run.a.traversal)
    oracle.render(oracle.OracleScene(run.sa), ofr, 'mk', o, win, 1536, 192, 16)
    x0, y0, w, h = win
    linf, ex = compare(g[y0:y0+h, x0:x0+w], o[y0:y0+h, x0:x0+w], 192)
    print(json.dumps({'case': name, 'linf': linf, 'identical': ex}), flush=True)


which = sys.argv[1]
if which == 'fresh':
    trial('stackless fresh', bench.BenchRun(bench.parse(['--traversal', 'stackless']), torch.device('cuda', 0)))
else:
    r0 = bench.BenchRun(bench.parse([]), torch.device('cuda', 0))
    trial('stack first', r0)
    trial('stackless after stack', bench.BenchRun(bench.parse(['--traversal', 'stackless']), torch.device('cuda', 0)))
    trial('stack again', r0)
