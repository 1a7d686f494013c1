#!/usr/bin/env python3
"""Diagnostic (not product): the wavefront parity windows of tests/test_gpu_parity.py
rendered by one library build at several tail thresholds (ptmi_wf_set_drain_at),
each compared with the CPU oracle pixel by pixel; with a trace build
(PTMI_WF_TRACE, variants tr*/ti*) every wf_drain segment record is saved too.

usage: PTMI_LIB=.../libptmi_X.so python tools/wf_drain_trace.py OUT.npz [REPS]
The records are compared across builds by tools/wf_drain_trace_diff.py."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), os.path.join(ROOT, 'tests'), ROOT]
import numpy as np  # noqa: E402
from parity_helpers import compare, gpu_render, oracle_render  # noqa: E402
from test_gpu_parity import CASES  # noqa: E402
from ptmi import _lib  # noqa: E402

WORDS = 12


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    lib = _lib.load()
    tr = getattr(lib, 'ptmi_wf_trace_read', None) if hasattr(lib, 'ptmi_wf_trace_read') else None
    if tr is not None:
        tr.restype = C.c_int64
        tr.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        tr(None, 0, 1)
    saved = {}
    oracle_cache = {}
    fails = 0
    for drain_at in (16, 1):
        prev = lib.ptmi_wf_set_drain_at(drain_at)
        for case in CASES:
            name, width, window, spp = case
            key = (name, width, window, spp)
            if key not in oracle_cache:
                oracle_cache[key] = oracle_render(name, width, 'wf', window, 0, spp)
            o, ost = oracle_cache[key]
            for rep in range(reps):
                t0 = time.time()
                g, gst, _ = gpu_render(name, width, 'wf', window, 0, spp)
                x0, y0, w, h = window
                linf, exact = compare(g[y0:y0 + h, x0:x0 + w], o[y0:y0 + h, x0:x0 + w], spp)
                bad = np.argwhere(np.any(g != o, axis=-1) & ~np.all(np.isnan(g) & np.isnan(o), axis=-1))
                row = {'lib': os.path.basename(_lib.LIB_PATH), 'drain_at': drain_at, 'case': f'{name}-{width}-{window}',
                       'rep': rep, 'linf': linf, 'exact': exact, 'bad_pixels': bad[:8].tolist(), 'n_bad': len(bad),
                       'gpu': gst, 'oracle': ost, 's': round(time.time() - t0, 2)}
                fails += len(bad) > 0
                if tr is not None:
                    n = tr(None, 0, 0)
                    buf = np.zeros((max(1, min(n, 1 << 22)), WORDS), np.uint32)
                    tr(buf.ctypes.data, buf.shape[0], 1)
                    row['trace_records'] = int(n)
                    saved[f'{drain_at}|{name}-{width}-{window[0]}_{window[1]}|{rep}'] = buf[:n]
                    saved[f'{drain_at}|{name}-{width}-{window[0]}_{window[1]}|{rep}|bad'] = bad.astype(np.int32)
                print(json.dumps(row), flush=True)
        lib.ptmi_wf_set_drain_at(prev)
    if saved:
        np.savez_compressed(out, **saved)
    print(json.dumps({'lib': os.path.basename(_lib.LIB_PATH), 'failing_renders': fails}), flush=True)


if __name__ == '__main__':
    main()
