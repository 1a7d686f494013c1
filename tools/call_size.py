#!/usr/bin/env python3
"""Throughput of the overlapped megakernel against call size (evidence tool, not product):
full-frame calls of S spp vs one 8-rank tile shard at 64 spp (same samples per call)."""
import json, os, sys, time
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'path-tracer-python_amd'), ROOT]
import torch
import bench
from ptmi import device
from ptmi.distributed import Shard


def rate(integ, fr, acc, npix, spp, calls=16, s0=1000):
    for k in range(3):
        integ.render_mk(fr, acc, k * spp, spp, overlap=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(calls):
        integ.render_mk(fr, acc, s0 + k * spp, spp, overlap=True)
    torch.cuda.synchronize()
    return npix * spp * calls / (time.perf_counter() - t) / 1e6


def main():
    a = bench.parse([])
    run = bench.BenchRun(a, torch.device('cuda', 0))
    W, H = run.W, run.H
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    out = {}
    for spp in [int(x) for x in os.environ.get('CALL_SIZE_SPP', '64,32,16,8').split(',')]:
        out[f'full_{spp}spp'] = round(rate(run.integ, run.frame, acc, W * H, spp), 1)
    shards = os.environ.get('CALL_SIZE_SHARDS', '8:4,8:8,4:8,2:8')
    for ranks, band in [tuple(int(v) for v in x.split(':')) for x in shards.split(',') if x]:
        sh = Shard(0, ranks, 'tiles', band)
        fr = device.make_frame(run.cam, run.bg, 50, 0, W, H, band=sh.band())
        out[f'rank0_of_{ranks}_band{band}_64spp'] = round(rate(run.integ, fr, acc, W * len(sh.rows(H)), 64), 1)
    if os.environ.get('CALL_SIZE_SHARDS') is not None:
        out['lib'] = os.path.basename(os.environ.get('PTMI_LIB', 'libptmi.so'))
        out['depth'] = os.environ.get('PTMI_OVERLAP_DEPTH', 'auto')
        print(json.dumps(out))
        return
    # a contiguous block of rows (no interleave) of the same size as one 8-rank shard
    fr = device.make_frame(run.cam, run.bg, 50, 0, W, H, window=(0, 352, W, 100))
    out['rows352_451_64spp'] = round(rate(run.integ, fr, acc, W * 100, 64), 1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
