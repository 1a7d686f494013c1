#!/usr/bin/env python3
"""Rehearsal of bench.py --gpus N on ONE GPU (evidence tool, not product).

Runs each rank's share of the bench workload (its interleaved row bands under
--shard tiles, or its sample shard under --shard samples) one rank after the
other on this GPU, with the bench's own call shape (bench.BenchRun), and
times each rank's K steps. With one process per GPU and no exchange before
the final reduce, the N-GPU wall time is about the slowest rank's time, so

    predicted value = total samples / max(rank time)

and max/mean of the rank times is the partition's load imbalance. Prints one
JSON line. Example: python tools/shard_balance.py --preset c5 --ranks 8 --steps 16
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'path-tracer-python_amd'))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--ranks', type=int, default=8)
    p.add_argument('--repeat', type=int, default=2, help='timed rounds over all ranks (min per rank kept)')
    p.add_argument('--band-rows', type=int, default=0, help='force this band height (default: Shard.balanced)')
    args, rest = p.parse_known_args()
    import torch
    import bench
    from ptmi import device
    from ptmi.distributed import Shard
    a = bench.parse(rest)
    run = bench.BenchRun(a, torch.device('cuda', 0))
    W, H, sps = run.W, run.H, run.sps
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    frames, shards = [], []
    for r in range(args.ranks):
        sh = Shard(r, args.ranks, a.shard, args.band_rows) if args.band_rows else \
            Shard.balanced(r, args.ranks, a.shard, H)
        shards.append(sh)
        frames.append(device.make_frame(run.cam, run.bg, a.max_depth, a.seed, W, H, band=sh.band(),
                                        traversal=a.traversal))

    def render(fr, s0):
        if a.variant == 'mk':
            run.integ.render_mk(fr, acc, s0, sps, overlap=not a.no_overlap)
        else:
            run.integ.render_wf(fr, acc, s0, sps)

    for r in range(args.ranks):  # warm-up (workspaces, streams)
        render(frames[r], shards[r].sample_range(0, sps)[0])
    torch.cuda.synchronize()
    times = [float('inf')] * args.ranks
    for _ in range(args.repeat):
        for r in range(args.ranks):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                render(frames[r], shards[r].sample_range(a.warmup + k, sps)[0])
            torch.cuda.synchronize()
            times[r] = min(times[r], time.perf_counter() - t0)
    rows = [len(sh.rows(H)) for sh in shards]
    samples = [W * n * sps * a.steps for n in rows]
    total = sum(samples) if a.shard == 'tiles' else samples[0] * args.ranks
    mean = sum(times) / len(times)
    print(json.dumps({
        'preset': a.preset, 'scene': a.scene, 'width': W, 'height': H, 'variant': a.variant,
        'partition': a.shard, 'ranks': args.ranks, 'band_rows': shards[0].band()[0],
        'steps': a.steps, 'spp_per_step': sps,
        'rank_rows': rows, 'rank_s': [round(t, 5) for t in times],
        'imbalance_max_over_mean': round(max(times) / mean, 4),
        'predicted_value_Msamples_s': round(total / max(times) / 1e6, 2),
        'per_gpu_Msamples_s': [round(s / t / 1e6, 2) for s, t in zip(samples, times)],
    }))


if __name__ == '__main__':
    main()
