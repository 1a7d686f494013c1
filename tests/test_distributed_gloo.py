"""World-size-2 multi-process test of the multi-GPU partition on CPU (gloo).

Each rank renders its shard with the CPU oracle standing in for its GPU (the
kernels themselves are covered by the -m gpu parity tests) and the product's
ptmi.distributed.assemble_image (the collective bench.py times) assembles
the image on rank 0:
  * tiles   -> a gather of owned row bands, bit-identical to the
               single-device render,
  * samples -> a sum-reduce, equal up to f32 summation order.
bench.py's own bookkeeping (balanced bands, the band gather it times,
gather_ranks, value) is run at world sizes 2, 4 and 8.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCENE, WIDTH, SPS, STEPS = 'vol2_final_scene', 64, 2, 2


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, out_path):
    import sys
    for p in (ROOT, os.path.join(ROOT, 'path-tracer-python_amd'), os.path.join(ROOT, 'tests')):
        sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from parity_helpers import oracle_render
    from ptmi import device
    from ptmi.distributed import Shard, assemble_image
    sh = Shard(rank, world, mode, band_rows=8)
    H = WIDTH
    acc = np.zeros((H, WIDTH, 3), np.float32)
    rows = sh.rows(H)
    for k in range(STEPS):
        b, c = sh.sample_range(k, SPS)
        # render exactly the rows the frame's band selects
        for r in rows:  # accumulate in place: same per-pixel float order as one device
            oracle_render(SCENE, WIDTH, 'mk', (0, r, WIDTH, 1), b, c, threads=1, acc=acc)
    t = torch.from_numpy(acc)
    assemble_image(t, sh, dst=0)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize('mode', ['tiles', 'samples'])
def test_two_rank_partition(tmp_path, mode):
    from parity_helpers import oracle_render
    out = str(tmp_path / f'{mode}.npy')
    mp.start_processes(_worker, args=(2, _free_port(), mode, out), nprocs=2, start_method='spawn')
    got = np.load(out)
    spp_total = SPS * STEPS * (2 if mode == 'samples' else 1)
    ref, _ = oracle_render(SCENE, WIDTH, 'mk', (0, 0, WIDTH, WIDTH), 0, spp_total)
    if mode == 'tiles':
        assert np.array_equal(got, ref, equal_nan=True)
    else:
        assert np.allclose(got / spp_total, ref / spp_total, rtol=1e-5, atol=1e-6, equal_nan=True)


def _bench_worker(rank, world, port, out_path):
    """bench.py's multi-rank bookkeeping on gloo: the balanced tile partition,
    the per-rank rows gathered to every rank (gather_ranks), the world size
    the JSON line records; each rank's rows rendered by the oracle standing in
    for its GPU, reduced onto rank 0."""
    import json
    import sys
    for p in (ROOT, os.path.join(ROOT, 'path-tracer-python_amd'), os.path.join(ROOT, 'tests')):
        sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    from parity_helpers import oracle_render
    from ptmi.distributed import Shard, assemble_image
    a = bench.parse(['--preset', 'c2', '--gpus', str(world), '--width', str(WIDTH), '--spp-per-step', str(SPS),
                     '--steps', str(STEPS), '--dist-backend', 'gloo'])
    H = WIDTH
    sh = Shard.balanced(rank, world, a.shard, H)
    acc = np.zeros((H, WIDTH, 3), np.float32)
    rows = sh.rows(H)
    for k in range(STEPS):
        b, c = sh.sample_range(k, SPS)
        for r in rows:
            oracle_render(SCENE, WIDTH, 'mk', (0, r, WIDTH, 1), b, c, threads=1, acc=acc)
    ranks = bench.gather_ranks([rank, len(rows)], 'cpu', world)
    total_spp, scaling, cfg = bench.describe(a, WIDTH, H, world, sh)
    t = torch.from_numpy(acc)
    assemble_image(t, sh, dst=0)  # the collective bench.py times
    if rank == 0:
        np.save(out_path, t.numpy())
        with open(out_path + '.json', 'w') as f:
            json.dump({'world_size': dist.get_world_size(), 'ranks': ranks, 'total_spp': total_spp,
                       'scaling': scaling, 'config': cfg}, f)
    dist.destroy_process_group()


def test_bench_tile_partition_two_ranks(tmp_path):
    import json
    out = str(tmp_path / 'bench_tiles.npy')
    mp.start_processes(_bench_worker, args=(2, _free_port(), out), nprocs=2, start_method='spawn')
    with open(out + '.json') as f:
        rec = json.load(f)
    assert rec['world_size'] == 2 and [int(r[0]) for r in rec['ranks']] == [0, 1]
    assert sum(int(r[1]) for r in rec['ranks']) == WIDTH  # every row on exactly one rank
    assert rec['config']['partition'] == 'tiles' and rec['scaling'] == 'strong'
    assert rec['total_spp'] == SPS * STEPS
    ref, _ = oracle_render_full()
    assert np.array_equal(np.load(out), ref, equal_nan=True)  # bit-identical to one device


def oracle_render_full():
    from parity_helpers import oracle_render
    return oracle_render(SCENE, WIDTH, 'mk', (0, 0, WIDTH, WIDTH), 0, SPS * STEPS)


def _bookkeeping_worker(rank, world, port, height, width, out_path):
    """bench.py's tiles bookkeeping at the BASELINE heights on gloo: balanced
    bands (Shard.balanced), each rank's owned rows filled with the one-rank
    image (a seeded stand-in: the kernels are covered by the -m gpu tests and
    rendering 800 or 2160 rows with the oracle would take minutes), the image
    assembled by ptmi.distributed.assemble_image (the gather bench.py times),
    per-rank rows gathered (gather_ranks), value = all samples / max wall."""
    import json
    import sys
    for p in (ROOT, os.path.join(ROOT, 'path-tracer-python_amd'), os.path.join(ROOT, 'tests')):
        sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    from ptmi.distributed import Shard, assemble_image, max_over_ranks
    a = bench.parse(['--preset', 'c2', '--gpus', str(world), '--dist-backend', 'gloo'])
    sh = Shard.balanced(rank, world, a.shard, height)
    img = np.random.default_rng(7).standard_normal((height, width, 3)).astype(np.float32)
    acc = np.zeros_like(img)
    rows = sh.rows(height)
    acc[rows] = img[rows]
    t = torch.from_numpy(acc)
    assemble_image(t, sh, dst=0)
    elapsed_rank = 1.0 + 0.125 * rank  # per-rank wall times; the slowest sets value
    samples_rank = width * len(rows) * a.spp_per_step * a.steps
    ranks = bench.gather_ranks([rank, len(rows), samples_rank, elapsed_rank], 'cpu', world)
    elapsed = max_over_ranks(elapsed_rank)
    value = bench.throughput(width * height * a.spp_per_step * a.steps, elapsed)
    _, scaling, cfg = bench.describe(a, width, height, world, sh)
    if rank == 0:
        np.save(out_path, t.numpy())
        with open(out_path + '.json', 'w') as f:
            json.dump({'ranks': ranks, 'value': value, 'elapsed': elapsed, 'band': sh.band_rows,
                       'scaling': scaling, 'parallelism': cfg['parallelism'], 'spp': a.spp_per_step * a.steps}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize('world, height', [(4, 800), (8, 800), (4, 2160), (8, 2160)])
def test_bench_tiles_bookkeeping_at_scale(tmp_path, world, height):
    """World sizes 4 and 8 at 800 and 2160 rows: every row assembled on rank 0
    exactly once and bit-identical to the one-rank image, balanced rows,
    value = samples / max-over-ranks wall time."""
    import json
    width = 8
    out = str(tmp_path / f'bk_{world}_{height}.npy')
    mp.start_processes(_bookkeeping_worker, args=(world, _free_port(), height, width, out), nprocs=world,
                       start_method='spawn')
    img = np.random.default_rng(7).standard_normal((height, width, 3)).astype(np.float32)
    assert np.array_equal(np.load(out), img)  # every row copied from its owner, no arithmetic
    with open(out + '.json') as f:
        rec = json.load(f)
    rows = [int(r[1]) for r in rec['ranks']]
    assert [int(r[0]) for r in rec['ranks']] == list(range(world)) and sum(rows) == height
    assert max(rows) - min(rows) <= rec['band']  # balanced to within one band
    if (world, height) == (8, 800):
        assert rec['band'] == 4 and rows == [100] * 8
    if (world, height) == (8, 2160):
        assert rec['band'] == 8 and max(rows) == 272
    want_elapsed = 1.0 + 0.125 * (world - 1)
    assert rec['elapsed'] == want_elapsed
    assert rec['value'] == width * height * rec['spp'] / want_elapsed / 1e6
    assert rec['scaling'] == 'strong' and 'gather of owned row bands' in rec['parallelism']


def _world_one_worker(rank, world, port, out_path):
    """A process group of one rank (bench.py --gpus 1 --dist-backend ...):
    every collective of the N-rank flow runs — the gather of assemble_image
    (tiles), its sum-reduce (samples), gather_ranks' all_gather and
    max_over_ranks' all_reduce — and leaves the one-rank values unchanged."""
    import json
    import sys
    for p in (ROOT, os.path.join(ROOT, 'path-tracer-python_amd'), os.path.join(ROOT, 'tests')):
        sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    from ptmi.distributed import Shard, assemble_image, max_over_ranks
    a = bench.parse(['--preset', 'c2', '--gpus', '1', '--dist-backend', 'gloo'])
    img = np.random.default_rng(3).standard_normal((37, 5, 3)).astype(np.float32)
    res = {'process_group': a.process_group, 'backend': a.dist_backend}
    for mode in ('tiles', 'samples'):
        sh = Shard.balanced(0, 1, mode, 37)
        t = torch.from_numpy(img.copy())
        assemble_image(t, sh, dst=0)
        res[mode] = bool(np.array_equal(t.numpy(), img))
    res['ranks'] = bench.gather_ranks([0, 37, 2.5], 'cpu', 1)
    res['max'] = max_over_ranks(1.25)
    with open(out_path, 'w') as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_collectives_run_at_world_size_one(tmp_path):
    import json
    out = str(tmp_path / 'w1.json')
    mp.start_processes(_world_one_worker, args=(1, _free_port(), out), nprocs=1, start_method='spawn')
    with open(out) as f:
        rec = json.load(f)
    assert rec['process_group'] is True and rec['backend'] == 'gloo'
    assert rec['tiles'] and rec['samples']
    assert rec['ranks'] == [[0.0, 37.0, 2.5]] and rec['max'] == 1.25


def test_bench_process_group_flag():
    import bench
    assert bench.parse(['--gpus', '1']).process_group is False
    assert bench.parse(['--gpus', '1', '--dist-backend', 'nccl']).process_group is True
    a = bench.parse(['--gpus', '2'])
    assert a.process_group is True and a.dist_backend == 'nccl'
