"""GPU: the multi-GPU partition end to end with the HIP integrators, two ranks
sharing the box's one GPU over gloo (RCCL needs one GPU per rank; the driver's
8-GPU run uses it; tests/test_gpu_rccl.py runs the same collectives on RCCL at
world size 1). Each rank renders its shard through the C-ABI into a CUDA
accumulator and the product's ptmi.distributed.assemble_image — the collective
bench.py times, here through its gloo host-staging branch — assembles the
image on rank 0:
  * tiles   -> gather of owned rows, bit-identical to a one-rank render,
  * samples -> sum-reduce, equal to it up to f32 summation order.
Mirrors tests/test_distributed_gloo.py, which runs the same flow on the CPU oracle."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENE, WIDTH, SPS, STEPS = 'vol2_final_scene', 800, 4, 2


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, variant, out_path):
    import sys
    for p in (ROOT, os.path.join(ROOT, 'path-tracer-python_amd'), os.path.join(ROOT, 'tests')):
        sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from parity_helpers import scene_inputs
    from ptmi import device
    from ptmi.distributed import Shard, assemble_image
    sa, cam, bg = scene_inputs(SCENE, WIDTH)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    sh = Shard(rank, world, mode)
    fr = device.make_frame(cam, bg, 50, 0, W, H, band=sh.band())
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    render = integ.render_mk if variant == 'mk' else integ.render_wf
    for k in range(STEPS):
        b, c = sh.sample_range(k, SPS)
        render(fr, acc, b, c)
    torch.cuda.synchronize()
    assemble_image(acc, sh, dst=0)
    if rank == 0:
        np.save(out_path, acc.cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize('variant', ['mk', 'wf'])
@pytest.mark.parametrize('mode', ['tiles', 'samples'])
def test_two_rank_partition_on_gpu(tmp_path, mode, variant):
    import torch.multiprocessing as mp
    from parity_helpers import gpu_render
    out = str(tmp_path / f'{mode}_{variant}.npy')
    mp.start_processes(_worker, args=(2, _free_port(), mode, variant, out), nprocs=2, start_method='spawn')
    got = np.load(out)
    n = 2 if mode == 'samples' else 1
    # one rank: the same samples in the same per-step chunks
    chunks = [(k * SPS * n, SPS * n) for k in range(STEPS)]
    ref, _, _ = gpu_render(SCENE, WIDTH, variant, None, 0, 0, chunks=chunks)
    spp_total = SPS * STEPS * n
    if mode == 'tiles':
        assert np.array_equal(got, ref, equal_nan=True)
    else:
        assert np.allclose(got / spp_total, ref / spp_total, rtol=1e-5, atol=1e-6, equal_nan=True)
