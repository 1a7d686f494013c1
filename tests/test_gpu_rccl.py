"""GPU: the RCCL code path of the multi-GPU bench, run on the box's one GPU
before the driver's 8-GPU run does. A fresh child process
creates a `nccl` process group (RCCL) at world size 1 with device_id=cuda:0,
exactly as bench.py does for --gpus N, and runs every collective bench.py
makes on device tensors: the gather of owned row bands inside
ptmi.distributed.assemble_image (tiles), its sum-reduce (samples),
gather_ranks' all_gather and max_over_ranks' all_reduce(MAX) of float64. Then
bench.py itself runs with --gpus 1 --dist-backend nccl, so the whole N-rank
flow (process group, barriers, timed gather, per-rank rows) executes on RCCL.
The reference is single-device (renderer.py:16): no collective to mirror."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, socket, sys
sys.path[:0] = [ROOT, os.path.join(ROOT, 'path-tracer-python_amd')]
with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1')
import torch
import torch.distributed as dist
from ptmi.distributed import Shard, assemble_image, gather_ranks, max_over_ranks
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
dist.init_process_group('nccl', device_id=dev)
res = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
g = torch.Generator(device='cpu').manual_seed(5)
img = torch.randn((800, 800, 3), generator=g).to(dev)
for mode in ('tiles', 'samples'):
    acc = img.clone()
    assemble_image(acc, Shard.balanced(0, 1, mode, 800), dst=0)
    torch.cuda.synchronize()
    res[mode] = bool(torch.equal(acc, img))
res['ranks'] = gather_ranks([0, 800, 40960000, 0.25], dev)
res['max'] = max_over_ranks(1.5, dev)
dist.barrier()
dist.destroy_process_group()
print('RESULT ' + json.dumps(res), flush=True)
'''.replace('ROOT', repr(ROOT))


def _child_env():
    env = dict(os.environ)
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    return env


def test_rccl_collectives_at_world_size_one():
    p = subprocess.run([sys.executable, '-c', CHILD], cwd=ROOT, env=_child_env(), capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [x for x in p.stdout.splitlines() if x.startswith('RESULT ')][-1]
    res = json.loads(line[len('RESULT '):])
    assert res['backend'] == 'nccl' and res['world'] == 1
    assert res['tiles'] and res['samples']
    assert res['ranks'] == [[0.0, 800.0, 40960000.0, 0.25]] and res['max'] == 1.5


def test_bench_runs_the_multi_gpu_flow_on_rccl():
    p = subprocess.run([sys.executable, 'bench.py', '--gpus', '1', '--dist-backend', 'nccl', '--steps', '2',
                        '--warmup', '1', '--spp-per-step', '4', '--no-cpu-baseline'], cwd=ROOT, env=_child_env(),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    rec = json.loads([x for x in p.stdout.splitlines() if x.startswith('{')][-1])
    assert rec['world_size'] == 1 and rec['n_gpus'] == 1
    assert rec['collectives']['backend'] == 'nccl' and rec['collectives']['world_size'] == 1
    assert len(rec['ranks']) == 1 and rec['ranks'][0]['samples'] == 800 * 800 * 4 * 2
    assert rec['value'] > 0
