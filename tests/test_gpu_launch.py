"""`python3 bench.py --gpus 2` on the GPU box with no launcher environment:
bench.py starts its two ranks itself (ptmi.launch), here two gloo ranks
sharing the box's one GPU, prints one JSON line, and the row-band image it
assembles is bit-identical to the 1-GPU run of the same steps."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
ARGS = ['--preset', 'c2', '--spp-per-step', '2', '--steps', '2', '--warmup', '1', '--no-cpu-baseline']


def _bench(gpus, tmp_path, extra=()):
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
    npy = str(tmp_path / f'acc{gpus}.npy')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', str(gpus), *ARGS,
                        '--save-accum', npy, *extra], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), np.load(npy)


def test_bench_self_launches_two_ranks_bit_identical(tmp_path):
    one, a1 = _bench(1, tmp_path)
    two, a2 = _bench(2, tmp_path, ('--dist-backend', 'gloo'))
    assert one['n_gpus'] == 1 and two['n_gpus'] == 2 and two['world_size'] == 2
    assert [r['rank'] for r in two['ranks']] == [0, 1]
    assert sum(r['rows'] for r in two['ranks']) == a2.shape[0]
    assert two['collectives']['backend'] == 'gloo'
    assert a1.shape == a2.shape and a1.sum() > 0
    assert np.array_equal(a1, a2, equal_nan=True)
