"""bench.py's own rank launcher (ptmi.launch): `python3 bench.py --gpus N` with
no torch.distributed.run environment starts N ranks itself, forwards rank 0's
JSON line and fails when a rank fails. CPU only (gloo ranks and stub
workers); tests/test_gpu_launch.py runs the real bench.py this way on a GPU."""
import io
import json
import os
import subprocess
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(ROOT, 'path-tracer-python_amd'))

from ptmi.launch import launch_ranks, rank_env  # noqa: E402

# A stand-in for one bench rank: the same environment contract, a gloo group,
# one all_gather of per-rank rows, rank 0 prints one JSON line.
WORKER = r'''
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group('gloo')
r, w = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ['RANK']) == int(os.environ['LOCAL_RANK'])
assert os.environ['MASTER_ADDR'] == '127.0.0.1'
t = torch.tensor([float(r), float(10 * r)], dtype=torch.float64)
out = [torch.zeros_like(t) for _ in range(w)]
dist.all_gather(out, t)
if r == 0:
    print(json.dumps({'world_size': w, 'ranks': [{'rank': int(o[0]), 'rows': int(o[1])} for o in out]}), flush=True)
dist.destroy_process_group()
'''


def test_rank_env_matches_torchrun_contract():
    env = rank_env(3, 8, 29500, base={'PATH': '/bin'})
    assert (env['RANK'], env['LOCAL_RANK'], env['WORLD_SIZE'], env['LOCAL_WORLD_SIZE']) == ('3', '3', '8', '8')
    assert (env['MASTER_ADDR'], env['MASTER_PORT'], env['GROUP_RANK']) == ('127.0.0.1', '29500', '0')
    assert env['HSA_ENABLE_IPC_MODE_LEGACY'] == '0' and env['PATH'] == '/bin'


def test_two_gloo_ranks_give_one_line():
    out, err = io.StringIO(), io.StringIO()
    rc = launch_ranks([sys.executable, '-c', WORKER], 2, timeout_s=120, out=out, err=err)
    assert rc == 0, err.getvalue()
    lines = [ln for ln in out.getvalue().splitlines() if ln.strip()]
    assert len(lines) == 1, out.getvalue()
    row = json.loads(lines[0])
    assert row['world_size'] == 2
    assert [r['rank'] for r in row['ranks']] == [0, 1] and [r['rows'] for r in row['ranks']] == [0, 10]


def test_failing_rank_stops_the_others():
    worker = ("import os, sys, time\n"
              "if os.environ['RANK'] == '1': sys.exit(3)\n"
              "time.sleep(300)\n")
    out, err = io.StringIO(), io.StringIO()
    t0 = time.monotonic()
    rc = launch_ranks([sys.executable, '-c', worker], 3, timeout_s=120, out=out, err=err)
    assert rc == 3
    assert time.monotonic() - t0 < 60  # the sleeping ranks were stopped, not waited for
    assert 'rank 1 exited with 3' in err.getvalue()


def test_timeout_stops_every_rank():
    out, err = io.StringIO(), io.StringIO()
    rc = launch_ranks([sys.executable, '-c', 'import time; time.sleep(300)'], 2, timeout_s=2, out=out, err=err)
    assert rc == 124 and 'timeout' in err.getvalue()


def test_bench_without_launcher_spawns_ranks_and_fails_loudly_without_gpu():
    """`python3 bench.py --gpus 2` with no RANK: the parent spawns two ranks
    (it does not exit with a world-size mismatch, round 5's behaviour); on this
    GPU-less host each rank refuses to render, so the parent exits non-zero and
    names the failing rank."""
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--dist-backend', 'gloo',
                        '--steps', '1', '--warmup', '0', '--no-cpu-baseline'], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode != 0
    assert '[launch] rank' in p.stderr and 'has 1 ranks' not in p.stderr + p.stdout
    assert p.stdout.strip() == ''  # no JSON line from a failed run
