"""One process per GPU without an external launcher.

``python3 bench.py --gpus N`` (N > 1, no RANK in the environment) starts N
fresh worker processes of the same command line, each with RANK, LOCAL_RANK,
WORLD_SIZE, LOCAL_WORLD_SIZE and MASTER_ADDR/MASTER_PORT set as
``torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr
127.0.0.1`` would set them, and waits for them. The parent never touches the
GPU and never replaces itself (no exec): it only spawns, forwards rank 0's
standard output and reports the first failure.

The reference has no multi-device code at all (renderer.py:16 initialises
one Taichi device); this is the launcher of the N-GPU row-band partition
(ptmi.distributed).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time


def free_port(addr='127.0.0.1'):
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None, addr='127.0.0.1'):
    """The environment of worker `rank` (torch.distributed.run's variables)."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK='0', MASTER_ADDR=addr, MASTER_PORT=str(port))
    # dmabuf IPC only on this pool's driver: RCCL needs the non-legacy mode
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return env


def _pump(stream, sink, prefix, other=None):
    """Copy `stream` line by line to `sink`; with `other`, only the lines that
    are JSON objects go to `sink` and the rest (e.g. gloo's connection notes on
    stdout) to `other` with the prefix."""
    for line in iter(stream.readline, ''):
        if other is not None and not line.lstrip().startswith('{'):
            other.write(prefix + line)
            other.flush()
            continue
        sink.write(line if other is not None else prefix + line)
        sink.flush()
    stream.close()


def _stop(procs, grace_s=10.0):
    """SIGTERM each still-running worker's process group (each worker leads its
    own), then SIGKILL what is left after `grace_s`."""
    live = [p for p in procs if p.poll() is None]
    for p in live:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
    t_end = time.monotonic() + grace_s
    for p in live:
        try:
            p.wait(timeout=max(0.1, t_end - time.monotonic()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def launch_ranks(cmd, world, timeout_s=3600.0, out=None, err=None, poll_s=0.2):
    """Run `cmd` as `world` ranks; rank 0's JSON lines on stdout go to `out`
    (default sys.stdout), every other output to `err` (default sys.stderr)
    with a "[rank r] " prefix. Returns 0 when every rank exits 0; otherwise the
    first failing rank's exit code (a signal's 128 + signo), after stopping
    the others; 124 when `timeout_s` passes first."""
    out = out or sys.stdout
    err = err or sys.stderr
    port = free_port()
    procs, pumps = [], []
    try:
        for r in range(world):
            p = subprocess.Popen(cmd, env=rank_env(r, world, port), stdout=subprocess.PIPE,
                                 stderr=subprocess.PIPE, text=True, bufsize=1, start_new_session=True)
            procs.append(p)
            for s, sink, pre, other in ((p.stdout, out if r == 0 else err, f'[rank {r}] ', err if r == 0 else None),
                                        (p.stderr, err, f'[rank {r}] ', None)):
                t = threading.Thread(target=_pump, args=(s, sink, pre, other), daemon=True)
                t.start()
                pumps.append(t)
        t_end = time.monotonic() + timeout_s
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                err.write(f'[launch] rank {r} exited with {c}; stopping the other ranks\n')
                rc = 128 - c if c < 0 else c
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > t_end:
                err.write(f'[launch] timeout after {timeout_s:.0f} s; stopping the ranks\n')
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        _stop(procs)
        for t in pumps:
            t.join(timeout=5.0)
    return rc
