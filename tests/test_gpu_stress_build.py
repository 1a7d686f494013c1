"""The register-budget stress build (libptmi_stress.so, PTMI_STRESS_WAVES=8 in
pt_device.hpp: every render kernel capped to the 8-wave VGPR budget, so the
kernels spill) renders the parity cases bit-identically to the oracle.

A legal register budget must not change a result. Round 5 found a wf_drain
build held to 5 waves/SIMD that rendered wrong pixels; round 6 traced it to
cont_position reading other lanes' registers after some lanes had branched
away (their registers undefined once spilled values are reloaded for the
active lanes only). This build makes such a dependence on
register allocation fail a test instead of waiting for a compiler change.
Each case runs in a child process (the library is loaded once per process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
STRESS = os.path.join(ROOT, 'path-tracer-python_amd', 'ptmi', '_lib', 'libptmi_stress.so')


def _env():
    assert os.path.exists(STRESS), 'libptmi_stress.so missing: run __graft_entry__.build()'
    return dict(os.environ, PTMI_LIB=STRESS)


def test_stress_build_parity_suite():
    """tests/test_gpu_parity.py (megakernel and wavefront windows, chunking,
    bands) with every kernel spilling."""
    p = subprocess.run([sys.executable, '-m', 'pytest', os.path.join(ROOT, 'tests', 'test_gpu_parity.py'), '-q', '-x',
                        '-p', 'no:cacheprovider'], env=_env(), capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]


def test_stress_build_wavefront_tail_windows(tmp_path):
    """Every wavefront parity window at the default tail threshold and with the
    tail launched as soon as the pool is dry (wf_drain traces the most paths):
    no pixel differs from the oracle (tools/wf_drain_trace.py)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'wf_drain_trace.py'), str(tmp_path / 't.npz'), '1'],
                       env=_env(), capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]
    rows = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{')]
    cases = [r for r in rows if 'case' in r]
    assert len(cases) >= 18 and {r['drain_at'] for r in cases} == {16, 1}
    bad = [(r['drain_at'], r['case'], r['n_bad'], r['linf']) for r in cases if r['n_bad'] or r['gpu'] != r['oracle']]
    assert not bad, bad


def test_stress_build_whole_frame_bench_calls():
    """One bench call over the whole frame (tests/test_gpu_bench_shapes.py: C2
    and C4 megakernel, C3 wavefront; 40.96 M, 33.6 M and 40.96 M paths) with
    every kernel spilling: every pixel and every device counter equal to the
    oracle's, as with the shipped build."""
    p = subprocess.run([sys.executable, '-m', 'pytest', os.path.join(ROOT, 'tests', 'test_gpu_bench_shapes.py'), '-q', '-x',
                        '-p', 'no:cacheprovider', '-k', 'one_bench_call_full_frame and (c2 or c3 or c4)'],
                       env=_env(), capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert '3 passed' in p.stdout, p.stdout[-2000:]
