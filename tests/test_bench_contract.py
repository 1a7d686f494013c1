"""CPU: bench.py's driver contract pieces that need no GPU: default workload
(BASELINE.json configs[1] at the north star's 1024 spp), the metric string,
and a committed PMC traffic figure for the dominant kernel of every preset
(profiles/traffic.json, read by measured_traffic)."""
import json
import os
import sys

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(argv):
    old = sys.argv
    sys.argv = ['bench.py'] + argv
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_default_is_configs1_at_1024_spp():
    a = _args([])
    assert (a.scene, a.width, a.variant, a.gpus) == ('vol2_final_scene', 800, 'mk', 1)
    assert a.spp_per_step * a.steps == 1024 and a.warmup >= 1


def test_metric_is_baselines():
    with open(os.path.join(ROOT, 'BASELINE.json')) as f:
        assert json.load(f)['metric'] == bench.METRIC


@pytest.mark.parametrize('preset,kernel', [('c2', 'megakernel'), ('c3', 'wf_intersect'), ('c4', 'megakernel'),
                                           ('c5', 'megakernel')])
def test_every_preset_has_measured_traffic(preset, kernel):
    a = _args(['--preset', preset, '--steps', '4'])
    t = bench.measured_traffic(a, kernel)
    assert t is not None and t['bytes_per_launch'] > 0
    src = t['source'].split(' ')[0].replace('{fetch,write}', 'fetch')
    assert os.path.exists(os.path.join(ROOT, src)), src


def test_algorithmic_bytes_cover_every_kernel_kind():
    assert set(bench.ALGO_BYTES) >= {'megakernel', 'wf_intersect', 'wf_shade', 'wf_medium', 'wf_generate',
                                     'wf_resolve', 'mk_resolve'}


def test_valu_diagnostic_for_the_default_workload():
    v = bench.valu_diagnostic(_args([]), 'megakernel')
    assert v is not None and 0 < v['valu_issue_frac'] <= 1 and 0 < v['lane_efficiency'] <= 1
