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
    assert set(bench.ALGO_BYTES) >= {'megakernel', 'wf_intersect', 'wf_scatter', 'wf_generate',
                                     'wf_resolve', 'mk_resolve'}


def test_valu_diagnostic_for_the_default_workload():
    v = bench.valu_diagnostic(_args([]), 'megakernel')
    assert v is not None and 0 < v['valu_issue_frac'] <= 1 and 0 < v['lane_efficiency'] <= 1


def test_multi_gpu_default_is_a_fixed_workload_tile_partition():
    """--gpus N: interleaved row bands of the fixed total workload (strong
    scaling, BASELINE.json configs[4]), total spp on the line."""
    from ptmi.distributed import Shard
    for preset, W, H, total in (('c2', 800, 800, 1024), ('c5', 3840, 2160, 4096)):
        a = _args(['--preset', preset, '--gpus', '8'])
        assert a.shard == 'tiles'
        spp, scaling, cfg = bench.describe(a, W, H, 8, Shard.balanced(0, 8, a.shard, H))
        assert spp == total == cfg['total_spp'] and scaling == 'strong'
        assert cfg['partition'] == 'tiles' and cfg['parallelism'].startswith('tiles-shard x8')
        assert f'@ {total} spp in total' in cfg['workload']
    a = _args(['--gpus', '8', '--shard', 'samples'])
    spp, scaling, _ = bench.describe(a, 800, 800, 8, Shard.balanced(0, 8, a.shard, 800))
    assert spp == 8 * 1024 and scaling == 'weak'


@pytest.mark.parametrize('H,world', [(800, 8), (800, 2), (800, 4), (2160, 8), (1024, 8), (225, 8), (7, 8)])
def test_balanced_bands_cover_every_row_once(H, world):
    import numpy as np
    from ptmi.distributed import Shard
    seen = np.zeros(H, np.int64)
    sizes = []
    for r in range(world):
        rows = Shard.balanced(r, world, 'tiles', H).rows(H)
        seen[rows] += 1
        sizes.append(len(rows))
    assert (seen == 1).all()
    best = -(-H // world)
    assert max(sizes) <= max(best * 1.01, best + 1) or H < world * 8


def test_cpu_baseline_records_the_host_and_times_the_whole_frame():
    """cpu_baseline (bench.py's CPU leg): the whole frame of the workload, the
    CPU model, os.cpu_count(), the allowed CPUs and the threads used."""
    sa, cam, bg, _ = bench.load_workload('wavefront_comparison', 400)
    r = bench.cpu_baseline(sa, cam, bg, 'wavefront_comparison', 'mk', 50, 0, 0.2)
    assert r['kind'] == 'port' and r['value'] > 0 and r['unit'] == 'Msamples/s'
    assert r['os_cpu_count'] >= r['affinity_cpus'] >= 1 and r['cores'] >= 1
    assert 'cpu_model' in r and 'the whole frame' in r['sample'] and '400x225' in r['sample']


@pytest.mark.parametrize('preset,kernel', [('c2', 'megakernel'), ('c3', 'wf_intersect'), ('c3', 'wf_scatter'),
                                           ('c4', 'megakernel'), ('c5', 'megakernel')])
def test_every_preset_has_a_valu_row_from_the_same_collection(preset, kernel):
    """The bench line's compute-side diagnostic exists for every preset's
    dominant kernel, and every traffic and VALU row the presets read names
    one and the same collection (the round's final kernel sources)."""
    v = bench.valu_diagnostic(_args(['--preset', preset]), kernel)
    assert v is not None and 0 < v['valu_issue_frac'] <= 1 and 0 < v['lane_efficiency'] <= 1
    src = v['source'].split(' ')[0].replace('{a,b,c}', 'a')
    assert os.path.exists(os.path.join(ROOT, src)), src
    import re
    heads = set()
    for p in ('c2', 'c3', 'c4', 'c5'):
        a = _args(['--preset', p])
        k = 'wf_intersect' if a.variant == 'wf' else 'megakernel'
        for s in (bench.measured_traffic(a, k)['source'], bench.valu_diagnostic(a, k)['source']):
            heads.update(re.findall(r'HEAD ([0-9a-f]{7,})', s))
    assert len(heads) == 1, heads


def test_wavefront_tail_segments_are_the_drains_units():
    """Segments the wavefront traced in its tail launch (counter [5]) are
    wf_drain's units, not wf_intersect's or wf_scatter's (ADVICE r04/r05:
    checked on the mapping itself with made-up counters)."""
    prof = {'wf_resolve': {'launches': 3}, 'mk_resolve': {'launches': 2}}
    seg, tail, samples, pix = 1_000_000, 12_345, 640_000, 640_000
    assert bench.kernel_units('wf_intersect', seg, tail, samples, pix, prof) == seg - tail
    assert bench.kernel_units('wf_scatter', seg, tail, samples, pix, prof) == seg - tail
    assert bench.kernel_units('wf_drain', seg, tail, samples, pix, prof) == tail
    assert bench.kernel_units('megakernel', seg, 0, samples, pix, prof) == samples
    assert bench.kernel_units('wf_resolve', seg, tail, samples, pix, prof) == 3 * pix
    assert bench.kernel_units('mk_resolve', seg, 0, samples, pix, prof) == 2 * pix
    # every kernel the roofline can name has a unit
    for k in bench.ALGO_BYTES:
        bench.kernel_units(k, seg, tail, samples, pix, prof)