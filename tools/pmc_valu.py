#!/usr/bin/env python3
"""VALU-side diagnostic of the megakernel from the committed PMC passes
(tools/gpu_pmc_latency.sh -> profiles/r01/pmc_latency/mk_{a,b,c}_counter_collection.csv),
for SURVEY.md §8(d)'s "report VALU utilization as a secondary diagnostic".

Per the largest mk_render_kernel dispatch of the run:
  cycles          = GRBM_GUI_ACTIVE / 8            (the counter sums the 8 XCDs)
  valu_issue_frac = 2 * SQ_INSTS_VALU / (1024 SIMDs * cycles)
                    (MI355X_MICROARCH.md: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles)
  lane_efficiency = SQ_THREAD_CYCLES_VALU / (64 * SQ_INSTS_VALU)
  wait_frac       = SQ_WAIT_ANY / SQ_WAVE_CYCLES,  issue_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
Writes profiles/valu.json[KEY] (KEY = scene:width:variant:kernel, as bench.py looks it up).
usage: pmc_valu.py [KEY] [DIR] [PREFIX] [KERNEL_SUBSTR]
PREFIX: the passes' file prefix (mk, wf); KERNEL_SUBSTR: the kernel (default
mk_render_kernel). A kernel launched many times (the wavefront's stages) is
summed over all its dispatches instead of taking the largest one (rocprofv3
serialises dispatches while it collects counters, so the sums are that
kernel's own)."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')


def main():
    key = sys.argv[1] if len(sys.argv) > 1 else 'vol2_final_scene:800:mk:megakernel'
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, 'profiles', 'r01', 'pmc_latency')
    prefix = sys.argv[3] if len(sys.argv) > 3 else 'mk'
    kern = sys.argv[4] if len(sys.argv) > 4 else 'mk_render_kernel'
    per = collections.defaultdict(dict)
    for p in 'abc':
        with open(os.path.join(d, f'{prefix}_{p}_counter_collection.csv')) as f:
            for r in csv.DictReader(f):
                if kern in r['Kernel_Name']:
                    c = per[(p, r['Dispatch_Id'])]
                    c[r['Counter_Name']] = c.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    v = {}
    for p in 'abc':
        runs = [c for (q, _), c in per.items() if q == p]
        if kern == 'mk_render_kernel':  # the largest dispatch of each pass (same launch in every pass)
            v.update(max(runs, key=lambda c: max(c.values())))
        else:  # every dispatch of the kernel
            tot = collections.Counter()
            for c in runs:
                tot.update(c)
            v.update(tot)
    cycles = v['GRBM_GUI_ACTIVE'] / 8
    out = {
        'valu_issue_frac': round(2 * v['SQ_INSTS_VALU'] / (1024 * cycles), 4),
        'lane_efficiency': round(v['SQ_THREAD_CYCLES_VALU'] / (64 * v['SQ_INSTS_VALU']), 4),
        'wave_wait_frac': round(v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES'], 4),
        'wave_issue_frac': round(v['SQ_ACTIVE_INST_ANY'] / v['SQ_WAVE_CYCLES'], 4),
        'valu_insts': v['SQ_INSTS_VALU'],
        'kernel_ms': round(cycles / 2.4e6, 3),
        'source': os.environ.get('PMC_SOURCE') or (
            os.path.relpath(d, ROOT) + f'/{prefix}_{{a,b,c}}_counter_collection.csv (tools/gpu_pmc_latency.sh: '
            f'tools/ab.py {prefix} 32 1, one 32-spp call; kernel {kern}); tools/pmc_valu.py'),
    }
    path = os.path.join(ROOT, 'profiles', 'valu.json')
    rows = {}
    if os.path.exists(path):
        with open(path) as f:
            rows = json.load(f)
    rows[key] = out
    with open(path, 'w') as f:
        json.dump(rows, f, indent=1, sort_keys=True)
    print(json.dumps({key: out}))


if __name__ == '__main__':
    main()
