#!/usr/bin/env python3
"""Per-kernel A/B report of one gpu_check.sh run (not product): for each lib
name, joins the kernel trace (abtrace_<lib>), the FETCH / WRITE / cache passes
(abpmc_<lib>) and the VALU passes (ablat_<lib>) of tools/ab.py over the same
workload. FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md
"HBM"); lane efficiency = SQ_THREAD_CYCLES_VALU / (64 SQ_INSTS_VALU); wait =
SQ_WAIT_ANY / SQ_WAVE_CYCLES. Counters are summed over every dispatch of the
kernel (rocprofv3 serialises dispatches while collecting).
usage: wf_pmc_report.py RUN_DIR MODE LIB [LIB ...]   (e.g. gpurun_out/r05c wf default bins1)"""
import collections
import csv
import json
import os
import sys


def kname(r):
    return r['Kernel_Name'].split('(')[0].replace('void ', '').split('<')[0].replace('ptmi::', '')


def sums(path, counters=None):
    out = collections.defaultdict(collections.Counter)
    disp = collections.defaultdict(set)
    if not os.path.exists(path):
        return out, disp
    with open(path) as f:
        for r in csv.DictReader(f):
            if counters and r['Counter_Name'] not in counters:
                continue
            k = kname(r)
            out[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r['Dispatch_Id'])
    return out, disp


def trace(path):
    t = collections.defaultdict(lambda: [0, 0.0])
    if not os.path.exists(path):
        return t
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kname(r)
            t[k][0] += 1
            t[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
    return t


def report(d, mode, lib):
    tr = trace(os.path.join(d, 'abtrace', f'{lib}_{mode}_kernel_trace.csv'))
    fe, disp = sums(os.path.join(d, 'abpmc', f'{lib}_{mode}_fetch_counter_collection.csv'), {'FETCH_SIZE'})
    wr, _ = sums(os.path.join(d, 'abpmc', f'{lib}_{mode}_write_counter_collection.csv'), {'WRITE_SIZE'})
    ca, _ = sums(os.path.join(d, 'abpmc', f'{lib}_{mode}_cache_counter_collection.csv'))
    va = collections.defaultdict(collections.Counter)
    for p in 'abc':
        s, _ = sums(os.path.join(d, f'ablat_{lib}', f'{mode}_{p}_counter_collection.csv'))
        for k, c in s.items():
            va[k].update(c)
    rows = {}
    for k in sorted(set(tr) | set(fe)):
        n = len(disp.get(k, ())) or tr[k][0]
        f = 2 * fe[k]['FETCH_SIZE'] * 1024
        w = wr[k]['WRITE_SIZE'] * 1024
        c, v = ca[k], va[k]
        hit, miss = c['TCC_HIT_sum'], c['TCC_MISS_sum']
        acc, l1m = c['TCP_TOTAL_CACHE_ACCESSES_sum'], c['TCP_TCC_READ_REQ_sum']
        rows[k] = {
            'trace_launches': tr[k][0], 'trace_ms': round(tr[k][1], 3),
            'pmc_dispatches': n,
            'fetch_MB': round(f / 1e6, 2), 'write_MB': round(w / 1e6, 2),
            'l1_hit': round(1 - l1m / acc, 4) if acc else None,
            'l2_hit': round(hit / (hit + miss), 4) if hit + miss else None,
            'valu_insts': v['SQ_INSTS_VALU'],
            'lane_eff': round(v['SQ_THREAD_CYCLES_VALU'] / (64 * v['SQ_INSTS_VALU']), 4) if v['SQ_INSTS_VALU'] else None,
            'wait_frac': round(v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES'], 4) if v['SQ_WAVE_CYCLES'] else None,
            'vmem_rd': v['SQ_INSTS_VMEM_RD'],
        }
    return rows


def main():
    d, mode = sys.argv[1], sys.argv[2]
    print(json.dumps({lib: report(d, mode, lib) for lib in sys.argv[3:]}, indent=1))


if __name__ == '__main__':
    main()
