#!/usr/bin/env python3
"""Per-kernel summary of one rocprofv3 PMC pass (not product).

Usage: pmc_kernel_summary.py COUNTER_CSV COUNTER OUT_CSV

Reads a ``*_counter_collection.csv`` of one ``--pmc COUNTER`` pass, sums the
counter over each dispatch's rows (one row per XCD/instance), and writes one
line per kernel: dispatches, mean KiB per dispatch, total KiB (raw counter
values; pmc_traffic.py applies the gfx950 FETCH_SIZE correction). The
per-dispatch CSVs of the wavefront run are ~3 MB each and are not kept.
"""
import csv
import sys
from collections import defaultdict


def main():
    src, counter, out = sys.argv[1:4]
    per = defaultdict(float)
    name = {}
    with open(src) as f:
        for r in csv.DictReader(f):
            if r['Counter_Name'] != counter:
                continue
            d = r['Dispatch_Id']
            per[d] += float(r['Counter_Value'])
            name[d] = r['Kernel_Name']
    by_kernel = defaultdict(list)
    for d, v in per.items():
        by_kernel[name[d]].append(v)
    rows = sorted(by_kernel.items(), key=lambda kv: -sum(kv[1]))
    with open(out, 'w', newline='') as f:
        w = csv.writer(f, quoting=csv.QUOTE_MINIMAL)
        w.writerow(['Kernel_Name', 'Counter_Name', 'Dispatches', 'Mean_KiB_per_dispatch', 'Total_KiB'])
        for k, vals in rows:
            w.writerow([k, counter, len(vals), round(sum(vals) / len(vals), 3), round(sum(vals), 2)])
    print(f'{out}: {len(rows)} kernels')


if __name__ == '__main__':
    main()
