#!/usr/bin/env python3
"""Per-launch HBM-side traffic of one kernel from rocprofv3 PMC passes.

Usage: pmc_traffic.py KEY KERNEL_SUBSTR FETCH_CSV WRITE_CSV [SOURCE]

FETCH_CSV / WRITE_CSV are rocprofv3 ``*_counter_collection.csv`` files of two
separate ``--pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` passes over the same
bench.py command (the two counters do not fit one gfx950 TCC pass). Counter
values are KiB. Per MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken
as is. Both count L2 -> fabric requests, so Infinity-Cache hits are included:
the figure is an upper bound on HBM bytes.

Writes profiles/traffic.json[KEY] = {bytes_per_launch, fetch_bytes, write_bytes,
dispatches, source}; KEY = scene:width:variant:spp_per_step:max_depth:kernel
(bench.py measured_traffic()).
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, kernel, counter):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter:
                d = r['Dispatch_Id']
                vals[d] = vals.get(d, 0.0) + float(r['Counter_Value'])
    return list(vals.values())


def main():
    key, kernel, fcsv, wcsv = sys.argv[1:5]
    source = sys.argv[5] if len(sys.argv) > 5 else f'{fcsv} + {wcsv}'
    fetch = per_dispatch(fcsv, kernel, 'FETCH_SIZE')
    write = per_dispatch(wcsv, kernel, 'WRITE_SIZE')
    if not fetch or not write:
        sys.exit(f'no {kernel} dispatches with FETCH_SIZE/WRITE_SIZE')
    fb = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    wb = 1024.0 * sum(write) / len(write)
    path = os.path.join(ROOT, 'profiles', 'traffic.json')
    try:
        with open(path) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        rows = {}
    rows[key] = {'bytes_per_launch': round(fb + wb), 'fetch_bytes': round(fb), 'write_bytes': round(wb),
                 'dispatches': [len(fetch), len(write)], 'source': source}
    with open(path, 'w') as f:
        json.dump(rows, f, indent=1, sort_keys=True)
    print(json.dumps({key: rows[key]}))


if __name__ == '__main__':
    main()
