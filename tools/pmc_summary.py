#!/usr/bin/env python3
"""Sum rocprofv3 PMC counters per kernel: pmc_summary.py CSV [CSV ...] -> csv on stdout
(kernel, dispatches, counter, sum over dispatches)."""
import csv
import sys
from collections import defaultdict


def main():
    tot = defaultdict(float)
    disp = defaultdict(set)
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r['Kernel_Name'].split('(')[0].replace('void ', '')
                tot[(k, r['Counter_Name'])] += float(r['Counter_Value'])
                disp[k].add((path, r['Dispatch_Id']))
    print('kernel,dispatches,counter,sum_over_dispatches')
    for (k, c), v in sorted(tot.items()):
        print(f'"{k}",{len(disp[k])},{c},{v:.6g}')


if __name__ == '__main__':
    main()
