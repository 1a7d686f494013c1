"""Summarise an L1/L2 hit-rate rocprofv3 pass (tools/gpu_pmc_cache.sh) per kernel (not product)."""
import collections
import csv
import json
import sys


def summarise(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == 'TCC_HIT_sum':
            n[k] += 1
    out = {}
    for k, d in agg.items():
        if not k.startswith('ptmi::'):
            continue
        acc, l1m = d['TCP_TOTAL_CACHE_ACCESSES_sum'], d['TCP_TCC_READ_REQ_sum']
        hit, miss = d['TCC_HIT_sum'], d['TCC_MISS_sum']
        out[k] = {'dispatches': n[k], 'l1_accesses': acc, 'l1_read_misses': l1m,
                  'l1_hit_rate': round(1 - l1m / acc, 4) if acc else None,
                  'l2_hits': hit, 'l2_misses': miss,
                  'l2_hit_rate': round(hit / (hit + miss), 4) if hit + miss else None}
    return out


if __name__ == '__main__':
    print(json.dumps({p: summarise(p) for p in sys.argv[1:]}, indent=1))
