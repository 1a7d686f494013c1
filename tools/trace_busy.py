#!/usr/bin/env python3
"""GPU time per launch of one kernel from a rocprofv3 kernel trace (not product).

usage: trace_busy.py KERNEL_TRACE_CSV KERNEL_SUBSTR [SKIP]

rocprofv3 --stats averages each dispatch's own Start->End duration. When
launches of a kernel overlap in time (bench.py's pipelined megakernel calls:
two traces in flight on two streams), that average counts the shared time
twice. This prints both that average and the union of the dispatches'
[Start, End] intervals divided by the dispatch count, the figure bench.py
reports as roofline.avg_launch_ms (ptmi_prof_stop_busy over the timed
region). SKIP drops that many leading dispatches (bench.py's warm-up calls).
"""
import csv
import json
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    iv = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if sub in r['Kernel_Name']:
                iv.append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    iv.sort()
    iv = iv[skip:]
    own = sum(e - s for s, e in iv) / max(1, len(iv)) / 1e6
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
    print(json.dumps({'kernel': sub, 'dispatches': len(iv), 'avg_own_ms': round(own, 4),
                      'busy_ms_per_launch': round(busy / max(1, len(iv)) / 1e6, 4),
                      'busy_span_ms': round(busy / 1e6, 3)}))


if __name__ == '__main__':
    main()
