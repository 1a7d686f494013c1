#!/usr/bin/env python3
"""Diagnostic (not product): compare the wf_drain segment records of two trace
builds (tools/wf_drain_trace.py output). A record is keyed by the segment's
input state (item, meta = depth | wave << 8, rng counter); a segment is a
pure function of it, so two builds that both traced it must agree on its
closest hit and its continuation. Prints every disagreement, and the records
of a bad path chained through its segments.

usage: python tools/wf_drain_trace_diff.py GOOD.npz BAD.npz"""
import sys

import numpy as np

FIELDS = ('item', 'meta', 'ctr', 't', 'ref', 'go', 'ctr_out', 'meta_out', 'x', 'y', 'z', 'lane')


def fmt(r):
    f = dict(zip(FIELDS, (int(v) for v in r)))
    t = np.uint32(r[3]).view(np.float32)
    xyz = np.asarray(r[8:11], np.uint32).view(np.float32)
    return (f"item {f['item']} depth {f['meta'] & 255} wave {(f['meta'] >> 8) & 255} ctr {f['ctr']} | "
            f"t {t:.6g} ref {f['ref'] & 0xffffffff:#010x} go {f['go']} ctr_out {f['ctr_out'] if f['go'] else '-'} "
            f"meta_out {f['meta_out'] if f['go'] else '-'} {'thr' if f['go'] else 'colour'} {xyz} lane {f['lane'] & 63}")


def index(recs):
    d = {}
    for r in recs:
        d.setdefault((int(r[0]), int(r[1]), int(r[2])), []).append(r)
    return d


def main():
    good, bad = np.load(sys.argv[1]), np.load(sys.argv[2])
    gidx = {}  # per case (drain threshold and rep dropped: a segment's record does not depend on them)
    for k in good.files:
        if not k.endswith('|bad'):
            case = k.split('|')[1]
            for key, rs in index(good[k]).items():
                gidx.setdefault((case,) + key, rs[0])
    total = mism = unmatched = 0
    for k in bad.files:
        if k.endswith('|bad'):
            continue
        recs = bad[k]
        case = k.split('|')[1]
        idx = index(recs)
        dup = sum(len(v) > 1 for v in idx.values())
        n_m = 0
        for key, rs in idx.items():
            total += 1
            g = gidx.get((case,) + key)
            if g is None:
                unmatched += 1
                continue
            if not np.array_equal(g[3:11], rs[0][3:11]):
                mism += 1
                n_m += 1
                if n_m <= 6:
                    print(f'[{k}] MISMATCH\n  good: {fmt(g)}\n  bad:  {fmt(rs[0])}')
        print(f'[{k}] records {len(recs)} keys {len(idx)} duplicate keys {dup} mismatches {n_m}')
    print(f'total keys {total}, matched {total - unmatched}, mismatched {mism}')


if __name__ == '__main__':
    main()
