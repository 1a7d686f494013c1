# wavefront knob sweep (HEAD base vs variants), two interleaved rounds
set -o pipefail
O=gpurun_out/wfknobs; mkdir -p $O; : > $O/ab.log
for r in 1 2; do
for v in base cap20 cap22 blk256 blk64 unr2 unr4; do
  export PTMI_LIB=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$v.so
  timeout -k 10 120 python tools/ab.py wf 64 3 2>/dev/null | tail -1 >> $O/ab.log || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 2 cornell_mesh_fog 1024 2>/dev/null | tail -1 >> $O/ab.log || exit 1
done; done
unset PTMI_LIB
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/wfknobs/ab.log'):
    r = json.loads(l); d[(r['lib'], r['scene'])].append(r['Msamples_s'])
for k, v in sorted(d.items()): print(k, v)
PY
