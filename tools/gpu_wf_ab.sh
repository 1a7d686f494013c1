# wavefront A/B: per-material shade kernels (HEAD) vs the saved base library; parity first
set -o pipefail
O=gpurun_out/wfab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wf or wavefront or fullframe or bench_shapes or edge or random or stackless" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for lib in base new; do
  if [ $lib = base ]; then export PTMI_LIB=path-tracer-python_amd/ptmi/_lib/variants/libptmi_base.so; else unset PTMI_LIB; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o new -- python3 tools/ab.py wf 64 3 > $O/prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/wfab/prof/**/*kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:5]:
        print(f"  {r['Name'][:34]:34s} calls={r['Calls']:>6} total_ms={float(r['TotalDurationNs'])/1e6:8.2f} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2>&1 && tail -1 $O/bench_c2.json | cut -c1-180
