# tests touched this round + wavefront A/B (base vs isectnt)
set -o pipefail
O=gpurun_out/ab2; mkdir -p $O; : > $O/ab.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "bench_shapes or host_state" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in base isectnt; do
  export PTMI_LIB=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$v.so
  timeout -k 10 120 python tools/ab.py wf 64 3 2>/dev/null | tail -1 >> $O/ab.log || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 2 cornell_mesh_fog 1024 2>/dev/null | tail -1 >> $O/ab.log || exit 1
done; done
unset PTMI_LIB
cat $O/ab.log
