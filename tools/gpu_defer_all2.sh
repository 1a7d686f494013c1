# HEAD with every-leaf deferral in all megakernels: full GPU suite, C2/C4/C5 bench lines; then wavefront
# deferral A/B (traverse() DEFER 8 / 12 / 20 vs HEAD off), C3 / mesh fog, two rounds
set -o pipefail
O=gpurun_out/dall2; mkdir -p $O; : > $O/ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for p in c2 c4 c5; do
timeout -k 10 300 python bench.py --preset $p --no-cpu-baseline > $O/bench_$p.json 2>&1 || { echo BENCH_FAIL; tail $O/bench_$p.json; exit 1; }
tail -1 $O/bench_$p.json | cut -c 1-200
done
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base w8 w12 w20; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
