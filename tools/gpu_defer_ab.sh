# leaf deferral in the mesh-scene megakernels (PTMI_MK_DEFER 4 / 8 / 12) vs HEAD (off): parity of the
# C4 bench shapes with each variant, then C4 A/B, two interleaved rounds
set -o pipefail
O=gpurun_out/defer; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for d in 4 8 12; do
PTMI_LIB=$V/libptmi_d$d.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread -k "c4 or edge or deep" > $O/tests_d$d.log 2>&1 || { echo TESTS_FAIL d$d; grep -E "FAILED|Error|^E " $O/tests_d$d.log | head -20; exit 1; }
tail -1 $O/tests_d$d.log
done
for r in 1 2; do
for lib in base d4 d8 d12; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
