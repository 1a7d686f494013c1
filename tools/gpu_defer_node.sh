# node deferral on top of leaf deferral: in a pass where >= 12 lanes pop a leaf test, a node step waits
# while fewer than K lanes have one (n4 / n8 / n16) vs HEAD; parity subset on n16; C2, C5 (8 spp), C4, 2 rounds
set -o pipefail
O=gpurun_out/dnode; mkdir -p $O; : > $O/ab.log
V=$PWD/path-tracer-python_amd/ptmi/_lib/variants
PTMI_LIB=$V/libptmi_n16.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or edge or bench_shapes" > $O/tests_n16.log 2>&1 || { tail -30 $O/tests_n16.log; exit 1; }
tail -1 $O/tests_n16.log
for r in 1 2; do
for lib in base n4 n8 n16; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 8 3 vol2_final_scene_comparison 3840 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
