# probes at HEAD, then per-type leaf deferral (a pass with leaf tests of several primitive types runs only the
# most common type; a lane of another type waits while fewer than K lanes have its type; c8 / c16 / c64) vs HEAD on C2, C5 (8 spp) and C4, two rounds;
# parity subset on c64
set -o pipefail
O=gpurun_out/dcls; mkdir -p $O; : > $O/ab.log; rm -f gpurun_out/probe.txt
bash tools/gpu_probe.sh || exit 1
cp gpurun_out/probe.txt $O/probe.txt
V=path-tracer-python_amd/ptmi/_lib/variants
PTMI_LIB=$PWD/$V/libptmi_c64.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "parity or bench_shapes or edge" > $O/tests_c64.log 2>&1 || { tail -30 $O/tests_c64.log; exit 1; }
tail -1 $O/tests_c64.log
for r in 1 2; do
for lib in base c8 c16 c64; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$PWD/$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 8 3 vol2_final_scene_comparison 3840 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
cat $O/probe.txt | cut -c 1-900
grep Msamples $O/ab.log
