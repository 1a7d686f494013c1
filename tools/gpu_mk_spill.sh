# staged megakernels of 17-19 stack slots with the slots past 16 spilled to the workspace (HEAD) vs all in
# LDS (nospill); parity: the GPU suite on HEAD, the parity / edge / bench-shape subset on s4 (4 LDS slots:
# most pushes spill); then C4 (32 spp), cornell_box and C2 (unchanged kernel), two rounds; C4 bench line
set -o pipefail
O=gpurun_out/mkspill; mkdir -p $O; : > $O/ab.log
V=$PWD/path-tracer-python_amd/ptmi/_lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PTMI_LIB=$V/libptmi_s4.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or edge or bench_shapes or fullframe" > $O/tests_s4.log 2>&1 || { tail -30 $O/tests_s4.log; exit 1; }
tail -1 $O/tests_s4.log
for r in 1 2; do
for lib in base nospill; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
timeout -k 10 300 python bench.py --preset c4 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c 1-200
PTMI_LIB=$V/libptmi_nospill.so timeout -k 10 300 python bench.py --preset c4 --no-cpu-baseline > $O/bench_c4_nospill.log 2>&1 || { tail $O/bench_c4_nospill.log; exit 1; }
tail -1 $O/bench_c4_nospill.log | cut -c 1-200
