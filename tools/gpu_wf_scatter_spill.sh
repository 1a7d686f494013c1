# wf_scatter with spilled stack slots: x16 (20-slot kernels keep 16 in LDS: 5 waves/SIMD), x13w6 (13 LDS slots,
# 6 waves/SIMD, 80 VGPRs) vs HEAD; parity subset on x7 (7 LDS slots: most medium-exit pushes spill) and x13w6;
# C3 and mesh fog, two rounds
set -o pipefail
O=gpurun_out/wfxs; mkdir -p $O; : > $O/ab.log
V=$PWD/path-tracer-python_amd/ptmi/_lib/variants
for v in x7 x13w6; do
PTMI_LIB=$V/libptmi_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or edge" > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
for r in 1 2; do
for lib in base x16 x13w6; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
