# wf_scatter at 5 waves/SIMD (<= 96 VGPRs, more scratch) vs 4 (HEAD); C3 and mesh fog, two rounds; parity subset on s5
set -o pipefail
O=gpurun_out/wfs5; mkdir -p $O; : > $O/ab.log
V=$PWD/path-tracer-python_amd/ptmi/_lib/variants
PTMI_LIB=$V/libptmi_s5.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or edge" > $O/tests_s5.log 2>&1 || { tail -30 $O/tests_s5.log; exit 1; }
tail -1 $O/tests_s5.log
for r in 1 2; do
for lib in base s5; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
