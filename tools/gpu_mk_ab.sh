# megakernel A/B: HEAD library vs variants/libptmi_base.so (C2, C4, C5 shapes), two interleaved rounds
set -o pipefail
O=gpurun_out/mkab; mkdir -p $O; : > $O/ab.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or fullframe or edge" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for lib in base new; do
  if [ $lib = base ]; then export PTMI_LIB=path-tracer-python_amd/ptmi/_lib/variants/libptmi_base.so; else unset PTMI_LIB; fi
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
