# wavefront intersect with independently progressing lanes (PTMI_WF_LANES, HEAD; refill at 16 busy lanes)
# vs the wave-synchronous slot loop (base), refill at 8 / 32: wavefront parity with HEAD, then C3 / mesh fog A/B
set -o pipefail
O=gpurun_out/wflanes; mkdir -p $O; : > $O/ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wf or wavefront or c3 or fullframe or edge or stackless or distributed" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base new r8 r32; do
  if [ $lib = new ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
