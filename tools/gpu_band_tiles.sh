# Band-shaped megakernel tiles (16x4 for 4-row bands): parity at the bench's 8-rank partition,
# then the 8-rank C2 rehearsal, HEAD vs variants/libptmi_base.so (-DPTMI_MK_BAND_TILES=0), two rounds
set -o pipefail
O=gpurun_out/bandtiles; mkdir -p $O; : > $O/ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread -k "partition or distributed or full_frame" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for lib in base new; do
  if [ $lib = base ]; then export PTMI_LIB=path-tracer-python_amd/ptmi/_lib/variants/libptmi_base.so; else unset PTMI_LIB; fi
  echo "lib=$lib round=$r" >> $O/ab.log
  timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 8 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep -E "^lib|predicted" $O/ab.log | sed -E 's/.*"rank_s"/"rank_s"/' | cut -c 1-300
