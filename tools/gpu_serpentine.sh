# serpentine band ownership: parity of the band partitions, then the 8-rank C2 rehearsal (both orders)
set -o pipefail
O=gpurun_out/serp; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_distributed.py tests/test_gpu_parity.py tests/test_host_abi.py -x -q --timeout 300 --timeout-method thread -k "partition or distributed or band or staged or host_abi" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for o in "" "--reverse" ""; do
timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 8 $o >> $O/bal8.json 2>&1 || { echo BAL_FAIL; exit 1; }
tail -1 $O/bal8.json | cut -c 160-700
done
timeout -k 10 200 python tools/shard_balance.py --preset c5 --ranks 8 --steps 16 >> $O/bal8.json 2>&1 && tail -1 $O/bal8.json | cut -c 160-700
