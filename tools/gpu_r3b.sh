set -o pipefail
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not bench_shapes" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail $O/bench_c2.err; exit 1; }
cut -c1-400 $O/bench_c2.json
timeout -k 10 300 python tools/shard_balance.py --preset c2 --ranks 8 > $O/bal_c2_8.json 2>&1 && cat $O/bal_c2_8.json
timeout -k 10 300 python tools/shard_balance.py --preset c5 --ranks 8 --steps 16 > $O/bal_c5_8.json 2>&1 && cat $O/bal_c5_8.json
