# full GPU suite + 2-rank gloo rehearsal of the multi-GPU bench + C2 bench
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|^E " $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 8 > $O/dist2.json 2> $O/dist2.err || { echo DIST_FAIL; tail -20 $O/dist2.err; exit 1; }
tail -1 $O/dist2.json | cut -c 1-600
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail $O/bench_c2.err; exit 1; }
tail -1 $O/bench_c2.json | cut -c 1-300
timeout -k 10 300 python bench.py --preset c4 > $O/bench_c4.json 2> $O/bench_c4.err || { echo BENCH_FAIL; tail $O/bench_c4.err; exit 1; }
tail -1 $O/bench_c4.json | cut -c 1-300
