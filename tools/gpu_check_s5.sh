# full GPU suite and the C3 bench line at HEAD (wf_scatter at 5 waves/SIMD)
set -o pipefail
O=gpurun_out/s5chk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --preset c3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c 1-200
