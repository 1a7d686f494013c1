# final check at HEAD: the full GPU suite, smoke(), and the default bench line
set -o pipefail
O=gpurun_out/final2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || { tail $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c 1-200
