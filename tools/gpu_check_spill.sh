# full GPU suite at HEAD (spilled wf_intersect stacks for 17-20-slot kernels), then the parity / edge /
# bench-shape subset on l3 (3 LDS slots in those kernels: most pushes spill), then the C3 bench line
set -o pipefail
O=gpurun_out/spillchk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/variants/libptmi_l3.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or edge or bench_shapes or fullframe" > $O/tests_l3.log 2>&1 || { tail -30 $O/tests_l3.log; exit 1; }
tail -1 $O/tests_l3.log
timeout -k 10 300 python bench.py --preset c3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c 1-200
