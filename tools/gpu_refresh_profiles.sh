#!/bin/bash
# Round-end evidence refresh (not product): kernel trace + stats of the default
# bench command, the two HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE: they do
# not fit one gfx950 TCC pass) and the VALU/latency passes of
# tools/gpu_pmc_latency.sh. Every step under its own time limit; stop on failure.
set -u
OUT=gpurun_out/refresh
mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -n 3 $OUT/$n.log; echo "=== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench 300 python bench.py
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c2 -- python bench.py --no-cpu-baseline
step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o fetch -- python bench.py --steps 4 --no-cpu-baseline
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc -o write -- python bench.py --steps 4 --no-cpu-baseline
step pmclat 600 bash tools/gpu_pmc_latency.sh
