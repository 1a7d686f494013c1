#!/bin/bash
# C3 evidence refresh (not product; round 3: after the fused wf_scatter, then its 5-wave build): bench line, rocprofv3 kernel trace + stats
# of the C3 bench command, the two traffic PMC passes, the wf_intersect VALU/latency passes.
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03c3
mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -n 1 $OUT/$n.log | cut -c 1-240; echo "=== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench_c3 300 python bench.py --preset c3
step trace_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o c3 -- python bench.py --preset c3 --no-cpu-baseline
step fetch_c3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o fetch_c3 -- python bench.py --preset c3 --steps 4 --no-cpu-baseline
step write_c3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc -o write_c3 -- python bench.py --preset c3 --steps 4 --no-cpu-baseline
step lat_wf_c3 400 env PMC_VARIANT=wf PMC_DIR=$OUT/pmc_latency_wf bash tools/gpu_pmc_latency.sh
echo done
