#!/bin/bash
# C4 evidence refresh after the leaf-deferring kernels (not product): bench line, rocprofv3 kernel
# trace + stats of the C4 bench command, the two traffic PMC passes, the VALU/latency passes.
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03c4
mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -n 1 $OUT/$n.log | cut -c 1-240; echo "=== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench_c4 300 python bench.py --preset c4
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o c4 -- python bench.py --preset c4 --no-cpu-baseline
step fetch_c4 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o fetch_c4 -- python bench.py --preset c4 --steps 4 --no-cpu-baseline
step write_c4 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc -o write_c4 -- python bench.py --preset c4 --steps 4 --no-cpu-baseline
step lat_mk_c4 400 env PMC_VARIANT=mk PMC_DIR=$OUT/pmc_latency_c4 PMC_SCENE_ARGS='cornell_mesh_fog 1024' bash tools/gpu_pmc_latency.sh
echo done
