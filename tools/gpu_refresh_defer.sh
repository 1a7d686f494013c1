#!/bin/bash
# Megakernel evidence refresh after leaf deferral in every megakernel (not product):
# bench lines C2/C4/C5, rocprofv3 kernel trace + stats of the C2 and C5 bench commands,
# the two traffic PMC passes per preset, the VALU/latency passes (C2, C4), the cache pass,
# then the full GPU suite. Every step under its own time limit; stop on failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03d
mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -n 1 $OUT/$n.log | cut -c 1-240; echo "=== $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench_c2 300 python bench.py
step bench_c4 300 python bench.py --preset c4 --no-cpu-baseline
step bench_c5 300 python bench.py --preset c5 --no-cpu-baseline
step trace_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o c2 -- python bench.py --no-cpu-baseline
step trace_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o c5 -- python bench.py --preset c5 --no-cpu-baseline
for p in c2 c4 c5; do
  step fetch_$p 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o fetch_$p -- python bench.py --preset $p --steps 4 --no-cpu-baseline
  step write_$p 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc -o write_$p -- python bench.py --preset $p --steps 4 --no-cpu-baseline
done
step lat_mk_c2 400 env PMC_VARIANT=mk PMC_DIR=$OUT/pmc_latency bash tools/gpu_pmc_latency.sh
step lat_mk_c4 400 env PMC_VARIANT=mk PMC_DIR=$OUT/pmc_latency_c4 PMC_SCENE_ARGS='cornell_mesh_fog 1024' bash tools/gpu_pmc_latency.sh
step cache_mk 200 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_cache -o mk -- python tools/ab.py mk 32 1
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
echo done
