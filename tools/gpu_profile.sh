#!/bin/bash
# rocprofv3 evidence for the bench: kernel trace + stats, then PMC passes
# (separate runs; no trace domains mixed with --pmc).
set -u
mkdir -p gpurun_out/prof
run() { local n=$1; shift; echo "=== $n"; timeout -k 10 600 "$@" > gpurun_out/prof/$n.log 2>&1; local rc=$?; tail -3 gpurun_out/prof/$n.log; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 4 --no-cpu-baseline"
run trace_mk rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o mk -- $B --variant mk
run trace_wf rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o wf -- $B --variant wf
for v in mk wf; do
run pmc_sq_$v rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/prof -o pmc_sq_$v -- $B --variant $v
run pmc_wait_$v rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof -o pmc_wait_$v -- $B --variant $v
run pmc_fetch_$v rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof -o pmc_fetch_$v -- $B --variant $v
run pmc_write_$v rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof -o pmc_write_$v -- $B --variant $v
done
