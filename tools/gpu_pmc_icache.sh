#!/bin/bash
# Instruction-cache PMC pass over one 32-spp launch of each integrator (diagnostic).
set -u
mkdir -p gpurun_out/pmcic
for V in mk wf; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmcic -o ${V}_ic -- python tools/ab.py $V 32 1 > gpurun_out/pmcic/${V}.log 2>&1
  rc=$?; echo "$V rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
