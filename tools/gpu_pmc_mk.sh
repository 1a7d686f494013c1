#!/bin/bash
# PMC passes over one short megakernel render (tools/ab.py), one rocprofv3 run
# per pass; usage: gpu_pmc_mk.sh TAG [ab.py args...]
set -u
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
P=(
"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
"SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
"SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_INST_CYCLES_SALU TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d gpurun_out/pmc_$tag -o p$i -- python tools/ab.py "$@" > gpurun_out/pmc_$tag/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py gpurun_out/pmc_$tag/p*_counter_collection.csv > gpurun_out/pmc_$tag/summary.csv
