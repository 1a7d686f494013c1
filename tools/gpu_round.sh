#!/bin/bash
# GPU-box driver: each GPU step under its own timeout; stop on crash/timeout
# (exit codes other than 0/1), continue past plain test failures.
set -u
mkdir -p gpurun_out
step() {
  local name=$1; shift
  local t=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    parity) step parity 900 python -m pytest tests -m gpu -x -q -s ;;
    explore) step explore 600 python tools/gpu_explore.py ;;
    bench) step bench 600 python bench.py ;;
    benchmk) step benchmk 600 python bench.py --variant mk --no-cpu-baseline ;;
    benchwf) step benchwf 600 python bench.py --variant wf --no-cpu-baseline ;;
    benchc3) step benchc3 600 python bench.py --preset c3 ;;
    benchc4) step benchc4 600 python bench.py --preset c4 ;;
    benchc5) step benchc5 900 python bench.py --preset c5 --no-cpu-baseline ;;
    rocprof) step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py ;;
    rocprofwf) step rocprofwf 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o benchwf -- python bench.py --variant wf --no-cpu-baseline ;;
    traffic) step trafficf 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic -o fetch -- python bench.py --steps 4 --no-cpu-baseline && step trafficw 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic -o write -- python bench.py --steps 4 --no-cpu-baseline ;;
    trafficwf) step trafficwff 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic -o wffetch -- python bench.py --variant wf --steps 4 --no-cpu-baseline && step trafficwfw 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic -o wfwrite -- python bench.py --variant wf --steps 4 --no-cpu-baseline ;;
    trafficp) for pr in ${TRAFFIC_PRESETS:-c4 c5}; do
               step traffic${pr}f 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic -o ${pr}fetch -- python bench.py --preset $pr --steps 4 --no-cpu-baseline || exit 1
               step traffic${pr}w 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic -o ${pr}write -- python bench.py --preset $pr --steps 4 --no-cpu-baseline || exit 1
             done ;;
    ab) step ab 900 bash tools/gpu_ab.sh ;;
    counters) step counters 120 rocprofv3 -L ;;
    pmc) step pmc1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc -o pass1 -- python tools/ab.py mk 32 1 && step pmc2 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o pass2 -- python tools/ab.py mk 32 1 && step pmc3 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o pass3 -- python tools/ab.py mk 32 1 ;;
    pmcwf) for ps in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
                 "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LEVEL_WAVES SQ_INSTS_LDS" \
                 "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum" "TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum"; do
             n=$((${n:-0}+1)); step pmcwf$n 600 rocprofv3 --pmc $ps --output-format csv -d gpurun_out/pmcwf -o p$n -- python tools/ab.py wf 64 1 || exit 1
           done ;;
    pmcta) for v in ${PMC_MODES:-mk wf}; do n=0; for ps in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
                 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
                 "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
                 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
             n=$((n+1)); step pmcta_${v}$n 600 rocprofv3 --pmc $ps --output-format csv -d gpurun_out/pmcta -o ${v}$n -- python tools/ab.py $v 64 1 || exit 1
           done; done ;;
    dist2) step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 ;;
    dist2t) step dist2t 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --shard tiles ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $s" ;;
  esac
done
