#!/bin/bash
# PMC passes behind DESIGN.md §5's latency reading of the megakernel (one
# rocprofv3 --pmc run per counter group; no trace domains mixed in).
set -u
V=${PMC_VARIANT:-mk}
D=${PMC_DIR:-gpurun_out/pmclat}  # PMC_SCENE_ARGS='cornell_mesh_fog 1024' profiles another scene
mkdir -p $D
run() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $D -o ${V}_$n -- python tools/ab.py $V 32 1 ${PMC_SCENE_ARGS:-} > $D/${V}_$n.log 2>&1; local rc=$?; echo "pass $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run a SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
run b SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY
run c SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM
