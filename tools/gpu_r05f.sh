set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05f; mkdir -p $OUT
rm -f gpurun_out/ab_runs.log
timeout -k 10 900 env AB_MODES=wf AB_REPS=3 bash tools/gpu_ab.sh > $OUT/ab_c3.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_runs.log
timeout -k 10 900 env AB_MODES=wf AB_REPS=3 AB_SCENE=cornell_mesh_fog AB_WIDTH=1024 AB_SPP=32 bash tools/gpu_ab.sh > $OUT/ab_fog.log 2>&1; rc=$?
exit $rc
