set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05h; mkdir -p $OUT
PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/variants/libptmi_rf16.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wf or wavefront or drain or bench_shapes or parity or edge" > $OUT/tests_rf16.log 2>&1; rc=$?
tail -3 $OUT/tests_rf16.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_runs.log
timeout -k 10 900 env AB_MODES=wf AB_REPS=3 bash tools/gpu_ab.sh > $OUT/ab_c3.log 2>&1; rc=$?; tail -8 $OUT/ab_c3.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_runs.log
timeout -k 10 900 env AB_MODES=wf AB_REPS=3 AB_SCENE=cornell_mesh_fog AB_WIDTH=1024 AB_SPP=32 bash tools/gpu_ab.sh > $OUT/ab_fog.log 2>&1; rc=$?; tail -8 $OUT/ab_fog.log
exit $rc
