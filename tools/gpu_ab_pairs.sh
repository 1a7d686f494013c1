#!/bin/bash
# A/B of (library, host env) pairs: gpu_ab_pairs.sh "LIBNAME [ENV=...]" ...
# LIBNAME: libptmi (the build) or a variant name under _lib/variants; two
# interleaved rounds; AB_PARITY=1 runs the GPU parity tests for each pair first.
set -u
mkdir -p gpurun_out
L=path-tracer-python_amd/ptmi/_lib
run_pair() {  # run_pair "LIB ENV..." CMD...
  local pr=$1; shift
  local lib=${pr%% *} envs=""
  [ "$lib" != "$pr" ] && envs=${pr#* }
  local path=$PWD/$L/variants/$lib.so
  [ "$lib" = libptmi ] && path=$PWD/$L/libptmi.so
  env PTMI_LIB=$path $envs "$@"
}
pairs=("$@")
if [ "${AB_PARITY:-0}" = 1 ]; then
  for pr in "${pairs[@]}"; do
    run_pair "$pr" timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x >> gpurun_out/ab_parity.log 2>&1
    rc=$?; echo "parity [$pr] rc=$rc" >> gpurun_out/ab_pairs.log; [ $rc -eq 0 ] || exit 1
  done
fi
for round in 1 2; do
  for v in ${AB_MODES:-mk wf}; do
    for pr in "${pairs[@]}"; do
      run_pair "$pr" timeout -k 10 120 python tools/ab.py $v ${AB_SPP:-64} ${AB_REPS:-4} ${AB_SCENE:-vol2_final_scene} ${AB_WIDTH:-800} > /tmp/ab_one.log 2>&1 || { echo "[$pr] $v failed" >> gpurun_out/ab_pairs.log; exit 1; }
      grep Msamples /tmp/ab_one.log | sed "s/^/[$pr] /" >> gpurun_out/ab_pairs.log
    done
  done
done
