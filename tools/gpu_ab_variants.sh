#!/bin/bash
# Parity (GPU parity + edge tests) of every variant build, then the A/B timing
# of tools/gpu_ab.sh. Each step under its own timeout; stops on a crash.
set -u
shopt -s nullglob
mkdir -p gpurun_out
for lib in path-tracer-python_amd/ptmi/_lib/variants/*.so; do
  v=$(basename $lib .so)
  PTMI_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest ${AB_TESTS:-tests/test_gpu_parity.py tests/test_gpu_edge.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -2 gpurun_out/parity_$v.log; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 900 bash tools/gpu_ab.sh
