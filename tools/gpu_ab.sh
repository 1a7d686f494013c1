#!/bin/bash
# A/B all variant builds + default; each under its own timeout.
set -u
shopt -s nullglob
mkdir -p gpurun_out
for v in ${AB_MODES:-mk wf}; do
  timeout -k 10 120 python tools/ab.py $v 64 3 >> gpurun_out/ab.log 2>&1 || { echo "default $v failed rc=$?"; exit 1; }
  for lib in path-tracer-python_amd/ptmi/_lib/variants/*.so; do
    PTMI_LIB=$PWD/$lib timeout -k 10 120 python tools/ab.py $v 64 3 >> gpurun_out/ab.log 2>&1 || { echo "$lib $v failed rc=$?"; exit 1; }
  done
done
cp gpurun_out/ab.log /tmp/ab_copy.log; grep -h Msamples /tmp/ab_copy.log
