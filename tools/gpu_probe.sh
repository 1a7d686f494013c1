#!/bin/bash
# Diagnostic probe builds (not product): counts (probe1) and wave timing (probe2)
set -u
mkdir -p gpurun_out
V=path-tracer-python_amd/ptmi/_lib/variants
for p in probe1 probe2; do
  for sc in "vol2_final_scene 800 8" "cornell_mesh_fog 1024 4"; do
    PTMI_LIB=$PWD/$V/libptmi_$p.so timeout -k 10 120 python tools/probe.py $sc 2>&1 | grep -v amdgpu.ids | sed "s/^/$p /" >> gpurun_out/probe.txt || exit 1
  done
done
