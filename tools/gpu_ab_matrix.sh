#!/bin/bash
# A/B matrix: every variant build (and the default) x every value of one host
# env knob (AB_ENV / AB_VALUES), over AB_WORKLOADS (scene:width:spp) and
# AB_MODES, two interleaved rounds; each run under its own timeout.
set -u
shopt -s nullglob
mkdir -p gpurun_out
libs=(path-tracer-python_amd/ptmi/_lib/libptmi.so path-tracer-python_amd/ptmi/_lib/variants/*.so)
for round in 1 2; do
  for w in ${AB_WORKLOADS:-vol2_final_scene:800:64}; do
    IFS=: read scene width spp <<< "$w"
    for m in ${AB_MODES:-mk}; do
      for lib in "${libs[@]}"; do
        for val in ${AB_VALUES:-x}; do
          echo -n "$(basename $lib) ${AB_ENV:-none}=$val " >> gpurun_out/ab_matrix.log
          env ${AB_ENV:-AB_NONE}=$val PTMI_LIB=$PWD/$lib timeout -k 10 180 python tools/ab.py $m $spp ${AB_REPS:-3} $scene $width >> gpurun_out/ab_matrix.log 2>&1 || { echo "failed rc=$?"; exit 1; }
        done
      done
    done
  done
done
grep Msamples gpurun_out/ab_matrix.log | sed 's/{"lib": "[^"]*", //'
