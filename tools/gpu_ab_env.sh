#!/bin/bash
# A/B of a host-side env knob: AB_ENV="NAME" AB_VALUES="0 1" over AB_MODES x AB_WORKLOADS
# (workload = scene:width:spp), two interleaved rounds, each run under its own timeout.
set -u
mkdir -p gpurun_out
for round in 1 2; do
  for w in ${AB_WORKLOADS:-vol2_final_scene:800:64}; do
    IFS=: read scene width spp <<< "$w"
    for m in ${AB_MODES:-mk wf}; do
      for val in ${AB_VALUES:-0 1}; do
        echo -n "$AB_ENV=$val " >> gpurun_out/ab_env.log
        env $AB_ENV=$val timeout -k 10 180 python tools/ab.py $m $spp ${AB_REPS:-3} $scene $width >> gpurun_out/ab_env.log 2>&1 || { echo "failed rc=$?"; exit 1; }
      done
    done
  done
done
cat gpurun_out/ab_env.log | grep Msamples
