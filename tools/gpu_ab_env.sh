#!/bin/bash
# A/B of (library build, PTMI_NODE_ORDER) pairs, two interleaved rounds (not
# product). Usage: OUT=... MODE=mk SCENE=... WIDTH=... SPP=... COMBOS="lib:order ..." bash tools/gpu_ab_env.sh
# lib = default | a variants/libptmi_<lib>.so name
set -u
mkdir -p "$OUT"
for round in 1 2; do
  for c in $COMBOS; do
    name=${c%%:*}; order=${c#*:}
    lib=path-tracer-python_amd/ptmi/_lib/libptmi.so; [ "$name" = default ] || lib=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$name.so
    PTMI_LIB=$PWD/$lib PTMI_NODE_ORDER=$order timeout -k 10 120 python tools/ab.py $MODE ${SPP:-64} ${REPS:-3} ${SCENE:-vol2_final_scene} ${WIDTH:-800} >> $OUT/ab_env_${MODE}_${SCENE:-vol2_final_scene}.log 2>&1 || { echo "$c failed"; exit 1; }
  done
done
grep -h Msamples $OUT/ab_env_${MODE}_${SCENE:-vol2_final_scene}.log
