#!/bin/bash
# A/B all variant builds + default, two interleaved rounds; each run under its
# own timeout. AB_PARITY=1 also runs the GPU parity tests against each variant.
set -u
shopt -s nullglob
mkdir -p gpurun_out
# AB_VARIANTS="a b": only variants/libptmi_{a,b}.so (default: every variant)
if [ -n "${AB_VARIANTS:-}" ]; then
  libs=(path-tracer-python_amd/ptmi/_lib/libptmi.so)
  for n in $AB_VARIANTS; do libs+=(path-tracer-python_amd/ptmi/_lib/variants/libptmi_$n.so); done
else
  libs=(path-tracer-python_amd/ptmi/_lib/libptmi.so path-tracer-python_amd/ptmi/_lib/variants/*.so)
fi
if [ "${AB_PARITY:-0}" = 1 ]; then
  for lib in "${libs[@]}"; do
    PTMI_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x >> gpurun_out/ab_parity.log 2>&1
    rc=$?; echo "parity $(basename $lib) rc=$rc"; [ $rc -le 1 ] || exit $rc
  done
fi
for round in 1 2; do
  for v in ${AB_MODES:-mk wf}; do
    for lib in "${libs[@]}"; do
      PTMI_LIB=$PWD/$lib timeout -k 10 120 python tools/ab.py $v ${AB_SPP:-64} ${AB_REPS:-4} ${AB_SCENE:-vol2_final_scene} ${AB_WIDTH:-800} >> gpurun_out/ab_runs.log 2>&1 || { echo "$lib $v failed rc=$?"; exit 1; }
    done
  done
done
cp gpurun_out/ab_runs.log /tmp/ab_copy.log; grep -h Msamples /tmp/ab_copy.log
