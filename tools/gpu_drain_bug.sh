#!/bin/bash
# Diagnostic (not product): the wavefront parity windows at two tail thresholds
# for each build in $LIBS (variants/libptmi_<name>.so; "default" = libptmi.so),
# trace records saved for the trace builds. Each build under its own time limit;
# the first failing step ends the script.
set -u
mkdir -p gpurun_out/drain_bug
for n in ${LIBS:-dr5 tr5 ti5 tr3 ti3}; do
  lib=path-tracer-python_amd/ptmi/_lib/libptmi.so
  [ "$n" = default ] || lib=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$n.so
  PTMI_LIB=$PWD/$lib timeout -k 10 ${STEP_S:-300} python -u tools/wf_drain_trace.py gpurun_out/drain_bug/$n.npz \
    ${REPS:-2} > gpurun_out/drain_bug/$n.log 2>&1
  rc=$?
  tail -n 1 gpurun_out/drain_bug/$n.log
  [ $rc -eq 0 ] || { echo "$n rc=$rc"; exit $rc; }
done
