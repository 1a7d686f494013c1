#!/bin/bash
# Drain-consolidation A/B (experiment, not product): parity of the first
# variant, then tools/ab.py and tools/call_size.py timings of MIG_VARIANTS.
mkdir -p gpurun_out/mig
V=path-tracer-python_amd/ptmi/_lib/variants
set -- ${MIG_VARIANTS:-mig16s16}
PTMI_LIB=$PWD/$V/libptmi_$1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py -q -x --timeout 200 --timeout-method thread > gpurun_out/mig/parity_$1.log 2>&1
rc=$?; echo "parity $1 rc=$rc"; tail -2 gpurun_out/mig/parity_$1.log; [ $rc -le 1 ] || exit $rc
AB_VARIANTS="$*" AB_MODES=mk AB_REPS=3 bash tools/gpu_ab.sh || exit 1
for round in 1 2; do
  for lib in libptmi.so $(for v in "$@"; do echo variants/libptmi_$v.so; done); do
    PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/$lib CALL_SIZE_SPP=64,8 CALL_SIZE_SHARDS=8:4 timeout -k 10 200 python tools/call_size.py 2>&1 | grep '^{' | sed "s|^|$lib |" | tee -a gpurun_out/mig/call_size.log || exit 1
  done
done
