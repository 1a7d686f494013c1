# wavefront knobs re-checked after the fused wf_scatter: 3 pipes, 2^22 slots, readback every 16 iterations,
# 2x blocks per pipe grid; vs HEAD; C3 and mesh fog, two rounds
set -o pipefail
O=gpurun_out/wfk2; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base p3 cap22 rb16 mb2x; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
