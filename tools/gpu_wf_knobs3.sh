# wavefront knobs re-checked with the 5-wave wf_scatter: 2^22 queue slots (cap22), 3 pipes (p3), 6144-block
# pipe grids (mb6) vs HEAD; C3 and mesh fog, two rounds
set -o pipefail
O=gpurun_out/wfk3; mkdir -p $O; : > $O/ab.log
V=$PWD/path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base cap22 p3 mb6; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
