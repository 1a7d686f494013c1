# shading threshold of the deep (>16-slot) kernels with leaf deferral on: 12 / 20 / 24 vs 16 (HEAD), C4, two rounds
set -o pipefail
O=gpurun_out/sad; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base sad12 sad20 sad24; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
