# leaf-deferring kernels: (shading threshold, deferral threshold) sweep vs HEAD (16, 12); C4 and cornell_box, two rounds
set -o pipefail
O=gpurun_out/dsweep; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base s20d12 s20d16 s24d16 s24d12 s20d8; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 64 4 cornell_box 600 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
