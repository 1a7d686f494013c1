# megakernel knobs re-checked with every-leaf deferral: pops per pass 2 / 4, deferral 10 / 14, shading at 28 / 32,
# vs HEAD (3, 12, 24); C2, C5 and C4 shapes, two rounds
set -o pipefail
O=gpurun_out/mkk3; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base u2 u4 d10 d14 s28 s32; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 8 3 vol2_final_scene_comparison 3840 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 32 4 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
