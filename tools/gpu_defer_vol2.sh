# vol2 with leaf deferral forced on (sphere tests only at 4 / 8 lanes; every leaf at 6 / 12) vs HEAD (off for scenes
# with spheres): C2 and C5 shapes, two rounds
set -o pipefail
O=gpurun_out/dvol2; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base s4 s8 a6 a12; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 8 3 vol2_final_scene_comparison 3840 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
