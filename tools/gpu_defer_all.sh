# leaf deferral for every scene (PTMI_MK_DEFER_ALL, threshold 12 / 6) vs HEAD (triangle scenes only):
# quad-only Cornell scenes and vol2, two interleaved rounds
set -o pipefail
O=gpurun_out/deferall; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base dall dall8; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py mk 64 4 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 64 4 cornell_smoke 600 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py mk 64 4 cornell_box 600 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log | cut -c 1-200
