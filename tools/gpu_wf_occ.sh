# occupancy sensitivity of wf_intersect (A/B probe): unused LDS slots lower it from 5 waves/SIMD to 4 (p4)
# and 3 (p10); C3 shape (64 spp) and mesh fog, two rounds, with per-kernel busy times from bench.py --preset c3
set -o pipefail
O=gpurun_out/wfocc; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base p4 p10; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$PWD/$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
