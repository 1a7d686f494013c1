# spilled wf_intersect stacks (11 LDS slots, 7 waves/SIMD) with larger pipe grids: 4096 (HEAD) / 6144 / 8192
# blocks over the 4 pipes, 6144 with 9 LDS slots; vs all slots in LDS at 4096 (nospill); C3 and mesh fog, 2 rounds
set -o pipefail
O=gpurun_out/wfspill2; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base nospill b6 b8 b6l9; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$PWD/$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
