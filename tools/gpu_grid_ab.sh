# persistent megakernel grid size (one-wave blocks per CU: 20 = the occupancy limit, 14 / 10 / 7)
# x overlap depth (2 / 3), overlapped 16-call runs: full frame at 64 and 8 spp, one 8-rank shard at 64 spp
set -o pipefail
O=gpurun_out/grid; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base w14 w10 w7; do
for d in 2 3; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  PTMI_OVERLAP_DEPTH=$d CALL_SIZE_SPP=64,8 CALL_SIZE_SHARDS=8:4 timeout -k 10 120 python tools/call_size.py >> $O/ab.log 2>&1 || exit 1
done; done; done
unset PTMI_LIB
cat $O/ab.log | grep full_
