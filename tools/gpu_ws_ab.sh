# overlapped megakernel calls: workspaces per side stream (1 = round-3 layout, 2) x overlap depth (2 / 3),
# with and without the fill launch ahead of each trace (variant "fill"); full frame at 64 and 8 spp,
# one 8-rank shard at 64 spp. The overlap tests first.
set -o pipefail
O=gpurun_out/wsab; mkdir -p $O; : > $O/ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "overlap or bench or host_state or staged" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=path-tracer-python_amd/ptmi/_lib/variants
for r in 1 2; do
for lib in base fill; do
for w in 1 2; do
for d in 2 3; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$V/libptmi_$lib.so; fi
  PTMI_OVERLAP_WS=$w PTMI_OVERLAP_DEPTH=$d CALL_SIZE_SPP=64,8 CALL_SIZE_SHARDS=8:4 timeout -k 10 120 python tools/call_size.py | sed "s/}/, \"ws\": $w}/" >> $O/ab.log 2>&1 || exit 1
done; done; done; done
unset PTMI_LIB
cat $O/ab.log
