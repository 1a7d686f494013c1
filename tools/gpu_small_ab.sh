# fetch sizing for small (sharded) calls: 8-rank rehearsal + full frame, per library variant
set -o pipefail
O=gpurun_out/smallab; mkdir -p $O; : > $O/ab.log
for r in 1 2; do
for v in base td1 td2 cs8; do
  if [ $v = base ]; then unset PTMI_LIB; else export PTMI_LIB=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$v.so; fi
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 8 --repeat 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$v', 'pred8', d['predicted_value_Msamples_s'], 'per_gpu', min(d['per_gpu_Msamples_s']))" >> $O/ab.log || exit 1
  timeout -k 10 120 python tools/ab.py mk 64 4 2>/dev/null | tail -1 >> $O/ab.log || exit 1
done; done
unset PTMI_LIB
cat $O/ab.log
