# overlapped-call depth for full-frame calls: 2 (HEAD) vs 3 (PTMI_OVERLAP_DEPTH=3), bench.py C2 and C5, 3 rounds
set -o pipefail
O=gpurun_out/depth; mkdir -p $O; : > $O/ab.log
for r in 1 2 3; do
for d in 0 3; do
  for p in c2 c5; do
    PTMI_OVERLAP_DEPTH=$d timeout -k 10 300 python bench.py --preset $p --no-cpu-baseline > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
    echo "depth=$d preset=$p $(tail -1 $O/b.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')" >> $O/ab.log
  done
done; done
cat $O/ab.log
