set -o pipefail
O=gpurun_out/staging; mkdir -p $O; : > $O/ab.log
for r in 1 2; do for b in 1073741824 2147483648 4294967296; do
  PTMI_STAGING_BYTES=$b timeout -k 10 200 python bench.py --preset c5 --steps 64 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('c5 staging $b', d['value'])" >> $O/ab.log || exit 1
  PTMI_STAGING_BYTES=$b timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('c2 staging $b', d['value'])" >> $O/ab.log || exit 1
done; done
cat $O/ab.log
