set -o pipefail
O=gpurun_out/bal2; mkdir -p $O
for d in 2 3 4; do
PTMI_OVERLAP_DEPTH=$d timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 8 > $O/c2_d$d.json 2>&1 && tail -1 $O/c2_d$d.json | cut -c 1-80,330-700 || exit 1
PTMI_OVERLAP_DEPTH=$d timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_d$d.json 2>&1 && tail -1 $O/bench_d$d.json | cut -c 1-200 || exit 1
done
