set -o pipefail
O=gpurun_out/bal; mkdir -p $O
for b in 8 4 2; do timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 8 --band-rows $b > $O/c2_b$b.json 2>&1 && tail -1 $O/c2_b$b.json || exit 1; done
timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 2 > $O/c2_r2.json 2>&1 && tail -1 $O/c2_r2.json
timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 4 > $O/c2_r4.json 2>&1 && tail -1 $O/c2_r4.json
timeout -k 10 200 python tools/shard_balance.py --preset c2 --ranks 1 > $O/c2_r1.json 2>&1 && tail -1 $O/c2_r1.json
