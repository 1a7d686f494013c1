# round-end rehearsal at HEAD: smoke(), 2-rank gloo rehearsal of the multi-GPU bench (tiles), the default
# bench line (C2, with the committed PMC summaries), C3 and C5 bench lines
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 8 > $O/dist2.json 2> $O/dist2.err || { echo DIST_FAIL; tail -20 $O/dist2.err; exit 1; }
tail -1 $O/dist2.json | cut -c 1-300
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || { tail $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c 1-300
timeout -k 10 300 python bench.py --preset c3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c 1-200
timeout -k 10 300 python bench.py --preset c5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || { tail $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c 1-200
