# where a small (8-GPU tile shard) megakernel call spends its time: kernel trace of the rehearsal
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/small; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bal -- python3 tools/shard_balance.py --preset c2 --ranks 8 --repeat 1 > $O/bal.log 2>&1 || exit 1
tail -1 $O/bal.log | cut -c 1-300
python3 tools/trace_busy.py $O/trace/bal_kernel_trace.csv mk_render_kernel || true
