set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r05i abtrace_default_wf abpmc_default_wf ablat_default_wf ta_wf ta_mk || exit 1
OUT=gpurun_out/r05i
for o in pairs bfs; do
  PTMI_NODE_ORDER=$o timeout -s KILL 240 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_ta -o mk_$o -- python tools/ab.py mk 32 1 > $OUT/ta_mk_$o.log 2>&1 || exit 1
  PTMI_NODE_ORDER=$o timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_cache -o mk_$o -- python tools/ab.py mk 32 1 > $OUT/cache_mk_$o.log 2>&1 || exit 1
done
timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_cache -o mk_preorder -- python tools/ab.py mk 32 1 > $OUT/cache_mk_preorder.log 2>&1 || exit 1
echo done
