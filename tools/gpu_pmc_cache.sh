set -u
mkdir -p gpurun_out/pmccache
for v in mk wf; do
  timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmccache -o $v -- python tools/ab.py $v 32 1 > gpurun_out/pmccache/$v.log 2>&1 || exit $?
done
