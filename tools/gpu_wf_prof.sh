# per-kernel time of the wavefront, base vs HEAD library (rocprofv3 kernel trace + stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/wfprof; mkdir -p $O
PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/variants/libptmi_base.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o base -- python3 tools/ab.py wf 64 3 > $O/base.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o new -- python3 tools/ab.py wf 64 3 > $O/new.log 2>&1 || exit 1
for f in $(find $O -name "*kernel_stats.csv"); do echo $f; cut -d, -f1-4 $f | head -12; done
