set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05e; mkdir -p $OUT
PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/variants/libptmi_n64.so PTMI_NODE_ORDER=pairs timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread > $OUT/parity_n64_pairs.log 2>&1; rc=$?; tail -2 $OUT/parity_n64_pairs.log; [ $rc -eq 0 ] || exit $rc
PTMI_NODE_ORDER=bfs timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/parity_bfs.log 2>&1; rc=$?; tail -2 $OUT/parity_bfs.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT MODE=mk COMBOS="default:preorder default:bfs default:pairs n64:preorder n64:pairs" timeout -k 10 600 bash tools/gpu_ab_env.sh || exit 1
OUT=$OUT MODE=mk SCENE=cornell_mesh_fog WIDTH=1024 SPP=32 COMBOS="default:preorder default:bfs default:pairs n64:preorder n64:pairs tri4:preorder" timeout -k 10 600 bash tools/gpu_ab_env.sh || exit 1
OUT=$OUT MODE=wf COMBOS="default:preorder default:bfs default:pairs n64:preorder n64:pairs" timeout -k 10 600 bash tools/gpu_ab_env.sh || exit 1
