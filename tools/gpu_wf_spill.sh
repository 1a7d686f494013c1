# wf_intersect with its deeper stack slots spilled to global memory (LDS slots 11 = HEAD, 13, 9) vs all
# slots in LDS (nospill, the previous kernel); parity: the wavefront GPU tests on HEAD and on l3 (3 LDS
# slots: most pushes spill); then C3 (64 spp) and mesh fog, two rounds
set -o pipefail
O=gpurun_out/wfspill; mkdir -p $O; : > $O/ab.log
V=path-tracer-python_amd/ptmi/_lib/variants
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wf or wavefront or c3 or edge or parity" > $O/tests_head.log 2>&1 || { tail -30 $O/tests_head.log; exit 1; }
tail -1 $O/tests_head.log
PTMI_LIB=$PWD/$V/libptmi_l3.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wf or wavefront or c3 or edge or parity" > $O/tests_l3.log 2>&1 || { tail -30 $O/tests_l3.log; exit 1; }
tail -1 $O/tests_l3.log
for r in 1 2; do
for lib in base nospill l13 l9; do
  if [ $lib = base ]; then unset PTMI_LIB; else export PTMI_LIB=$PWD/$V/libptmi_$lib.so; fi
  timeout -k 10 120 python tools/ab.py wf 64 3 >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab.py wf 32 3 cornell_mesh_fog 1024 >> $O/ab.log 2>&1 || exit 1
done; done
unset PTMI_LIB
grep Msamples $O/ab.log
