#!/bin/bash
# GPU check at HEAD (not product). Usage: bash tools/gpu_check.sh OUT [STEP ...]
# Steps (default: tests smoke c2 c3):
#   tests        full `pytest -m gpu` suite
#   smoke        __graft_entry__.smoke()
#   c2|c3|c4|c5  bench.py --preset <c> (one JSON line)
#   trace_<c>    rocprofv3 --kernel-trace --stats of the bench command
#   fetch_<c> / write_<c>   FETCH_SIZE / WRITE_SIZE PMC passes (4 steps)
#   dist2        2-rank gloo rehearsal of the multi-GPU bench on the one GPU
#   ab_wf_c3 / ab_wf_fog / ab_mk_c2 / ab_mk_c4 / ab_mk_c5
#                A/B timing (tools/gpu_ab.sh) of every variants/*.so against
#                the default build: wavefront on vol2 800x800 or the mesh-fog
#                scene, megakernel on C2 / C4 / C5 shapes
#                (WF_VARIANTS / MK_VARIANTS="a b": only variants/libptmi_{a,b}.so)
#   ab_wf_both   wavefront A/B (three calls per lib and round) on C3 and on the mesh-fog scene
#   wftests      the wavefront / parity / edge subset of the GPU suite (PTMI_LIB: another build)
#   parity_variants  the GPU parity tests against each variants/*.so
#   cache_mk / cache_wf   L1/L2 hit-rate PMC pass of one 32-spp call (tools/pmc_cache_summary.py reads it)
#   lat_mk / lat_wf       VALU / wait PMC passes (tools/gpu_pmc_latency.sh; tools/pmc_valu.py reads them)
#   latc4_mk / latc4_wf / latc5_mk   the same on the C4 mesh-fog scene / the C5 4K scene
#   ta_mk / ta_wf         texture-address (vector memory address) unit busy cycles of one 32-spp call
#   abtrace_<lib>_<mk|wf> rocprofv3 kernel trace + stats of tools/ab.py (64 spp x 2) with variants/libptmi_<lib>.so
#                         (<lib> = default: the default build)
#   abpmc_<lib>_<mk|wf>   FETCH_SIZE, WRITE_SIZE and cache-hit PMC passes of tools/ab.py (32 spp x 1), same libs
#   ablat_<lib>_<mk|wf>   the VALU / wait PMC passes (tools/gpu_pmc_latency.sh) with variants/libptmi_<lib>.so
#   drainbug              tools/gpu_drain_bug.sh: wavefront parity windows at two tail thresholds per build
#                         (DRAIN_LIBS, default "dr5 tr5 tr3": the 5-wave wf_drain and the trace builds)
#   probe                 the diagnostic probe builds (tools/gpu_probe.sh; variants libptmi_probe{1,2}.so)
#   abbench_<c>           bench.py --preset <c> (no CPU baseline) for the default build and every variants/*.so
#                         (MK_VARIANTS: only those), two interleaved rounds -> OUT/abbench_<c>.txt
#   callsize              tools/call_size.py (whole frame at 64 / 8 spp per call, an 8-rank tile shard at 64)
#                         for the default build and every variants/*.so (MK_VARIANTS: only those), two rounds
# Every step has its own time limit; the script stops at the first failure.
set -u
shopt -s nullglob  # no variants built: the variant loops run over none
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
STEPS=${*:-tests smoke c2 c3}
step() {
  local n=$1 t=$2; shift 2
  echo "=== $n $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$n.log" 2>&1
  local rc=$?
  tail -n 1 "$OUT/$n.log" | cut -c 1-400
  echo "=== $n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
for s in $STEPS; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    c2|c3|c4|c5) step bench_$s 300 python bench.py --preset $s ;;
    trace_*) c=${s#trace_}; step $s 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof" -o $c -- python bench.py --preset $c --no-cpu-baseline ;;
    fetch_*) c=${s#fetch_}; step $s 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o fetch_$c -- python bench.py --preset $c --steps 4 --no-cpu-baseline ;;
    write_*) c=${s#write_}; step $s 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc" -o write_$c -- python bench.py --preset $c --steps 4 --no-cpu-baseline ;;
    dist2) step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 8 ;;
    ab_wf_c3) step $s 900 env AB_MODES=wf AB_VARIANTS="${WF_VARIANTS:-}" bash tools/gpu_ab.sh ;;
    ab_wf_fog) step $s 900 env AB_MODES=wf AB_VARIANTS="${WF_VARIANTS:-}" AB_SCENE=cornell_mesh_fog AB_WIDTH=1024 AB_SPP=32 bash tools/gpu_ab.sh ;;
    ab_mk_c2) step $s 900 env AB_MODES=mk AB_VARIANTS="${MK_VARIANTS:-}" bash tools/gpu_ab.sh ;;
    ab_mk_c4) step $s 900 env AB_MODES=mk AB_VARIANTS="${MK_VARIANTS:-}" AB_SCENE=cornell_mesh_fog AB_WIDTH=1024 AB_SPP=32 bash tools/gpu_ab.sh ;;
    ab_mk_c5) step $s 900 env AB_MODES=mk AB_VARIANTS="${MK_VARIANTS:-}" AB_SCENE=vol2_final_scene_comparison AB_WIDTH=3840 AB_SPP=16 bash tools/gpu_ab.sh ;;
    ab_wf_both) rm -f gpurun_out/ab_runs.log; step ab_wf_c3 900 env AB_MODES=wf AB_REPS=3 AB_VARIANTS="${WF_VARIANTS:-}" bash tools/gpu_ab.sh &&
      { rm -f gpurun_out/ab_runs.log; step ab_wf_fog 900 env AB_MODES=wf AB_REPS=3 AB_VARIANTS="${WF_VARIANTS:-}" AB_SCENE=cornell_mesh_fog AB_WIDTH=1024 AB_SPP=32 bash tools/gpu_ab.sh; } ;;
    wftests) step wftests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wf or wavefront or drain or bench_shapes or parity or edge" ;;
    parity_variants) for lib in path-tracer-python_amd/ptmi/_lib/variants/*.so; do
        step parity_$(basename $lib .so) 600 env PTMI_LIB=$PWD/$lib python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread; done ;;
    cache_mk|cache_wf) v=${s#cache_}; step $s 300 timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_cache" -o $v -- python tools/ab.py $v 32 1 ;;
    ta_mk|ta_wf) v=${s#ta_}; step $s 300 timeout -s KILL 240 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_ta" -o $v -- python tools/ab.py $v 32 1 ;;
    lat_mk|lat_wf) v=${s#lat_}; step $s 600 env PMC_VARIANT=$v PMC_DIR=$OUT/pmc_latency_$v bash tools/gpu_pmc_latency.sh ;;
    latc4_mk|latc4_wf) v=${s#latc4_}; step $s 600 env PMC_VARIANT=$v PMC_DIR=$OUT/pmc_latency_c4_$v PMC_SCENE_ARGS="cornell_mesh_fog 1024" bash tools/gpu_pmc_latency.sh ;;
    latc5_mk) step $s 600 env PMC_VARIANT=mk PMC_DIR=$OUT/pmc_latency_c5_mk PMC_SCENE_ARGS="vol2_final_scene_comparison 3840" bash tools/gpu_pmc_latency.sh ;;
    probe) step probe 600 bash tools/gpu_probe.sh ;;
    drainbug) step drainbug 1200 env LIBS="${DRAIN_LIBS:-dr5 tr5 tr3}" STEP_S=300 bash tools/gpu_drain_bug.sh ;;
    abbench_*) c=${s#abbench_}; libs=(path-tracer-python_amd/ptmi/_lib/libptmi.so)
      if [ -n "${MK_VARIANTS:-}" ]; then for n in $MK_VARIANTS; do libs+=(path-tracer-python_amd/ptmi/_lib/variants/libptmi_$n.so); done
      else libs+=(path-tracer-python_amd/ptmi/_lib/variants/*.so); fi
      for r in 1 2; do for lib in "${libs[@]}"; do n=$(basename $lib .so)
        PTMI_LIB=$PWD/$lib step abbench_${c}_${n}_$r 300 python bench.py --preset $c --no-cpu-baseline
        echo "$n $(grep -o '"value": [0-9.]*' "$OUT/abbench_${c}_${n}_$r.log" | head -1)" >> "$OUT/abbench_$c.txt"; done; done ;;
    callsize) libs=(path-tracer-python_amd/ptmi/_lib/libptmi.so)
      if [ -n "${MK_VARIANTS:-}" ]; then for n in $MK_VARIANTS; do libs+=(path-tracer-python_amd/ptmi/_lib/variants/libptmi_$n.so); done
      else libs+=(path-tracer-python_amd/ptmi/_lib/variants/*.so); fi
      for r in 1 2; do for lib in "${libs[@]}"; do
        PTMI_LIB=$PWD/$lib CALL_SIZE_SPP=64,8 CALL_SIZE_SHARDS=8:4 step callsize_$(basename $lib .so)_$r 300 python tools/call_size.py
        cat "$OUT/callsize_$(basename $lib .so)_$r.log" | grep full_ | sed "s/^/$(basename $lib .so) /" >> "$OUT/callsize.txt"; done; done ;;
    abtrace_*) r=${s#abtrace_}; name=${r%_*}; mode=${r##*_}
      lib=path-tracer-python_amd/ptmi/_lib/libptmi.so; [ "$name" = default ] || lib=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$name.so
      PTMI_LIB=$PWD/$lib step $s 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/abtrace" -o ${name}_$mode -- python tools/ab.py $mode 64 2 ${AB_SCENE:-vol2_final_scene} ${AB_WIDTH:-800} ;;
    abpmc_*) r=${s#abpmc_}; name=${r%_*}; mode=${r##*_}
      lib=path-tracer-python_amd/ptmi/_lib/libptmi.so; [ "$name" = default ] || lib=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$name.so
      PTMI_LIB=$PWD/$lib step ${s}_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/abpmc" -o ${name}_${mode}_fetch -- python tools/ab.py $mode 32 1 &&
      PTMI_LIB=$PWD/$lib step ${s}_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/abpmc" -o ${name}_${mode}_write -- python tools/ab.py $mode 32 1 &&
      PTMI_LIB=$PWD/$lib step ${s}_cache 300 timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/abpmc" -o ${name}_${mode}_cache -- python tools/ab.py $mode 32 1 ;;
    ablat_*) r=${s#ablat_}; name=${r%_*}; mode=${r##*_}
      lib=path-tracer-python_amd/ptmi/_lib/libptmi.so; [ "$name" = default ] || lib=path-tracer-python_amd/ptmi/_lib/variants/libptmi_$name.so
      PTMI_LIB=$PWD/$lib step $s 600 env PMC_VARIANT=$mode PMC_DIR=$OUT/ablat_$name bash tools/gpu_pmc_latency.sh ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
