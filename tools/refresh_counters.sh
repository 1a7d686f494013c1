#!/bin/bash
# Fold one counter re-collection (not product) into profiles/: the output of
#   bash tools/gpu_check.sh OUT trace_c2 trace_c3 fetch_c2 write_c2 fetch_c3 write_c3 \
#     fetch_c4 write_c4 fetch_c5 write_c5 lat_mk lat_wf latc4_mk latc5_mk ta_mk ta_wf cache_mk cache_wf
# merged back under gpurun_out/OUT is compressed into profiles/$ROUND/{pmc_final,rocprof}/ (ROUND: r06)
# and profiles/traffic.json, profiles/valu.json, the TA / cache summaries and the
# trace busy figures are regenerated, every row naming HASH (the last commit that
# touched the kernel sources). Usage: bash tools/refresh_counters.sh OUT
set -eu
cd "$(dirname "$0")/.."
SRC=gpurun_out/$1
HASH=$(git log -1 --format=%h -- path-tracer-python_amd/csrc include)
ROUND=${ROUND:-r06}
P=profiles/$ROUND/pmc_final
R=profiles/$ROUND/rocprof
mkdir -p "$P" "$R"
for c in c2 c3 c4 c5; do
  for k in fetch write; do gzip -9nc "$SRC/pmc/${k}_${c}_counter_collection.csv" > "$P/${k}_${c}_counter_collection.csv.gz"; done
done
for d in pmc_latency_mk pmc_latency_wf pmc_latency_c4_mk pmc_latency_c5_mk pmc_ta pmc_cache; do
  mkdir -p "$P/$d"
  for f in "$SRC/$d"/*_counter_collection.csv; do gzip -9nc "$f" > "$P/$d/$(basename "$f").gz"; done
done
for c in c2 c3; do
  gzip -9nc "$SRC/rocprof/${c}_kernel_trace.csv" > "$R/${c}_kernel_trace.csv.gz"
  cp "$SRC/rocprof/${c}_kernel_stats.csv" "$R/"
  cp "$SRC/trace_$c.log" "$R/bench_${c}_under_trace.log"
done
python3 tools/trace_busy.py "$SRC/rocprof/c2_kernel_trace.csv" mk_render_kernel 2 > "$R/c2_busy.json"
python3 tools/trace_busy.py "$SRC/rocprof/c3_kernel_trace.csv" wf_intersect > "$R/c3_intersect_busy.json"

TMP=$(mktemp -d)
z() { gunzip -c "$1" > "$TMP/$(basename "$1" .gz)"; echo "$TMP/$(basename "$1" .gz)"; }
traffic() {  # key kernel preset
  python3 tools/pmc_traffic.py "$1" "$2" "$(z $P/fetch_$3_counter_collection.csv.gz)" "$(z $P/write_$3_counter_collection.csv.gz)" \
    "$P/{fetch,write}_$3_counter_collection.csv.gz ($ROUND HEAD $HASH; bench.py --preset $3 --steps 4 --no-cpu-baseline under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"
}
traffic vol2_final_scene:800:mk:64:50:megakernel mk_render_kernel c2
traffic vol2_final_scene:800:wf:64:50:wf_intersect wf_intersect c3
traffic vol2_final_scene:800:wf:64:50:wf_scatter wf_scatter c3
traffic vol2_final_scene:800:wf:64:50:wf_drain wf_drain c3
traffic cornell_mesh_fog:1024:mk:32:50:megakernel mk_render_kernel c4
traffic vol2_final_scene_comparison:3840:mk:16:50:megakernel mk_render_kernel c5

valu() {  # key dir prefix kernel scene
  local d=$TMP/$2; mkdir -p "$d"
  for f in $P/$2/*_counter_collection.csv.gz; do gunzip -c "$f" > "$d/$(basename "$f" .gz)"; done
  PMC_SOURCE="$P/$2/$3_{a,b,c}_counter_collection.csv.gz ($ROUND HEAD $HASH; tools/gpu_pmc_latency.sh: tools/ab.py $3 32 1, one 32-spp call on $5; kernel $4); tools/pmc_valu.py" \
    python3 tools/pmc_valu.py "$1" "$d" "$3" "$4"
}
valu vol2_final_scene:800:mk:megakernel pmc_latency_mk mk mk_render_kernel "vol2_final_scene 800"
valu vol2_final_scene:800:wf:wf_intersect pmc_latency_wf wf wf_intersect "vol2_final_scene 800"
valu vol2_final_scene:800:wf:wf_scatter pmc_latency_wf wf wf_scatter "vol2_final_scene 800"
valu cornell_mesh_fog:1024:mk:megakernel pmc_latency_c4_mk mk mk_render_kernel "cornell_mesh_fog 1024"
valu vol2_final_scene_comparison:3840:mk:megakernel pmc_latency_c5_mk mk mk_render_kernel "vol2_final_scene_comparison 3840"

python3 tools/pmc_cache_summary.py "$SRC/pmc_cache/mk_counter_collection.csv" "$SRC/pmc_cache/wf_counter_collection.csv" > "$P/cache_summary.json"
python3 - "$SRC" "$P" <<'EOF'
import collections, csv, json, sys
src, p = sys.argv[1:3]
out = {}
for v, kernels in (('mk', ['mk_render_kernel']), ('wf', ['wf_intersect', 'wf_scatter'])):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f'{src}/pmc_ta/{v}_counter_collection.csv')):
        for k in kernels:
            if k in r['Kernel_Name']:
                per[(k, r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
    for k in kernels:
        runs = [c for (q, _), c in per.items() if q == k]
        if k == 'mk_render_kernel':  # the measured call (the largest dispatch), not the warm-up
            runs = [max(runs, key=lambda c: c['GRBM_GUI_ACTIVE'])]
        out[k] = round(sum(c['TA_BUSY_avr'] for c in runs) / (sum(c['GRBM_GUI_ACTIVE'] for c in runs) / 8), 4)
json.dump({'ta_busy_frac': out, 'source': f'{p}/pmc_ta/{{mk,wf}}_counter_collection.csv.gz (TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8), one 32-spp call of tools/ab.py)'},
          open(f'{p}/ta_summary.json', 'w'), indent=1)
EOF
rm -rf "$TMP"
echo "counters folded in at $HASH"
