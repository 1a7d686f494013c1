#!/bin/bash
# PMC pass (one counter set) of tools/ab.py for the default lib and every
# variant: pmc_ab.sh MODE SPP "COUNTERS..." -> gpurun_out/pmcab/<lib>_*.csv
set -u
shopt -s nullglob
mkdir -p gpurun_out/pmcab
libs=(path-tracer-python_amd/ptmi/_lib/libptmi.so path-tracer-python_amd/ptmi/_lib/variants/*.so)
for lib in "${libs[@]}"; do
  name=$(basename $lib .so)
  PTMI_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --pmc $3 --output-format csv -d gpurun_out/pmcab -o $name -- python tools/ab.py $1 $2 1 ${AB_SCENE:-vol2_final_scene} ${AB_WIDTH:-800} > gpurun_out/pmcab/$name.log 2>&1 || { echo "$name rc=$?"; exit 1; }
done
