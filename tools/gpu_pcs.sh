set -u
mkdir -p gpurun_out
PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/variants/libptmi_probe.so timeout -k 10 120 python tools/probe.py vol2_final_scene 800 8 > gpurun_out/probe_c2.txt 2>&1 || exit 1
PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/variants/libptmi_probe.so timeout -k 10 120 python tools/probe.py cornell_mesh_fog 1024 4 > gpurun_out/probe_c4.txt 2>&1 || exit 1
rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d gpurun_out/pcs -o mk -- python tools/ab.py mk 64 1 > gpurun_out/pcs.log 2>&1
echo "pcs rc=$?"
