mkdir -p gpurun_out/wpc
for round in 1 2; do
  for lib in ${WPC_LIBS:-libptmi.so}; do
    PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/$lib CALL_SIZE_SPP=64,8 CALL_SIZE_SHARDS=${WPC_SHARDS:-8:4,4:8} timeout -k 10 200 python tools/call_size.py 2>&1 | grep '^{' | sed "s|^|$lib |" | tee -a gpurun_out/wpc/call_size.log || exit 1
  done
done
