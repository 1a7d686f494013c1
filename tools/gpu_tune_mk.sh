set -u
for sc in "vol2_final_scene 800" "cornell_mesh_fog 1024"; do
for l in libptmi.so variants/libptmi_td2.so variants/libptmi_td8.so variants/libptmi_cs16.so variants/libptmi_cs64.so; do
  echo "== $l $sc"; PROBE_N=${PN:-64} PTMI_LIB=$PWD/path-tracer-python_amd/ptmi/_lib/$l timeout -k 10 300 python tools/overlap_probe.py $sc 256 || exit 1
done; done
