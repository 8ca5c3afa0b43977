export SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_DEBUG=2
for a in "mr-grid 0 2 200000 16" "mr-angle 0 3 20000 8" "mr-angle 2 3 6000 8" "mr-grid 1 3 100000 8" "mr-angle 1 5 20000 8"; do
  echo "== $a"; timeout -k 10 60 python tools/tiny_debug.py $a 2>&1 | grep -v "phase\|amdgpu.ids\|sfs" || exit 1
done > gpurun_out/tdbg6.txt 2>&1
unset SKYLINE_HIP_LIB SKY_DEBUG
bash tools/gpu_r05_tiny.sh r05t
