#!/bin/bash
# round-5 dominance A/B: the product library against build_ab2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05d}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mbr.py tests/test_gpu_dist_step.py > ${O}_mbr.log 2>&1 || exit 1
for n in 2000000 10000000; do
  for v in prod ab2 prod ab2; do
    L=flink-skyline-qos_amd/build/libskyline_hip.so; [ $v != prod ] && L=flink-skyline-qos_amd/build_$v/libskyline_hip.so
    timeout -k 10 200 env SKYLINE_HIP_LIB=$L python -u tools/dom_bench.py $n 3 >> ${O}_${v}_$n.json 2>&1 || exit 1
  done
done
