#!/bin/bash
# round 5: pair pass v2 (product) vs v1 (build_ab2); the 10M query with the prefilter off traced
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mbr.py tests/test_gpu_dist_step.py > ${O}_mbr.log 2>&1 || exit 1
for n in 2000000 10000000; do
  for v in prod ab2; do
    L=flink-skyline-qos_amd/build/libskyline_hip.so; [ $v != prod ] && L=flink-skyline-qos_amd/build_$v/libskyline_hip.so
    timeout -k 10 200 env SKYLINE_HIP_LIB=$L python -u tools/dom_bench.py $n 3 > ${O}_${v}_$n.json 2>&1 || exit 1
    timeout -k 10 200 env SKYLINE_HIP_LIB=$L SKY_PREFILTER=0 python -u tools/dom_bench.py $n 3 > ${O}_${v}_nopf_$n.json 2>&1 || exit 1
  done
done
timeout -k 10 200 env SKY_PREFILTER=0 rocprofv3 --kernel-trace --stats -d ${O}_prof -o t -- python3 tools/dom_bench.py 10000000 2 > ${O}_prof.log 2>&1 || exit 1
