#!/bin/bash
# round-5 A/B: the pair pass's register budget (waves per SIMD 6 = build_measure, 5, 7)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05w}
for n in 10000000 2000000; do
  for v in measure ab5 ab7 measure ab5 ab7; do
    L=flink-skyline-qos_amd/build_$v/libskyline_hip.so
    timeout -k 10 200 env SKYLINE_HIP_LIB=$L python -u tools/dom_bench.py $n 3 >> ${O}_${v}_$n.json 2>&1 || exit 1
  done
done
