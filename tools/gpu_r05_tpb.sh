#!/bin/bash
# round 5 late: k_filter tiles per workgroup on C2 / C3 (measurement build's SKY_FILTER_TPB; launch shape only)
set -o pipefail
O=gpurun_out/r05t2
export SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so
for c in C2 C3; do
  for t in 4 1 2 4 1 2; do
    echo "== $c tpb $t" >> ${O}.txt
    SKY_FILTER_TPB=$t timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> ${O}.txt || exit 1
  done
done
