#!/bin/bash
# round 5 late: k_filter tiles per workgroup with the cap at spans / 256 (build_ab9) against the current cap
set -o pipefail
O=gpurun_out/r05t3
run() {  # lib tpb config
  SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_$1/libskyline_hip.so SKY_FILTER_TPB=$2 timeout -k 10 200 python -u bench.py --config $3 --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 tpb $2 $3', d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> ${O}.txt
}
for rep in 1 2; do
  run measure 4 C2 || exit 1; run ab9 4 C2 || exit 1; run ab9 8 C2 || exit 1; run ab9 16 C2 || exit 1
  run measure 4 C4 || exit 1; run ab9 8 C4 || exit 1; run ab9 16 C4 || exit 1
done
