#!/bin/bash
# round 5 PMC: k_filter HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes, warm dispatches
# averaged by tools/prof_summary.py), k_filter's store counts from the measurement build, and the
# k_mbr_pairs instruction mix / wait counters at std-anti 8D 2M
set -e
export TMPDIR=/tmp
TAG=${1:-r05}
bash tools/gpu_pmc.sh $TAG
M=flink-skyline-qos_amd/build_measure/libskyline_hip.so
timeout -k 10 200 env SKYLINE_HIP_LIB=$M SKY_FILTER_COUNT=1 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator > gpurun_out/${TAG}_filter_count.json \
    2> gpurun_out/${TAG}_filter_count.err
TAG=$TAG SKIP_PMC= NS="" bash tools/gpu_mbr_pmc.sh
