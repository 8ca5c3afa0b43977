#!/bin/bash
# round 5: the one-workgroup tail's phase clocks (measurement build), its tests, the C1 line
set -o pipefail
O=gpurun_out/${1:-r05c}
SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_TINY_CLK=1 timeout -k 10 120 python tools/tiny_debug.py mr-dim 0 2 1000000 8 > ${O}_clk.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plan.py > ${O}_pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1.json 2> ${O}_c1.err || exit 1
