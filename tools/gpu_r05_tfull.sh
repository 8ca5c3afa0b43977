#!/bin/bash
# round 5: the tail's phase clocks (measurement build), the C1 / C2 lines, the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}
SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_TINY_CLK=1 timeout -k 10 120 python tools/tiny_debug.py mr-dim 0 2 1000000 8 > ${O}_clk.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan.py > ${O}_plan.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1.json 2> ${O}_c1.err || exit 1
timeout -k 10 300 python -u bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c2.json 2> ${O}_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c1prof -o t -- python3 bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c2prof -o t -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c2prof.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_pytest.txt 2>&1 || exit 1
