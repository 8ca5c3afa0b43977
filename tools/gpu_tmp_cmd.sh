#!/bin/bash
# round-6 scratch GPU call (edited per call; each GPU step under its own limit, chained with &&)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out
ML=flink-skyline-qos_amd/build_measure/libskyline_hip.so
timeout -k 10 1080 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu_f.log 2>&1 || { tail -40 $O/pytest_gpu_f.log; exit 1; }
tail -3 $O/pytest_gpu_f.log
