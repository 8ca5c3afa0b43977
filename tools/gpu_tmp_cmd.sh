#!/bin/bash
# round-6 scratch GPU call (edited per call; each GPU step under its own limit, chained with &&)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_dense.py tests/test_gpu_mbr.py tests/test_gpu_dist_step.py tests/test_gpu_dist.py \
   "tests/test_gpu_configs.py::test_c4_8way_decomposition" "tests/test_gpu_configs.py::test_c4_angle_8d_anti_100m" \
   tests/test_gpu_plan.py > gpurun_out/tests_d.log 2>&1 || { tail -40 gpurun_out/tests_d.log; exit 1; }
tail -3 gpurun_out/tests_d.log
timeout -k 10 900 python -u tools/dist_phases.py --out gpurun_out/r06_dist_phases_d.json > gpurun_out/distphases_d.log 2>&1 || { tail -30 gpurun_out/distphases_d.log; exit 1; }
grep '^{' gpurun_out/distphases_d.log | cut -c1-700
timeout -k 10 400 python -u tools/dom_bench.py 100000000 1 > gpurun_out/dom100M_d.log 2>&1 || { tail -30 gpurun_out/dom100M_d.log; exit 1; }
tail -3 gpurun_out/dom100M_d.log
TL_N=60 timeout -k 10 400 bash tools/gpu_timeline.sh c1_d --config C1 || { tail -20 gpurun_out/tl_c1_d.log; exit 1; }
head -70 gpurun_out/tl_c1_d.txt
