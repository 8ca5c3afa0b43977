#!/bin/bash
# round-6 scratch GPU call (edited per call; each GPU step under its own limit, chained with &&)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_plan.py \
    tests/test_gpu_configs.py tests/test_gpu_mbr.py > $O/tests_k.log 2>&1 || { tail -40 $O/tests_k.log; exit 1; }
tail -2 $O/tests_k.log
timeout -k 10 200 python -u tools/dense_bench.py 16384 65536 > $O/dense_k.log 2>&1 || { tail -20 $O/dense_k.log; exit 1; }
grep '^{' $O/dense_k.log | cut -c1-400
timeout -k 10 300 python -u tools/c5_ab.py > $O/c5ab_k.log 2>&1 || { tail -20 $O/c5ab_k.log; exit 1; }
grep '^{' $O/c5ab_k.log
ML=flink-skyline-qos_amd/build_measure/libskyline_hip.so
: > $O/atom_k.log
for c in C1 C2 C4R C3; do
  for m in 0 4 1; do
    CFG=$c SKYLINE_HIP_LIB=$ML SKY_FILTER_DBG=$m timeout -k 10 120 python -u tools/small_query_ab.py >> $O/atom_k.log 2>&1 || { tail -20 $O/atom_k.log; exit 1; }
  done
done
grep '^{' $O/atom_k.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = d['kernel_mean_ms_profiled']
    print(d['config'], 'dbg', d['filter_dbg'], 'filter_ms', round(k.get('filter', 0), 4))
"
