#!/bin/bash
# stream + operator GPU tests, then the C5 trigger latency A/B (tools/c5_ab.py)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_operators.py -m gpu > $OUT/st_m30.log 2>&1 || { tail -40 $OUT/st_m30.log; exit 1; }
tail -2 $OUT/st_m30.log
timeout -k 10 300 python -u tools/c5_ab.py > $OUT/c5ab_m30.log 2>&1 || { tail -20 $OUT/c5ab_m30.log; exit 1; }
grep '^{' $OUT/c5ab_m30.log
