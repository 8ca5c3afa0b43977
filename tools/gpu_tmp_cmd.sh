#!/bin/bash
# scratch GPU command for the current A/B (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_plan.py tests/test_gpu_configs.py -m gpu > $OUT/st_$TAG.log 2>&1 || { tail -40 $OUT/st_$TAG.log; exit 1; }
tail -2 $OUT/st_$TAG.log
timeout -k 10 300 python -u tools/c5_ab.py > $OUT/c5ab_$TAG.log 2>&1 || { tail -20 $OUT/c5ab_$TAG.log; exit 1; }
grep '^{' $OUT/c5ab_$TAG.log
for i in 1 2; do CFG=C3 timeout -k 10 120 python -u tools/small_query_ab.py > $OUT/c3_${TAG}_$i.log 2>&1 || exit 1; grep '^{' $OUT/c3_${TAG}_$i.log | cut -c1-250; done
