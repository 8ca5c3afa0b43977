#!/bin/bash
# scratch GPU command (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_configs.py tests/test_gpu_engine.py tests/test_gpu_stream.py -m gpu > $OUT/plan_$TAG.log 2>&1 || { tail -40 $OUT/plan_$TAG.log; exit 1; }
tail -2 $OUT/plan_$TAG.log
for i in 1 2; do CFG=C1 timeout -k 10 120 python -u tools/small_query_ab.py > $OUT/c1_${TAG}_$i.log 2>&1 || { tail -20 $OUT/c1_${TAG}_$i.log; exit 1; }
grep '^{' $OUT/c1_${TAG}_$i.log | cut -c1-260; done
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-dominance --no-csv --no-sort --no-e2e --no-operator > $OUT/bcfg_$TAG.json 2> $OUT/bcfg_$TAG.err || { tail -30 $OUT/bcfg_$TAG.err; exit 1; }
python3 tools/bsum.py $OUT/bcfg_$TAG.json
