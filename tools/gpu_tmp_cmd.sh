#!/bin/bash
# scratch GPU command for the current A/B (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_configs.py -m gpu > $OUT/plan_$TAG.log 2>&1 || { tail -40 $OUT/plan_$TAG.log; exit 1; }
tail -3 $OUT/plan_$TAG.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dominance --no-csv --no-stream --no-configs --no-e2e --no-operator > $OUT/bsort_$TAG.json 2> $OUT/bsort_$TAG.err || { tail -30 $OUT/bsort_$TAG.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open('$OUT/bsort_$TAG.json').readline()); print(d['ms_per_step'], json.dumps(d.get('sort_roofline'))[:400])"
