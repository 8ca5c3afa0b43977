#!/bin/bash
# gpu parity tests, then the C4 bench line with batched fills/read-backs and with
# per-range read-backs (SKY_GATHER=0), each under its own time limit.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
A="--steps 20 --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort"
for v in ${GVALS:-1 0 1 0}; do
  SKY_GATHER=$v timeout -k 10 200 python -u bench.py $A > $OUT/ab_gather_$v.json 2> $OUT/ab_gather_$v.err || { tail -20 $OUT/ab_gather_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab_gather_$v.json').read().strip().splitlines()[-1]);print('SKY_GATHER=$v', round(d['ms_per_step'],4), round(d['p50_query_latency_ms'],4), round(d['value']/1e9,2))"
done
