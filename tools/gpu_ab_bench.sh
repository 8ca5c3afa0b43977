#!/bin/bash
# In-box A/B of one environment variable on the C4 bench line only: VAR=name VALUES="a b a b"
# (each run under its own time limit; prints ms/step, k_filter ms and frac, phases)
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export PYTHONUNBUFFERED=1
A="--steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator ${BENCH_ARGS}"
i=0
for v in $VALUES; do
  i=$((i+1))
  env $VAR=$v timeout -k 10 200 python -u bench.py $A > $OUT/abb_$i.json 2> $OUT/abb_$i.err || { tail -20 $OUT/abb_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/abb_$i.json').read().strip().splitlines()[-1]);print('$VAR=$v', round(d['ms_per_step'],4), 'p50', round(d['p50_query_latency_ms'],4), 'k_filter', round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3), {k:round(x,3) for k,x in d['phases_ms_last_step'].items()})"
done
