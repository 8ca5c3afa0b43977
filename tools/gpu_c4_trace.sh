#!/bin/bash
# C4 alone under rocprofv3 --kernel-trace --stats (the bench line's k_filter and the step's
# other kernels); $1 = tag, extra env (A/B knobs) passes through.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-c4}
rm -rf $OUT/trace_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$TAG -o run -- python3 -u $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator > $OUT/trace_$TAG.log 2>&1
grep '^{' $OUT/trace_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'phases', d['phases_ms_last_step'])"
python3 $R/tools/prof_summary.py trace $OUT/trace_$TAG > $OUT/trace_${TAG}_summary.txt
head -22 $OUT/trace_${TAG}_summary.txt
