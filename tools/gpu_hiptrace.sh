#!/bin/bash
# One C4 step's kernels with the host time of their launch calls (rocprofv3 --kernel-trace
# --hip-trace, no counters): where a gap between kernels comes from the host.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
TAG=${1:-ht}
export TMPDIR=/tmp
rm -rf $OUT/ht_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -f csv -d $OUT/ht_$TAG -o run -- python3 -u $R/bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-e2e --no-csv --no-sort --no-configs --no-dominance --no-stream --no-operator > $OUT/ht_$TAG.log 2>&1
python3 $R/tools/hiptrace_join.py $OUT/ht_$TAG > $OUT/ht_${TAG}.txt
rm -rf $OUT/ht_$TAG
