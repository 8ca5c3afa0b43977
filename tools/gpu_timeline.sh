#!/bin/bash
# One-step dispatch timeline of a bench config under rocprofv3 --kernel-trace (GPU box).
# usage: tools/gpu_timeline.sh <tag> [bench args...]
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
TAG=$1; shift
export TMPDIR=/tmp
rm -rf $OUT/tl_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/tl_$TAG -o run -- python3 -u $R/bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-e2e --no-csv --no-sort --no-configs --no-dominance --no-stream --no-operator "$@" > $OUT/tl_$TAG.log 2>&1
python3 $R/tools/prof_summary.py timeline $OUT/tl_$TAG ${TL_N:-90} > $OUT/tl_${TAG}.txt
rm -rf $OUT/tl_$TAG
