#!/bin/bash
# scratch GPU command for the current A/B (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
export TMPDIR=/tmp
for C in C2 C1; do
rm -rf $OUT/sq_${C}_$TAG
CFG=$C timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/sq_${C}_$TAG -o run -- python3 -u tools/small_query_ab.py > $OUT/sq_${C}_$TAG.log 2>&1 || { tail -30 $OUT/sq_${C}_$TAG.log; exit 1; }
python3 tools/prof_summary.py trace $OUT/sq_${C}_$TAG > $OUT/sq_${C}_${TAG}_summary.txt
rm -rf $OUT/sq_${C}_$TAG
echo "== $C"; head -24 $OUT/sq_${C}_${TAG}_summary.txt
done
