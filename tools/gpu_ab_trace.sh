#!/bin/bash
# Kernel trace of an interleaved A/B run (tools/filter_ab2.py), summarised per kernel
# name (template arguments included, so variants that differ in them separate).
set -e
export TMPDIR=/tmp
OUT=gpurun_out; rm -rf $OUT/abt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/abt -o run -- python3 -u tools/filter_ab2.py > $OUT/abt.log 2>&1
python3 tools/prof_summary.py trace $OUT/abt > $OUT/abt_summary.txt
cat $OUT/abt.log | tail -30
head -40 $OUT/abt_summary.txt
