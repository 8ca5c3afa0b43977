#!/bin/bash
# The final small-query record (profiles/r06_small_query_final.log): tools/small_query_ab.py per config
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
for C in C1 C2 C5T C3 C4R; do CFG=$C timeout -k 10 120 python -u tools/small_query_ab.py 2>/dev/null | grep '^{' >> $OUT/r06_small_query_final.log || exit 1; done
cut -c1-330 $OUT/r06_small_query_final.log
