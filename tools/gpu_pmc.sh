#!/bin/bash
# HBM traffic of k_filter from PMC counters: separate rocprofv3 passes (FETCH_SIZE
# and WRITE_SIZE cannot share one pass on gfx950), kernel-trace only, each under its
# own time limit.  Writes profiles/traffic_filter.json via tools/prof_summary.py.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r01}
KRE=${KRE:-k_filter<}
N=${N:-100000000}
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmc_${TAG}_$C
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_${TAG}_$C -o run -- \
      python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator --tuples $N ${BENCH_ARGS} > $OUT/pmc_${TAG}_$C.log 2>&1 \
      || { tail -20 $OUT/pmc_${TAG}_$C.log; exit 1; }
done
python tools/prof_summary.py pmc $OUT/pmc_${TAG}_FETCH_SIZE "k_filter<" --n $N --dims 8 --dist anti_correlated
python tools/prof_summary.py pmc $OUT/pmc_${TAG}_WRITE_SIZE "k_filter<" --n $N --dims 8 --dist anti_correlated
cp profiles/traffic_filter.json $OUT/traffic_filter_$TAG.json
