#!/bin/bash
# One rocprofv3 --pmc pass per argument (each argument = a space-separated counter
# list that fits one pass), kernel-trace only, each under its own time limit.
#   KRE=<kernel regex> BENCH_ARGS="..." bash tools/gpu_pmc_counters.sh TAG "C1 C2" "C3 C4" ...
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; shift
KRE=${KRE:-k_filter<}
i=0
for CS in "$@"; do
  i=$((i+1))
  rm -rf $OUT/pmc_${TAG}_$i
  timeout -k 10 300 rocprofv3 --pmc $CS --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_${TAG}_$i -o run -- \
      python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/pmc_${TAG}_$i.log 2>&1 \
      || { tail -20 $OUT/pmc_${TAG}_$i.log; exit 1; }
  python tools/prof_summary.py pmcshow $OUT/pmc_${TAG}_$i "$KRE"
done
