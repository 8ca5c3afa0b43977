#!/bin/bash
# rocprofv3 --kernel-trace --stats of each BASELINE configuration's bench line alone
# (bench.py --config Cn), summaries under gpurun_out/trace_cfg_<Cn>_summary.txt.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
for C in ${CONFIGS:-C1 C2 C3 C5}; do
  rm -rf $OUT/trace_cfg_$C
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_cfg_$C -o run -- python3 -u $R/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline > $OUT/trace_cfg_$C.log 2>&1
  grep '^{' $OUT/trace_cfg_$C.log > $OUT/bench_cfg_$C.json || true
  python3 $R/tools/prof_summary.py trace $OUT/trace_cfg_$C > $OUT/trace_cfg_${C}_summary.txt
  echo "== $C"; head -6 $OUT/trace_cfg_${C}_summary.txt
done
