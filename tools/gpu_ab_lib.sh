#!/bin/bash
# In-box A/B of two builds of the library (SKYLINE_HIP_LIB), C4 bench line only,
# alternating, each run under its own time limit; optional gpu tests first.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
OLD=$R/flink-skyline-qos_amd/build/libskyline_hip_ab_old.so
NEW=$R/flink-skyline-qos_amd/build/libskyline_hip.so
# LIBS: build names under flink-skyline-qos_amd/build/ to alternate (default: new, old twice)
if [ -n "$LIBS" ]; then L2=""; for x in $LIBS; do L2="$L2 $R/flink-skyline-qos_amd/build/$x"; done; ORDER="$L2 $L2";
else ORDER="$NEW $OLD $NEW $OLD"; fi
A="--steps 20 --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator ${BENCH_ARGS}"
i=0
for L in $ORDER; do
  i=$((i+1))
  SKYLINE_HIP_LIB=$L timeout -k 10 200 python -u bench.py $A > $OUT/ab_lib_$i.json 2> $OUT/ab_lib_$i.err || { tail -20 $OUT/ab_lib_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab_lib_$i.json').read().strip().splitlines()[-1]);print('$(basename $L)', round(d['ms_per_step'],4), 'k_filter', round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3))"
done
