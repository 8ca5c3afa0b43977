#!/bin/bash
# Round-6 GPU-box steps (parametrised; every GPU step under its own time limit, chained so the
# first failure ends the call).  Usage: tools/gpu_r06.sh STEP[,STEP...] [TAG]
#   disttests   the multi-GPU decomposition and step tests
#   distphases  tools/dist_phases.py -> gpurun_out/r06_dist_phases_$TAG.json
#   gputests    the whole -m gpu suite
#   bench       bench.py (default line) -> gpurun_out/bench_$TAG.json
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export PYTHONUNBUFFERED=1
STEPS=$1; TAG=${2:-r06}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in ${STEPS//,/ }; do
  case $s in
    disttests)
      timeout -k 10 900 $PYT tests/test_gpu_dist_step.py tests/test_gpu_dist.py \
        "tests/test_gpu_configs.py::test_c4_8way_decomposition" \
        "tests/test_gpu_configs.py::test_c3_angle_4d_anti_50m_one_gpu_and_sharded" > $OUT/disttests_$TAG.log 2>&1 \
        || { tail -40 $OUT/disttests_$TAG.log; exit 1; }
      tail -3 $OUT/disttests_$TAG.log ;;
    distphases)
      timeout -k 10 900 python -u tools/dist_phases.py ${DIST_ONLY:+--only $DIST_ONLY} \
        --out $OUT/r06_dist_phases_$TAG.json > $OUT/distphases_$TAG.log 2>&1 || { tail -30 $OUT/distphases_$TAG.log; exit 1; }
      grep '^{' $OUT/distphases_$TAG.log | cut -c1-600 ;;
    gputests)
      timeout -k 10 1000 $PYT tests -m gpu > $OUT/pytest_gpu_$TAG.log 2>&1 || { tail -40 $OUT/pytest_gpu_$TAG.log; exit 1; }
      tail -3 $OUT/pytest_gpu_$TAG.log ;;
    bench)
      timeout -k 10 500 python -u bench.py ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -30 $OUT/bench_$TAG.err; exit 1; }
      cut -c1-1500 $OUT/bench_$TAG.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
