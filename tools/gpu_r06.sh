#!/bin/bash
# Round-6 GPU-box steps (parametrised; every GPU step under its own time limit, chained so the
# first failure ends the call).  Usage: tools/gpu_r06.sh STEP[,STEP...] [TAG]
#   disttests   the multi-GPU decomposition and step tests
#   distphases  tools/dist_phases.py -> gpurun_out/r06_dist_phases_$TAG.json
#   gputests    the whole -m gpu suite
#   bench       bench.py (default line) -> gpurun_out/bench_$TAG.json
#   smoke       __graft_entry__.smoke()
#   trace       rocprofv3 --kernel-trace --stats of the C4 headline alone -> trace_$TAG_summary.txt
#   traffic     k_filter HBM bytes from PMC (FETCH_SIZE / WRITE_SIZE passes) -> profiles/traffic_filter.json
#   rehearse    bench.py --gpus 2 over gloo on the one GPU (the multi-GPU control flow)
#   probe       tools/probe/valu_probe (VALU rates on this box)
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
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
      tail -1 $OUT/smoke_$TAG.log ;;
    trace)
      export TMPDIR=/tmp
      rm -rf $OUT/trace_$TAG
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$TAG -o run -- python3 -u $R/bench.py --steps 10 --warmup 2 \
          --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator > $OUT/trace_$TAG.log 2>&1 \
          || { tail -30 $OUT/trace_$TAG.log; exit 1; }
      grep '^{' $OUT/trace_$TAG.log > $OUT/bench_trace_$TAG.json || true
      python tools/prof_summary.py trace $OUT/trace_$TAG > $OUT/trace_${TAG}_summary.txt
      rm -rf $OUT/trace_$TAG
      head -30 $OUT/trace_${TAG}_summary.txt ;;
    traffic)
      timeout -k 10 700 bash tools/gpu_pmc.sh $TAG > $OUT/traffic_$TAG.log 2>&1 || { tail -30 $OUT/traffic_$TAG.log; exit 1; }
      cat $OUT/traffic_filter_$TAG.json | head -20 ;;
    rehearse)
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
         --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $OUT/rehearsal2_$TAG.json 2> $OUT/rehearsal2_$TAG.err \
         || { tail -30 $OUT/rehearsal2_$TAG.err; exit 1; }
      grep '^{' $OUT/rehearsal2_$TAG.json | cut -c1-300 ;;
    probe)
      timeout -k 10 120 tools/probe/valu_probe > $OUT/valu_probe_$TAG.json 2>&1 || { cat $OUT/valu_probe_$TAG.json; exit 1; }
      cat $OUT/valu_probe_$TAG.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
