#!/bin/bash
# Round-3 GPU pass: STEPS (comma list) of
#   dist   the multi-GPU step tests (emulated ranks, 2-process gloo, C4 8-way)
#   tests  the whole gpu suite
#   bench  bench.py (BENCH_ARGS), its JSON line to gpurun_out/bench_$TAG.json
#   rehearse  bench.py --gpus 2 --dist-backend gloo (self-launched ranks on one GPU)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
TAG=${TAG:-r03}
STEPS=${STEPS:-dist}
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [[ $STEPS == *funnel* ]]; then
  # the bounding-box scan's funnel (groups / tiles passing / listed / tested / pair tests)
  for V in ${FUNNEL_KNOBS:-"SKY_MBR_ORDER=hilbert" "SKY_MBR_ORDER=morton"}; do
    T=$(echo $V | tr ' =' '__')
    env $V SKY_MBR_DBG=4 timeout -k 10 200 python -u tools/dom_bench.py ${MBR_N:-2000000} 3 > $OUT/funnel_${TAG}_$T.log 2>&1 || { tail -30 $OUT/funnel_${TAG}_$T.log; exit 1; }
    echo "$V"; grep -v "^\[mbr\]" $OUT/funnel_${TAG}_$T.log; grep "^\[mbr\]" $OUT/funnel_${TAG}_$T.log | tail -1
  done
fi
if [[ $STEPS == *c5probe* ]]; then
  for K in default ${C5KNOBS}; do
    for W in 0 10000000; do
      env ${K/default/SKY_X=0} SKY_MBR_DBG=4 timeout -k 10 200 python -u tools/c5_probe.py $W --phases > $OUT/c5probe_${TAG}_${K}_$W.log 2>&1 || { tail -30 $OUT/c5probe_${TAG}_${K}_$W.log; exit 1; }
      echo "$K W=$W"; grep pass $OUT/c5probe_${TAG}_${K}_$W.log
    done
  done
fi
if [[ $STEPS == *dist* ]]; then
  timeout -k 10 900 $PYT tests/test_gpu_dist_step.py tests/test_gpu_dist.py \
      "tests/test_gpu_operators.py::test_multi_rank_decomposition" "tests/test_gpu_configs.py::test_c4_8way_decomposition" \
      ${DIST_EXTRA} > $OUT/pytest_dist_$TAG.log 2>&1 || { tail -60 $OUT/pytest_dist_$TAG.log; exit 1; }
  tail -4 $OUT/pytest_dist_$TAG.log
fi
if [[ $STEPS == *parts* ]]; then
  timeout -k 10 600 $PYT tests/test_gpu_part.py tests/test_gpu_operators.py tests/test_gpu_replay.py \
      > $OUT/pytest_parts_$TAG.log 2>&1 || { tail -60 $OUT/pytest_parts_$TAG.log; exit 1; }
  tail -4 $OUT/pytest_parts_$TAG.log
fi
if [[ ,$STEPS, == *,tests,* ]]; then
  timeout -k 10 1000 $PYT tests -m gpu ${TEST_EXTRA} > $OUT/pytest_gpu_$TAG.log 2>&1 || { tail -60 $OUT/pytest_gpu_$TAG.log; exit 1; }
  tail -4 $OUT/pytest_gpu_$TAG.log
fi
if [[ ,$STEPS, == *,bench,* ]]; then
  timeout -k 10 500 python -u bench.py ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -30 $OUT/bench_$TAG.err; exit 1; }
  cut -c1-1500 $OUT/bench_$TAG.json
fi
if [[ $STEPS == *rehearse* ]]; then
  timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --tuples ${REH_TUPLES:-50000000} \
      > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err || { tail -30 $OUT/bench_gloo2_$TAG.err; exit 1; }
  grep '^{' $OUT/bench_gloo2_$TAG.json | cut -c1-1500
fi
if [[ $STEPS == *union* ]]; then
  timeout -k 10 300 python -u tools/dist_union_bench.py ${UNION_PER:-2000000} ${UNION_W:-4} > $OUT/dist_union_$TAG.json 2> $OUT/dist_union_$TAG.err || { tail -30 $OUT/dist_union_$TAG.err; exit 1; }
  cat $OUT/dist_union_$TAG.json
fi
if [[ $STEPS == *mbrpmc* ]]; then
  TAG=$TAG NS="${MBR_NS:-2000000 10000000}" bash tools/gpu_mbr_pmc.sh
fi
if [[ $STEPS == *c4ab* ]]; then
  # C4 alone, the round's default path and the A/B knobs in KNOBS (e.g. "SKY_PLANES=0")
  C4ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator"
  timeout -k 10 200 python -u bench.py $C4ARGS > $OUT/c4_$TAG.json 2> $OUT/c4_$TAG.err || { tail -30 $OUT/c4_$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_$TAG.json'));print('default', d['ms_per_step'], d['p50_query_latency_ms'], d['roofline']['avg_launch_ms'])"
  for K in ${KNOBS}; do
    env $K timeout -k 10 200 python -u bench.py $C4ARGS > $OUT/c4_${TAG}_$K.json 2> $OUT/c4_${TAG}_$K.err || { tail -30 $OUT/c4_${TAG}_$K.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/c4_${TAG}_$K.json'));print('$K', d['ms_per_step'], d['p50_query_latency_ms'], d['roofline']['avg_launch_ms'])"
  done
fi
if [[ $STEPS == *optrace* ]]; then
  # the operator path (sky_parts_insert flushes) under the kernel trace: GPU time per call vs host time
  export TMPDIR=/tmp
  rm -rf $OUT/optrace_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/optrace_$TAG -o run -- python3 -u tools/op_bench.py ${OP_N:-10000000} \
      > $OUT/optrace_$TAG.json 2> $OUT/optrace_$TAG.err || { tail -30 $OUT/optrace_$TAG.err; exit 1; }
  python3 tools/prof_summary.py trace $OUT/optrace_$TAG > $OUT/optrace_${TAG}_summary.txt
  head -16 $OUT/optrace_${TAG}_summary.txt
  cut -c1-600 $OUT/optrace_$TAG.json
fi
if [[ $STEPS == *filterpmc* ]]; then
  bash tools/gpu_pmc.sh $TAG
fi
if [[ $STEPS == *c5bench* ]]; then
  timeout -k 10 300 python -u bench.py --config C5 > $OUT/c5_$TAG.json 2> $OUT/c5_$TAG.err || { tail -30 $OUT/c5_$TAG.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c5_$TAG.json'))
for k in ('landmark','sliding_10M'):
    x=d[k]; print(k, 'p50', round(x['p50_query_latency_ms'],3), 'p90', round(x['p90_query_latency_ms'],3), 'max', round(x['max_query_latency_ms'],3), x['latencies_ms'])"
fi
if [[ $STEPS == *mbrtests* ]]; then
  timeout -k 10 600 $PYT tests/test_gpu_mbr.py tests/test_gpu_dist_step.py > $OUT/pytest_mbr_$TAG.log 2>&1 || { tail -60 $OUT/pytest_mbr_$TAG.log; exit 1; }
  tail -3 $OUT/pytest_mbr_$TAG.log
fi
if [[ $STEPS == *domab* ]]; then
  # the dominance companion (std-anti 8D) under the A/B knobs in DOMKNOBS, at each N in DOM_NS
  for N in ${DOM_NS:-2000000}; do
    for K in default ${DOMKNOBS}; do
      env ${K/default/SKY_X=0} timeout -k 10 300 python3 -u tools/dom_bench.py $N 2 > $OUT/domab_${TAG}_${K}_$N.json 2> $OUT/domab_${TAG}_${K}_$N.err \
          || { tail -20 $OUT/domab_${TAG}_${K}_$N.err; exit 1; }
      echo "$K N=$N $(cat $OUT/domab_${TAG}_${K}_$N.json)"
    done
  done
fi
if [[ $STEPS == *ophost* ]]; then
  # the operator path with the host-side split of every insert call (SKY_PART_HOSTPROF)
  SKY_PART_HOSTPROF=1 timeout -k 10 300 python3 -u tools/op_bench.py ${OP_N:-10000000} > $OUT/ophost_$TAG.json 2> $OUT/ophost_$TAG.err || { tail -30 $OUT/ophost_$TAG.err; exit 1; }
  grep "^\[part\]" $OUT/ophost_$TAG.err
  python3 -c "import json; d=json.load(open('$OUT/ophost_$TAG.json')); b=d['batched']; print('batched', b['insert_phase_s'], b['query_phase_s'], d['tuples_per_s'], b['p50_call_ms'])"
  for T in 1 2 8; do
    SKY_STAGE_THREADS=$T SKY_PART_HOSTPROF=1 timeout -k 10 300 python3 -u tools/op_bench.py ${OP_N:-10000000} > $OUT/ophost_${TAG}_t$T.json 2> $OUT/ophost_${TAG}_t$T.err || { tail -30 $OUT/ophost_${TAG}_t$T.err; exit 1; }
    echo "threads $T: $(grep '^\[part\]' $OUT/ophost_${TAG}_t$T.err | tail -1)"
  done
fi
if [[ $STEPS == *csvtests* ]]; then
  timeout -k 10 600 $PYT tests/test_gpu_csv.py tests/test_gpu_replay.py > $OUT/pytest_csv_$TAG.log 2>&1 || { tail -60 $OUT/pytest_csv_$TAG.log; exit 1; }
  tail -3 $OUT/pytest_csv_$TAG.log
fi
if [[ $STEPS == *csvpmc* ]]; then
  # instruction mix of k_csv_fields (one counter pass, kernel trace only), 20M records
  export TMPDIR=/tmp
  rm -rf $OUT/csvpmc_$TAG $OUT/csvpmc2_$TAG
  timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex k_csv_fields -f csv -d $OUT/csvpmc_$TAG -o run -- python3 -u $R/tools/csv_bench.py 20000000 > $OUT/csvpmc_$TAG.log 2>&1 || { tail -20 $OUT/csvpmc_$TAG.log; exit 1; }
  python tools/prof_summary.py pmcshow $OUT/csvpmc_$TAG k_csv_fields | tee $OUT/csvpmc_${TAG}_summary.txt
  if [ -n "$CSVPMC2" ]; then
    timeout -k 10 180 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
      --kernel-include-regex k_csv_fields -f csv -d $OUT/csvpmc2_$TAG -o run -- python3 -u $R/tools/csv_bench.py 20000000 > $OUT/csvpmc2_$TAG.log 2>&1 || { tail -20 $OUT/csvpmc2_$TAG.log; exit 1; }
    python tools/prof_summary.py pmcshow $OUT/csvpmc2_$TAG k_csv_fields | tee -a $OUT/csvpmc_${TAG}_summary.txt
  fi
fi
if [[ $STEPS == *csvab* ]]; then
  # the CSV companion (C4 stream as producer text) with the one-pass newline index and without
  for K in ${CSVKNOBS:-default}; do
    env ${K/default/SKY_X=0} timeout -k 10 300 python3 -u tools/csv_bench.py > $OUT/csvab_${TAG}_$K.json 2> $OUT/csvab_${TAG}_$K.err || { tail -20 $OUT/csvab_${TAG}_$K.err; exit 1; }
    echo "$K $(cut -c1-600 $OUT/csvab_${TAG}_$K.json)"
  done
fi
