#!/bin/bash
# Round-4 GPU pass: STEPS (comma list) of
#   tests   the whole gpu suite (PYTEST_ARGS narrows it)
#   bench   bench.py (BENCH_ARGS) -> gpurun_out/bench_$TAG.json
#   dom     tools/dom_bench.py at 2M and 10M std-anti (DOM_ARGS)
#   trace   rocprofv3 kernel-trace of bench.py (BENCH_ARGS)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
TAG=${TAG:-r04}
STEPS=${STEPS:-tests}
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 $PYT -m gpu ${PYTEST_ARGS:-tests} > $OUT/pytest_$TAG.log 2>&1 || { tail -60 $OUT/pytest_$TAG.log; exit 1; }
  tail -3 $OUT/pytest_$TAG.log
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
  tail -2 $OUT/smoke_$TAG.log
fi
if [[ $STEPS == *dom* ]]; then
  for N in ${DOM_NS:-2000000 10000000}; do
    timeout -k 10 300 python -u tools/dom_bench.py $N 3 ${DOM_ARGS} > $OUT/dom_${TAG}_$N.log 2>&1 || { tail -30 $OUT/dom_${TAG}_$N.log; exit 1; }
    tail -3 $OUT/dom_${TAG}_$N.log
  done
fi
if [[ $STEPS == *mtrace* ]]; then
  # measurement build: the pair pass's per-work-item timeline (SKY_MBR_DBG=8)
  # MBR_VARIANTS: space-separated variants, each a comma-separated list of NAME=VALUE
  for V in ${MBR_VARIANTS:-SKY_MBR_ORDER=hilbert}; do
  for N in ${DOM_NS:-2000000 10000000}; do
    env ${V//,/ } SKYLINE_HIP_LIB=$R/flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_MBR_DBG=${MBR_DBG:-8} \
      timeout -k 10 300 python -u tools/dom_bench.py $N 2 > $OUT/mtrace_${TAG}_${V}_$N.log 2>&1 || { tail -30 $OUT/mtrace_${TAG}_${V}_$N.log; exit 1; }
    echo "$V $N"; grep "mbr-trace" $OUT/mtrace_${TAG}_${V}_$N.log | tail -2; tail -1 $OUT/mtrace_${TAG}_${V}_$N.log | cut -c1-200
  done
  done
fi
if [[ $STEPS == *mdbg* ]]; then
  # measurement build, results invalid: SKY_MBR_DBG=1 stops each tile after its box tests
  # (the scan + corner-test cost), =2 after the group / tile scans
  for M in ${MBR_DBGS:-1 2}; do
  for N in ${DOM_NS:-2000000 10000000}; do
    SKYLINE_HIP_LIB=$R/flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_MBR_DBG=$M \
      timeout -k 10 300 python -u tools/dom_bench.py $N 2 > $OUT/mdbg_${TAG}_${M}_$N.log 2>&1 || { tail -30 $OUT/mdbg_${TAG}_${M}_$N.log; exit 1; }
    echo "dbg=$M $N $(tail -1 $OUT/mdbg_${TAG}_${M}_$N.log | cut -c1-160)"
  done
  done
fi
if [[ $STEPS == *mpmc* ]]; then
  TAG=$TAG NS="" KRE=k_mbr_pairs PMC_N=${PMC_N:-2000000} bash tools/gpu_mbr_pmc.sh
fi
if [[ $STEPS == *cpmc* ]]; then
  # k_csv_fields (chunk route) on the C4 stream as producer text: instruction mix + HBM bytes
  export TMPDIR=/tmp
  i=0
  for CS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    rm -rf $OUT/pmc_csv_${TAG}_$i
    timeout -s KILL 120 rocprofv3 --pmc $CS --kernel-include-regex "k_csv_fields" -f csv -d $OUT/pmc_csv_${TAG}_$i -o run -- \
        python3 -u $R/tools/csv_bench.py 20000000 > $OUT/pmc_csv_${TAG}_$i.log 2>&1 || { tail -20 $OUT/pmc_csv_${TAG}_$i.log; exit 1; }
    python tools/prof_summary.py pmcshow $OUT/pmc_csv_${TAG}_$i "k_csv_fields" | tee -a $OUT/pmc_csv_${TAG}.txt
  done
fi
if [[ $STEPS == *fpmc* ]]; then
  bash tools/gpu_pmc.sh $TAG
fi
if [[ $STEPS == *rehearse* ]]; then
  # two ranks on the one GPU over gloo (bench.py starts its own ranks): the per-step phase split
  timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/rehearsal_$TAG.json 2> $OUT/rehearsal_$TAG.err || { tail -30 $OUT/rehearsal_$TAG.err; exit 1; }
  cut -c1-600 $OUT/rehearsal_$TAG.json
fi
if [[ $STEPS == *csv* ]]; then
  for C in 1 0; do
    SKY_CSV_CHUNKS=$C timeout -k 10 240 python -u tools/csv_bench.py > $OUT/csv_${TAG}_$C.log 2>&1 || { tail -30 $OUT/csv_${TAG}_$C.log; exit 1; }
    echo "chunks=$C $(tail -1 $OUT/csv_${TAG}_$C.log)"
  done
fi
if [[ $STEPS == *probe* ]]; then
  timeout -k 10 120 ./tools/probe/filter_probe > $OUT/filter_probe_$TAG.log 2>&1 || { tail -20 $OUT/filter_probe_$TAG.log; exit 1; }
  cat $OUT/filter_probe_$TAG.log
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -30 $OUT/bench_$TAG.err; exit 1; }
  cut -c1-1500 $OUT/bench_$TAG.json
fi
if [[ $STEPS == *dtrace* ]]; then
  export TMPDIR=/tmp
  for N in ${DOM_NS:-2000000 10000000}; do
    rm -rf $OUT/dtrace_${TAG}_$N
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/dtrace_${TAG}_$N -o run -- python3 -u $R/tools/dom_bench.py $N 2 > $OUT/dtrace_${TAG}_$N.log 2>&1 || { tail -30 $OUT/dtrace_${TAG}_$N.log; exit 1; }
    python tools/prof_summary.py trace $OUT/dtrace_${TAG}_$N > $OUT/dtrace_${TAG}_${N}_summary.txt
    head -16 $OUT/dtrace_${TAG}_${N}_summary.txt
  done
fi
if [[ $STEPS == *ktrace* ]]; then
  export TMPDIR=/tmp
  rm -rf $OUT/trace_$TAG
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$TAG -o run -- python3 -u $R/bench.py ${BENCH_ARGS} > $OUT/trace_$TAG.log 2>&1 || { tail -30 $OUT/trace_$TAG.log; exit 1; }
  python tools/prof_summary.py trace $OUT/trace_$TAG > $OUT/trace_${TAG}_summary.txt
  head -30 $OUT/trace_${TAG}_summary.txt
fi
