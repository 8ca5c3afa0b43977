#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, bench, rocprofv3 kernel-trace of the bench.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
TAG=${1:-r01}
STEPS=${STEPS:-tests,smoke,bench,trace}
export PYTHONUNBUFFERED=1
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -30 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
if [[ $STEPS == *dist* ]]; then
  # two ranks rehearsed on the one GPU over gloo (the driver's 8-GPU run uses RCCL)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --tuples 50000000 \
      > $OUT/bench_dist2_$TAG.json 2> $OUT/bench_dist2_$TAG.err || { tail -30 $OUT/bench_dist2_$TAG.err; exit 1; }
  grep '^{' $OUT/bench_dist2_$TAG.json | cut -c1-400
fi
if [[ $STEPS == *trace* ]]; then
  export TMPDIR=/tmp
  rm -rf $OUT/trace_$TAG
  # C4 alone (the bench line's k_filter), then the dominance-bound companion alone
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$TAG -o run -- python3 -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dominance ${BENCH_ARGS} > $OUT/trace_$TAG.log 2>&1 || { tail -30 $OUT/trace_$TAG.log; exit 1; }
  grep '^{' $OUT/trace_$TAG.log > $OUT/bench_trace_$TAG.json || true
  python tools/prof_summary.py trace $OUT/trace_$TAG > $OUT/trace_${TAG}_summary.txt
  head -25 $OUT/trace_${TAG}_summary.txt
  rm -rf $OUT/trace_dom_$TAG
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_dom_$TAG -o run -- python3 -u $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dominance --dist std_anti --tuples 2000000 > $OUT/trace_dom_$TAG.log 2>&1 || { tail -30 $OUT/trace_dom_$TAG.log; exit 1; }
  python tools/prof_summary.py trace $OUT/trace_dom_$TAG > $OUT/trace_dom_${TAG}_summary.txt
  head -12 $OUT/trace_dom_${TAG}_summary.txt
fi
