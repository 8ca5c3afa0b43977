#!/bin/bash
# scratch GPU command for the current A/B (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_configs.py tests/test_gpu_engine.py -m gpu > $OUT/plan_$TAG.log 2>&1 || { tail -40 $OUT/plan_$TAG.log; exit 1; }
tail -3 $OUT/plan_$TAG.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-dominance --no-csv --no-sort --no-e2e --no-operator > $OUT/bcfg_$TAG.json 2> $OUT/bcfg_$TAG.err || { tail -30 $OUT/bcfg_$TAG.err; exit 1; }
python3 tools/bsum.py $OUT/bcfg_$TAG.json
SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_TINY_CLK=1 CFG=C1 timeout -k 10 120 python -u tools/small_query_ab.py > $OUT/tclk_$TAG.log 2>&1 || { tail -20 $OUT/tclk_$TAG.log; exit 1; }
grep tiny-clk $OUT/tclk_$TAG.log | tail -4
