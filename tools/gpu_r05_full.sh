#!/bin/bash
# round 5: full GPU suite, the dominance companion at 2M / 10M, region clocks + funnel from the
# measurement build, and the C4 headline alone
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_pytest.log 2>&1 || exit 1
for n in 2000000 10000000; do
  timeout -k 10 200 python -u tools/dom_bench.py $n 3 > ${O}_dom_$n.json 2>&1 || exit 1
done
M=flink-skyline-qos_amd/build_measure/libskyline_hip.so
for n in 2000000 10000000; do
  timeout -k 10 200 env SKYLINE_HIP_LIB=$M SKY_MBR_DBG=20 python -u tools/dom_bench.py $n 1 > ${O}_domclock_$n.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator > ${O}_c4.json 2> ${O}_c4.err || exit 1
