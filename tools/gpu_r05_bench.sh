#!/bin/bash
# round 5: the default bench line (every companion) and the kernel traces committed under profiles/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05b}
timeout -k 10 600 python -u bench.py > ${O}_bench_full.json 2> ${O}_bench_full.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c4prof -o t -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator > ${O}_c4prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c1prof -o t -- python3 bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_domprof -o t -- python3 tools/dom_bench.py 10000000 2 > ${O}_domprof.log 2>&1 || exit 1
