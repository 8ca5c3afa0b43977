#!/bin/bash
# round 5 final tree: the whole GPU suite, the default bench line, C4 / C1 / C2 traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan.py > ${O}_plan.txt 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_pytest.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > ${O}_bench_full.json 2> ${O}_bench_full.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c4prof -o t -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort --no-configs --no-e2e --no-operator > ${O}_c4prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c1prof -o t -- python3 bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c2prof -o t -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c2prof.log 2>&1 || exit 1
