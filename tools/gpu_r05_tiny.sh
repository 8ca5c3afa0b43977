#!/bin/bash
# round 5: the one-workgroup planned tail -- its parity tests, the C1 / C2 / C5 lines, C1's and C2's launches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05t}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_configs.py > ${O}_pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1.json 2> ${O}_c1.err || exit 1
SKY_TINY=0 timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1_notiny.json 2>> ${O}_c1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c1prof -o t -- python3 bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c2prof -o t -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c2prof.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline > ${O}_c5.json 2> ${O}_c5.err || exit 1
