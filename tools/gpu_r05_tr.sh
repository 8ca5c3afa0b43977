#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ${O}_def -o t -- python3 tools/dom_bench.py 2000000 3 > ${O}_def.log 2>&1 || exit 1
timeout -k 10 200 env SKY_PREFILTER=0 rocprofv3 --kernel-trace --stats -d ${O}_nopf -o t -- python3 tools/dom_bench.py 2000000 3 > ${O}_nopf.log 2>&1 || exit 1
