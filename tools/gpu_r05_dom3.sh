#!/bin/bash
# round 5 late: the pair pass with the per-work-item-size register budget -- tests and the two dominance sizes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05m}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mbr.py tests/test_gpu_dist_step.py > ${O}_mbr.txt 2>&1 || exit 1
for n in 2000000 10000000; do
  timeout -k 10 200 python -u tools/dom_bench.py $n 3 >> ${O}_$n.json 2>&1 || exit 1
  timeout -k 10 200 python -u tools/dom_bench.py $n 3 >> ${O}_$n.json 2>&1 || exit 1
done
