#!/bin/bash
# round 5: k_tiny_tail's instruction mix / waits on C1 (one rocprofv3 --pmc pass per counter group),
# then the plan tests and the C1 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05p}
i=0
for CS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
          "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
          "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  rm -rf ${O}_pmc_$i
  timeout -k 10 120 rocprofv3 --pmc $CS --kernel-include-regex k_tiny_tail -f csv -d ${O}_pmc_$i -o run -- \
      python3 -u bench.py --config C1 --steps 5 --warmup 2 --no-cpu-baseline > ${O}_pmc_$i.log 2>&1 || exit 1
  python tools/prof_summary.py pmcshow ${O}_pmc_$i k_tiny_tail >> ${O}_pmc.txt || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_engine.py > ${O}_pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1.json 2> ${O}_c1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_c1prof -o t -- python3 bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > ${O}_c1prof.log 2>&1 || exit 1
