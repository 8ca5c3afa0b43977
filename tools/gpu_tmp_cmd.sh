#!/bin/bash
# round-6 scratch GPU call (edited per call; each GPU step under its own limit, chained with &&)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out
ML=flink-skyline-qos_amd/build_measure/libskyline_hip.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_plan.py \
    tests/test_gpu_configs.py > $O/tests_h.log 2>&1 || { tail -40 $O/tests_h.log; exit 1; }
tail -2 $O/tests_h.log
timeout -k 10 200 python -u tools/dense_bench.py 16384 65536 > $O/dense_h.log 2>&1 || { tail -20 $O/dense_h.log; exit 1; }
grep '^{' $O/dense_h.log
export TMPDIR=/tmp
i=0
for CS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD" \
          "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" \
          "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  rm -rf $O/pmc_dense_$i
  timeout -k 10 180 rocprofv3 --pmc $CS --kernel-include-regex "k_brute16_pairs" -f csv -d $O/pmc_dense_$i -o run -- \
      python3 -u tools/dense_bench.py 65536 > $O/pmc_dense_$i.log 2>&1 || { tail -20 $O/pmc_dense_$i.log; exit 1; }
  python tools/prof_summary.py pmcshow $O/pmc_dense_$i "k_brute16_pairs" | tee -a $O/pmc_dense_h.txt
  rm -rf $O/pmc_dense_$i
done
for yt in 1 2; do
  SKYLINE_HIP_LIB=$ML SKY_MBR_YT=$yt timeout -k 10 600 python -u tools/dist_phases.py --only std_anti_4x2M > $O/union_yt$yt.log 2>&1 || { tail -20 $O/union_yt$yt.log; exit 1; }
  grep '^{' $O/union_yt$yt.log | cut -c1-900
done
