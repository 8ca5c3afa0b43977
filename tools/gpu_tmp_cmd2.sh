#!/bin/bash
# round-6 scratch GPU call 2: small-query A/B (product; measurement-build filter tiles per workgroup)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out
ML=flink-skyline-qos_amd/build_measure/libskyline_hip.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist_step.py tests/test_gpu_dist.py \
   "tests/test_gpu_configs.py::test_c4_8way_decomposition" "tests/test_gpu_configs.py::test_c3_angle_4d_anti_50m_one_gpu_and_sharded" \
   tests/test_gpu_operators.py > $O/disttests_g.log 2>&1 || { tail -40 $O/disttests_g.log; exit 1; }
tail -2 $O/disttests_g.log
timeout -k 10 600 python -u tools/dist_phases.py --only c4_8way,c3_8way --out $O/r06_dist_phases_g.json > $O/distphases_g.log 2>&1 || { tail -30 $O/distphases_g.log; exit 1; }
grep '^{' $O/distphases_g.log | cut -c1-600
: > $O/sq_g.log
for c in C1 C2 C5T C4R; do
  CFG=$c timeout -k 10 120 python -u tools/small_query_ab.py >> $O/sq_g.log 2>&1 || { tail -20 $O/sq_g.log; exit 1; }
done
for t in 1 2 4 8; do
  CFG=C4R SKYLINE_HIP_LIB=$ML SKY_FILTER_TPB=$t timeout -k 10 120 python -u tools/small_query_ab.py >> $O/sq_g.log 2>&1 || { tail -20 $O/sq_g.log; exit 1; }
done
grep '^{' $O/sq_g.log
timeout -k 10 200 python -u tools/dense_bench.py 16384 65536 > $O/dense_g.log 2>&1 || { tail -20 $O/dense_g.log; exit 1; }
grep '^{' $O/dense_g.log
export TMPDIR=/tmp
i=0
for CS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD" \
          "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" \
          "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  rm -rf $O/pmc_dense_$i
  timeout -k 10 180 rocprofv3 --pmc $CS --kernel-include-regex "k_brute16_pairs" -f csv -d $O/pmc_dense_$i -o run -- \
      python3 -u tools/dense_bench.py 65536 > $O/pmc_dense_$i.log 2>&1 || { tail -20 $O/pmc_dense_$i.log; exit 1; }
  python tools/prof_summary.py pmcshow $O/pmc_dense_$i "k_brute16_pairs" | tee -a $O/pmc_dense.txt
  rm -rf $O/pmc_dense_$i
done
