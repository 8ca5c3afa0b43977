#!/bin/bash
# k_mbr_pairs evidence on the dominance-bound companion (std-anti 8D, MR-Angle P=16):
# PMC instruction mix / wait counters (one rocprofv3 --pmc pass per counter group,
# kernel-trace only, each under its own time limit) and the pass's growth with N.
#   TAG=r03 NS="2000000 10000000" bash tools/gpu_mbr_pmc.sh
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r03}
KRE=${KRE:-k_mbr_pairs}
PMC_N=${PMC_N:-2000000}
NS=${NS-"2000000 10000000"}
if [ -z "$SKIP_PMC" ]; then
  i=0
  for CS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    rm -rf $OUT/pmc_mbr_${TAG}_$i
    timeout -k 10 240 rocprofv3 --pmc $CS --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_mbr_${TAG}_$i -o run -- \
        python3 -u $R/tools/dom_bench.py $PMC_N 1 > $OUT/pmc_mbr_${TAG}_$i.log 2>&1 \
        || { tail -20 $OUT/pmc_mbr_${TAG}_$i.log; exit 1; }
    python tools/prof_summary.py pmcshow $OUT/pmc_mbr_${TAG}_$i "$KRE" | tee -a $OUT/pmc_mbr_${TAG}.txt
  done
fi
for N in $NS; do
  timeout -k 10 300 python3 -u tools/dom_bench.py $N 2 > $OUT/dom_${TAG}_$N.json 2> $OUT/dom_${TAG}_$N.err \
      || { tail -20 $OUT/dom_${TAG}_$N.err; exit 1; }
  cat $OUT/dom_${TAG}_$N.json
done
