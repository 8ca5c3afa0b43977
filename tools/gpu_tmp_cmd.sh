#!/bin/bash
# scratch GPU command for the current A/B (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_engine.py tests/test_gpu_configs.py -m gpu > $OUT/st_$TAG.log 2>&1 || { tail -40 $OUT/st_$TAG.log; exit 1; }
tail -2 $OUT/st_$TAG.log
for C in C2 C1; do for k in 1 0; do SKY_SPARSE_OUT=$k CFG=$C timeout -k 10 120 python -u tools/small_query_ab.py > $OUT/sp_${TAG}_${C}_$k.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads([l for l in open('$OUT/sp_${TAG}_${C}_$k.log') if l.startswith('{')][-1])
print('$C sparse=$k', 'entry_p50', round(d['c_entry_p50_ms'],4), {a: round(b,4) for a,b in d['kernel_mean_ms_profiled'].items()})"
done; done
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-dominance --no-csv --no-sort --no-e2e --no-operator --no-stream > $OUT/bcfg_$TAG.json 2> $OUT/bcfg_$TAG.err || { tail -30 $OUT/bcfg_$TAG.err; exit 1; }
python3 tools/bsum.py $OUT/bcfg_$TAG.json
