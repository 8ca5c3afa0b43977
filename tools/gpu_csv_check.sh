#!/bin/bash
# CSV parity tests + the CSV-ingest companion timing (GPU box), each step under its own limit.
set -e
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_csv.py tests/test_gpu_replay.py -x -q --timeout 300 --timeout-method thread > $OUT/pt_csv.log 2>&1 || { tail -30 $OUT/pt_csv.log; exit 1; }
tail -2 $OUT/pt_csv.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dominance --no-stream --no-sort --no-configs --no-e2e --no-operator > $OUT/b_csv.json 2> $OUT/b_csv.err || { tail -20 $OUT/b_csv.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/b_csv.json').read().strip().splitlines()[-1]); c = d['csv_ingest']
print('decode_ms', round(c['decode_ms'], 3), {k: round(v, 3) for k, v in c['kernel_ms'].items()}, 'frac', round(c['frac'], 3))"
