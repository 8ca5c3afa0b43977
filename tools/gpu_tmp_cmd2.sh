#!/bin/bash
# scratch GPU command (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
for C in C2 C3 C4R; do for MW in 1024 512 256; do for T in 4 8 16; do
SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_FILTER_MINWG=$MW SKY_FILTER_TPB=$T CFG=$C timeout -k 10 120 python -u tools/small_query_ab.py > $OUT/tpb_${TAG}_${C}_${MW}_$T.log 2>&1 || { tail -20 $OUT/tpb_${TAG}_${C}_${MW}_$T.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$OUT/tpb_${TAG}_${C}_${MW}_$T.log') if l.startswith('{')][-1])
print('$C', 'minwg', $MW, 'tpb', $T, 'entry_p50', round(d['c_entry_p50_ms'],4), 'filter', round(d['kernel_mean_ms_profiled'].get('filter',0),4))"
done; done; done
