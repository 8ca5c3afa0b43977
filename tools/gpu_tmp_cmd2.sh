#!/bin/bash
# scratch GPU command (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
for C in C4R C2 C5T; do for W in 256 128 64; do for rep in 1 2; do SKYLINE_HIP_LIB=flink-skyline-qos_amd/build_measure/libskyline_hip.so SKY_SAMPLE_WG=$W CFG=$C timeout -k 10 120 python -u tools/small_query_ab.py > $OUT/sw_${TAG}_${C}_$W.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads([l for l in open('$OUT/sw_${TAG}_${C}_$W.log') if l.startswith('{')][-1])
print('$C sample_wg=$W', 'entry_p50', round(d['c_entry_p50_ms'],4), 'min', round(d['c_entry_min_ms'],4))"
done; done; done
