#!/bin/bash
# scratch GPU command for the current A/B (not part of the record)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
TAG=$1
export TMPDIR=/tmp
rm -rf $OUT/c5tl_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/c5tl_$TAG -o run -- python3 -u -c "
import sys, time; sys.path.insert(0, 'flink-skyline-qos_amd')
import numpy as np, skyline
from skyline import _abi
D, P, per, batch, trig = 6, 8, 1000000, 50000, 6
vals, ids = skyline.synth_host(_abi.DISTS['mixed'], D, per * trig, seed=1240)
eng = skyline.SkylineEngine(D, P, 'mr-angle', 1000.0, 0)
eng.warmup()
st = skyline.SkylineStream(eng, 0)
st.reserve(per * trig)
lat = []
for t in range(trig):
    for b0 in range(t * per, (t + 1) * per, batch):
        st.append(ids[b0:b0 + batch], vals[b0:b0 + batch])
    t0 = time.perf_counter(); st.query_async_host_view(); lat.append((time.perf_counter() - t0) * 1e3)
    st.wait()
print('latencies_ms', [round(x, 3) for x in lat])
st.close(); eng.close()
" > $OUT/c5tl_$TAG.log 2>&1 || { tail -30 $OUT/c5tl_$TAG.log; exit 1; }
python3 tools/prof_summary.py timeline $OUT/c5tl_$TAG 60 > $OUT/c5tl_${TAG}.txt
rm -rf $OUT/c5tl_$TAG
grep latencies $OUT/c5tl_$TAG.log; tail -34 $OUT/c5tl_${TAG}.txt
