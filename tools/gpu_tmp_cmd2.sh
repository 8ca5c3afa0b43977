#!/bin/bash
# round-6 scratch GPU call 2: k_filter rows in flight per lane (PF 1 / 2) by stream size (measurement build)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out
ML=flink-skyline-qos_amd/build_measure/libskyline_hip.so
timeout -k 10 60 tools/probe/valu_probe > $O/valu_probe_j.json 2>&1 && cat $O/valu_probe_j.json
: > $O/pf_j.log
for c in C1 C5T C3R C2 C4R C4H C3; do
  for pf in 1 2; do
    CFG=$c SKYLINE_HIP_LIB=$ML SKY_FILTER_PF=$pf timeout -k 10 120 python -u tools/small_query_ab.py >> $O/pf_j.log 2>&1 || { tail -20 $O/pf_j.log; exit 1; }
  done
done
grep '^{' $O/pf_j.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = d['kernel_mean_ms_profiled']
    print(d['config'], 'pf', d['filter_pf'], 'wall', round(d['wall_p50_ms'], 4), 'c_entry', round(d['c_entry_p50_ms'], 4), 'filter_ms', round(k.get('filter', 0), 4))
"
