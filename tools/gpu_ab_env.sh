#!/bin/bash
# A/B of the k_filter stream under one environment variable: VAR=name VALUES="a b c"
# runs tools/filter_ab.py once per value (each under its own time limit).
set -e
mkdir -p gpurun_out
for v in $VALUES; do
  env $VAR=$v timeout -k 10 150 python3 -u tools/filter_ab.py > gpurun_out/ab_${VAR}_$v.json
  python3 -c "import json;d=json.load(open('gpurun_out/ab_${VAR}_$v.json'));print('$VAR=$v', {k:(round(v['filter_ms'],3),round(v['GBps'])) for k,v in d.items()})"
done
