#!/bin/bash
# round-6 scratch GPU call (edited per call; each GPU step under its own limit, chained with &&)
set -e
export PYTHONUNBUFFERED=1
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out
timeout -k 10 120 tools/probe/valu_probe > $O/valu_probe_i.json 2>&1 || { cat $O/valu_probe_i.json; exit 1; }
cat $O/valu_probe_i.json
timeout -k 10 900 python -u bench.py > $O/bench_i.json 2> $O/bench_i.err || { tail -30 $O/bench_i.err; exit 1; }
cut -c1-1200 $O/bench_i.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
   --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $O/rehearsal2_i.json 2> $O/rehearsal2_i.err || { tail -30 $O/rehearsal2_i.err; exit 1; }
grep '^{' $O/rehearsal2_i.json | cut -c1-300
