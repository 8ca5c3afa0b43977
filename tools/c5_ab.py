#!/usr/bin/env python3
"""C5 landmark / sliding trigger latency A/B: the engine on the process's torch stream
(use_torch_stream, the bench default) vs on its own stream (BENCH_OWN_STREAM=1), same box."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream(device=torch.device("cuda", 0)))
for rep in range(2):
    for own in ("", "1"):
        if own:
            os.environ["BENCH_OWN_STREAM"] = "1"
        else:
            os.environ.pop("BENCH_OWN_STREAM", None)
        r = bench.stream_run(0, 1234 + 6)
        print(json.dumps({"own_stream": bool(own), "rep": rep, "p50": r["p50_query_latency_ms"],
                          "p90": r["p90_query_latency_ms"], "ingest": r["ingest_tuples_per_s"]}), flush=True)
