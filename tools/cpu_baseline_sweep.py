#!/usr/bin/env python3
"""CPU baseline sweep: the reference algorithm restated in C (oracle/:
per-key BNL with 5000-tuple buffers, one thread per Flink subtask, single-threaded global
BNL merge — FlinkSkyline.java:265-316, :417-444, :548-566) timed over N and the subtask
count p, for the BASELINE configurations.  The reference's cost is quadratic in the
duplicate all-zero tuples its anti-correlated / correlated formulas produce,
so C2-C4 at full size (10M-100M) are out of reach: the sweep fits t(N) = a * N^alpha per
(config, p) and reports the extrapolation to the full size AS AN EXTRAPOLATION.

Output: one JSON document (stdout or --out).  Test infrastructure only: it times the
checker, never the product.
"""
import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import Oracle  # noqa: E402

CONFIGS = {
    "C1": dict(algo="dim", dims=2, dist=0, P=8, full=1_000_000, ns=[100_000, 250_000, 500_000, 1_000_000]),
    "C2": dict(algo="grid", dims=4, dist=1, P=8, full=10_000_000, ns=[100_000, 250_000, 500_000, 1_000_000]),
    "C3": dict(algo="angle", dims=4, dist=2, P=8, full=50_000_000, ns=[50_000, 100_000, 200_000, 400_000]),
    "C4": dict(algo="angle", dims=8, dist=2, P=16, full=100_000_000, ns=[25_000, 50_000, 100_000, 200_000]),
}


def fit_power(ns, ts):
    x = np.log(np.asarray(ns, float))
    y = np.log(np.asarray(ts, float))
    alpha, loga = np.polyfit(x, y, 1)
    return float(alpha), float(math.exp(loga))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4")
    ap.add_argument("--threads", default="1,4,8")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    orc = Oracle()
    res = {"host": platform.node(), "cpus": len(os.sched_getaffinity(0)), "kind": "port",
           "what": "oracle/ C restatement of the reference operators: per-key BNL (buffer 5000), one thread "
                   "per subtask (keys round-robin), single-threaded global BNL", "configs": {}}
    for name in args.configs.split(","):
        c = CONFIGS[name]
        seed = 1234 + c["dims"]
        nmax = max(c["ns"])
        vals = orc.synth(c["dist"], c["dims"], nmax, seed=seed)
        ids = np.arange(nmax, dtype=np.int64)
        rows = []
        for p in [int(x) for x in args.threads.split(",")]:
            for n in c["ns"]:
                t0 = time.perf_counter()
                if p == 1:
                    g, _, _, _ = orc.query_bnl(c["algo"], vals[:n], ids[:n], c["P"])
                else:
                    g, _, _, _ = orc.query_bnl_mt(c["algo"], vals[:n], ids[:n], c["P"], p)
                dt = time.perf_counter() - t0
                rows.append({"p": p, "n": n, "seconds": dt, "tuples_per_s": n / dt, "skyline": int(len(g))})
                print(name, rows[-1], file=sys.stderr, flush=True)
        fits = {}
        for p in sorted({r["p"] for r in rows}):
            rr = [r for r in rows if r["p"] == p]
            alpha, a = fit_power([r["n"] for r in rr], [r["seconds"] for r in rr])
            t_full = a * c["full"] ** alpha
            fits[str(p)] = {"alpha": alpha, "a": a, "full_n": c["full"], "extrapolated_seconds": t_full,
                            "extrapolated_tuples_per_s": c["full"] / t_full,
                            "note": "extrapolation of t = a * N^alpha fitted over the sweep, not a measurement"}
        res["configs"][name] = {"algo": c["algo"], "dims": c["dims"], "dist": c["dist"], "P": c["P"], "seed": seed,
                                "runs": rows, "fit": fits}
    txt = json.dumps(res, indent=1)
    if args.out:
        open(args.out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
