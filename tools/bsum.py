#!/usr/bin/env python3
"""Print the key numbers of a bench.py JSON line (the last JSON line of a file)."""
import json
import sys

lines = [l for l in open(sys.argv[1]).read().split("\n") if l.startswith("{")]
d = json.loads(lines[-1])
r = d.get("roofline") or {}
print(f"HEAD {d['config']['workload'][:40]}: {d['value']/1e9:.2f} G/s  {d['ms_per_step']:.3f} ms  p50 {d['p50_query_latency_ms']:.3f}"
      f"  filter {r.get('avg_launch_ms', 0):.3f} ms frac {r.get('frac', 0):.3f}")
print("  phases", {k: round(v, 3) for k, v in d.get("phases_ms_last_step", {}).items()})
print("  counters", d.get("counters_last_step"))
for k, v in (d.get("configs") or {}).items():
    if k == "C5":
        for w, x in v.items():
            print(f"  C5 {w}: ingest {x['ingest_tuples_per_s']/1e6:.0f} M/s p50 {x['p50_query_latency_ms']:.2f} "
                  f"p90 {x['p90_query_latency_ms']:.2f} max {x['max_query_latency_ms']:.2f}")
        continue
    rr = v.get("roofline") or {}
    cb = v.get("cpu_baseline") or {}
    print(f"  {k}: {v['value']/1e9:.2f} G/s {v['ms_per_step']:.3f} ms filter {rr.get('avg_launch_ms', 0):.3f} "
          f"frac {rr.get('frac', 0):.3f} cpu {cb.get('value', 0):.0f}/s", {a: round(b, 3) for a, b in v['phases_ms_last_step'].items()})
for k in ("dominance_roofline", "csv_ingest", "sort_roofline"):
    if d.get(k):
        x = d[k]
        print(f"  {k}: frac {x['frac']:.3f} achieved {x['achieved']:.4g} {x['unit']}",
              {a: round(x[a], 3) for a in ("ms_per_query", "global_sfs_ms", "local_sfs_ms", "decode_ms", "ms") if a in x})
if d.get("end_to_end"):
    for k, x in d["end_to_end"].items():
        print(f"  e2e {k}: {x['tuples_per_s']/1e9:.3f} G/s {x['ms_per_step']:.1f} ms")
