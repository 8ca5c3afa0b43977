#!/usr/bin/env python3
"""Summarise rocprofv3 output for the skyline kernels.

  kernel-trace:  python tools/prof_summary.py trace <dir>            -> per-kernel stats (avg/total us)
  counters:      python tools/prof_summary.py pmc <dir> <kernel-substr> [--n N --dims D --dist X]
                 -> per-launch counter averages; with FETCH_SIZE / WRITE_SIZE it writes
                    profiles/traffic_filter.json (HBM bytes per launch)

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE
counts 64 B per 128-B request of a wide coalesced stream, i.e. HALF the bytes read,
so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are reported by
rocprofv3 in KiB.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(d, pattern):
    files = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                yield r


def _db_kernels(d):
    """(name, duration_ns) of every dispatch in rocprofv3's rocpd SQLite output."""
    import sqlite3
    for f in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
        con = sqlite3.connect(f)
        try:
            for name, dur in con.execute("select name, duration from kernels"):
                yield name, int(dur)
        finally:
            con.close()


def trace(d):
    agg = defaultdict(lambda: [0, 0.0])
    for r in _rows(d, "*kernel_trace.csv"):
        name = r.get("Kernel_Name", "?")
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        agg[name][0] += 1
        agg[name][1] += dt
    if not agg:
        for name, dur in _db_kernels(d):
            agg[name][0] += 1
            agg[name][1] += dur / 1000.0
    out = sorted(((v[1], k, v[0]) for k, v in agg.items()), reverse=True)
    tot = sum(v[0] for v in out) or 1.0
    print(f"{'total_us':>12} {'calls':>6} {'avg_us':>10} {'pct':>6}  kernel")
    for t, k, c in out[:40]:
        print(f"{t:12.1f} {c:6d} {t / c:10.2f} {100 * t / tot:6.1f}  {k[:110]}")
    return out


def pmc(d, sub, meta):
    per = defaultdict(lambda: defaultdict(float))
    for r in _rows(d, "*counter_collection.csv"):
        if sub not in r.get("Kernel_Name", ""):
            continue
        per[r.get("Dispatch_Id", r.get("Correlation_Id", "?"))][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        print("no dispatches matched", sub)
        return None
    names = sorted({c for v in per.values() for c in v})

    def _key(k):
        try:
            return int(k)
        except ValueError:
            return 0
    order = sorted(per, key=_key)
    # the first dispatch of a run is cold (k_filter: no designated duplicate group yet, so every
    # kept status word is stored); the steady state is every later one
    warm = order[1:] if len(order) > 1 else order
    avg = {c: sum(per[k].get(c, 0.0) for k in warm) / len(warm) for c in names}
    print(f"{len(per)} dispatches of *{sub}* (averaging the {len(warm)} warm ones)")
    for c in names:
        print(f"  {c:28s} {avg[c]:.6g}   per dispatch: " + " ".join(f"{per[k].get(c, 0.0):.6g}" for k in order))
    res = {"kernel_substr": sub, "dispatches": len(per), "warm_dispatches": len(warm), "avg": avg,
           "per_dispatch": {c: [per[k].get(c, 0.0) for k in order] for c in names}}
    res.update(meta)
    return res


def main():
    mode, d = sys.argv[1], sys.argv[2]
    if mode == "trace":
        trace(d)
        return
    if mode == "pmcshow":      # print per-launch averages only (no traffic file)
        import re
        rx = re.compile(sys.argv[3])
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in _rows(d, "*counter_collection.csv"):
            if not rx.search(r.get("Kernel_Name", "")):
                continue
            key = r.get("Dispatch_Id", "?")
            names[key] = r["Kernel_Name"]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        by_k = defaultdict(list)
        for key, c in per.items():
            by_k[names[key]].append(c)
        for kname, lst in by_k.items():
            cs = sorted({c for v in lst for c in v})
            print(f"{len(lst)} dispatches of {kname[:90]}")
            for c in cs:
                print(f"  {c:28s} {sum(v.get(c, 0.0) for v in lst) / len(lst):.6g}")
        return
    sub = sys.argv[3]
    meta = {}
    args = sys.argv[4:]
    for i in range(0, len(args), 2):
        k = args[i].lstrip("-")
        meta[k] = int(args[i + 1]) if args[i + 1].isdigit() else args[i + 1]
    res = pmc(d, sub, meta)
    if res is None:
        return
    out = os.path.join(REPO, "profiles", "traffic_filter.json")
    old = json.load(open(out)) if os.path.exists(out) else {}
    old.update({k: v for k, v in res.items() if k not in ("avg", "per_dispatch")})
    old.setdefault("counters_per_dispatch", {}).update(res["per_dispatch"])
    old["note"] = ("counters averaged over the warm dispatches (every one after a run's first, which runs "
                   "before the designated duplicate group is known); per dispatch values in "
                   "counters_per_dispatch, in dispatch order")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from src_hash import kernel_src_sha
    old["kernel_src_sha"] = kernel_src_sha("k_filter")     # bench.py reports it for this build only
    old.setdefault("counters", {}).update(res["avg"])
    c = old["counters"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd = 2.0 * c["FETCH_SIZE"] * 1024.0      # gfx950: FETCH_SIZE reads half of a wide stream
        wr = c["WRITE_SIZE"] * 1024.0
        old["hbm_read_bytes_per_launch"] = rd
        old["hbm_write_bytes_per_launch"] = wr
        old["hbm_bytes_per_launch"] = rd + wr
        old["correction"] = "read = 2 x FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB"
    json.dump(old, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__" and sys.argv[1] != "timeline":
    main()


def timeline(d, last_n=120):
    """The last `last_n` dispatches in start order: name, start offset (us), duration, gap."""
    rows = []
    for r in _rows(d, "*kernel_trace.csv"):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?")))
    rows.sort()
    rows = rows[-last_n:]
    t0 = rows[0][0]
    prev_end = t0
    for s, e, n in rows:
        print(f"{(s - t0) / 1000:10.1f} {(e - s) / 1000:9.1f} gap {(s - prev_end) / 1000:8.1f}  {n[:90]}")
        prev_end = max(prev_end, e)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "timeline":
    timeline(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 120)
