"""A C caller of the ABI (tests/operator_replay.c, built by the package Makefile as
build/operator_replay) replays the reference operators' call sequence -- device CSV decode,
getKey, per-key 5000-tuple buffers flushed through sky_part_insert, a trigger after the last
tuple answered by sky_part_snapshot per key, sky_global_merge + sky_global_stats, the JSON of
FlinkSkyline.java:631-648 -- exactly as the JNI shim (jni/skyline_hip_jni.c) drives the
library from the Java operators (full buffers grouped into sky_parts_insert calls, as
HipSkylineOperators does).  Its output must equal the golden results, also with single-buffer
inserts, and across a checkpoint -> close -> reopen -> restore-by-insert in mid-stream."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, golden_streams, load_golden

pytestmark = pytest.mark.gpu

BIN = os.path.join(REPO, "flink-skyline-qos_amd", "build", "operator_replay")
ALGO = {"dim": 0, "grid": 1, "angle": 2}


def java_format_4f(x):
    import decimal
    d = decimal.Decimal(repr(float(x)))
    return str(d.quantize(decimal.Decimal("0.0001"), rounding=decimal.ROUND_HALF_UP))


@pytest.mark.parametrize("path", [p for p in golden_streams() if "_2d" in p or "_4d" in p or "_8d" in p],
                         ids=lambda p: os.path.basename(p)[7:-4])
def test_c_caller_replays_operator_sequence(path, tmp_path):
    assert os.path.exists(BIN), "build/operator_replay missing: run __graft_entry__.build()"
    g = load_golden(path)
    vals, ids = g["values"], g["ids"]
    D = vals.shape[1]
    csv = tmp_path / "stream.csv"
    with open(csv, "w") as f:   # the producers' payload, python/unified_producer.py:174
        for i, row in zip(ids, vals):
            f.write(f"{int(i)}," + ",".join(str(int(x)) for x in row) + "\n")
    n = len(ids)
    # (domain, checkpoint position or -1, buffers per sky_parts_insert group)
    modes = [[], ["1000.0", str(n // 2), "8"], ["1000.0", "-1", "1"], ["1000.0", str(n // 3), "3"]]
    for algo in ("dim", "grid", "angle"):
        for P in (4, 8, 16):
            for extra in modes:
                r = subprocess.run([BIN, str(csv), str(D), str(P // 2), str(ALGO[algo])] + extra,
                                   capture_output=True, text=True, timeout=120)
                assert r.returncode == 0, r.stderr
                lines = r.stdout.strip().split("\n")
                js = json.loads(lines[0])
                got_ids = np.array([int(x) for x in lines[1].split()[1:]], np.int64)
                lsz = np.array([int(x) for x in lines[2].split()[1:]], np.int64)
                surv = np.array([int(x) for x in lines[3].split()[1:]], np.int64)
                np.testing.assert_array_equal(got_ids, np.sort(ids[g[f"gsky_{algo}_{P}"]]))
                np.testing.assert_array_equal(lsz, g[f"lsz_{algo}_{P}"])
                np.testing.assert_array_equal(surv, g[f"surv_{algo}_{P}"])
                assert js["skyline_size"] == len(got_ids) and js["record_count"] == len(ids)
                opt = sum(surv[i] / lsz[i] for i in range(P) if lsz[i] > 0) / P
                assert lines[0].split('"optimality": ')[1].split(",")[0] == java_format_4f(opt)
                assert "query_latency_ms" in js


def _drain_model(keys, P, group, buf=5000):
    """HipSkylineOperators.drainFull's call sequence: (calls, parts over all calls)."""
    fill = {}
    full = []
    calls = parts = 0

    def drain():
        nonlocal full, calls, parts
        while full:
            seen, rnd, later = set(), [], []
            for k in full:
                (later if k in seen else rnd).append(k)
                seen.add(k)
            calls += 1
            parts += len(rnd)
            full = later
    for k in keys.tolist():
        fill[k] = fill.get(k, 0) + 1
        if fill[k] == buf:
            fill[k] = 0
            full.append(k)
            if len(full) >= group:
                drain()
    drain()
    return calls, parts


@pytest.mark.parametrize("dist,D,algo,proto", [(2, 8, "angle", 0), (2, 8, "angle", 1), (3, 4, "angle", 0),
                                               (1, 4, "grid", 0), (0, 2, "dim", 0)])
def test_c_caller_java_sequence_large(dist, D, algo, proto, tmp_path, oracle):
    """The operators' exact call sequence at a size where buffers fill: drainFull rounds of
    sky_parts_insert (arrival order, one buffer per key per round, every 8 full buffers), then per
    key flush + sky_part_sizes + sky_part_snapshot_reps and sky_global_merge_reps (proto 0, the
    Java operators' LocalSkyline messages) or the round-3 ids + values messages (proto 1).  The
    answer equals the oracle's two-level skyline, and the calls equal the drainFull model's."""
    n, P = 240_000, 8
    vals = oracle.synth(dist, D, n, seed=300 + D)
    ids = np.arange(n, dtype=np.int64) + 7
    csv = tmp_path / "stream.csv"
    with open(csv, "w") as f:
        for i, row in zip(ids, vals):
            f.write(f"{int(i)}," + ",".join(str(int(x)) for x in row) + "\n")
    r = subprocess.run([BIN, str(csv), str(D), str(P // 2), str(ALGO[algo]), "1000.0", "-1", "8", str(proto)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    got_ids = np.array([int(x) for x in lines[1].split()[1:]], np.int64)
    lsz = np.array([int(x) for x in lines[2].split()[1:]], np.int64)
    surv = np.array([int(x) for x in lines[3].split()[1:]], np.int64)
    e_or, _, e_ls, e_sv = oracle.query_sfs(algo, vals, P)
    np.testing.assert_array_equal(got_ids, np.sort(ids[e_or]))
    np.testing.assert_array_equal(lsz, e_ls)
    np.testing.assert_array_equal(surv, e_sv)
    calls = [ln for ln in r.stderr.split("\n") if ln.startswith("calls ")][-1].split()
    keys = oracle.keys(algo, vals, P)
    assert (int(calls[1]), int(calls[3])) == _drain_model(keys, P, 8)
    assert int(calls[1]) > 0


@pytest.mark.parametrize("path", [p for p in golden_streams() if "_4d" in p or "_8d" in p],
                         ids=lambda p: os.path.basename(p)[7:-4])
def test_c_caller_stats_count_differs_from_partitions(path, tmp_path):
    """proto 2: the aggregator merges the P triggered keys' messages plus empty messages of the
    MR-Grid keys >= P that hold state but never receive the trigger, so sky_global_stats' K (one
    entry per list) is not P.  The caller sizes its arrays from the K the library returns (as
    HipSkylineOperators does), sums only partitions < P, and the answer is unchanged."""
    assert os.path.exists(BIN), "build/operator_replay missing: run __graft_entry__.build()"
    g = load_golden(path)
    vals, ids = g["values"], g["ids"]
    D = vals.shape[1]
    csv = tmp_path / "stream.csv"
    with open(csv, "w") as f:
        for i, row in zip(ids, vals):
            f.write(f"{int(i)}," + ",".join(str(int(x)) for x in row) + "\n")
    seen_k_ne_p = False
    for P in (4, 8):
        r = subprocess.run([BIN, str(csv), str(D), str(P // 2), str(ALGO["grid"]), "1000.0", "-1", "8", "2"],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        lines = r.stdout.strip().split("\n")
        got_ids = np.array([int(x) for x in lines[1].split()[1:]], np.int64)
        lsz = np.array([int(x) for x in lines[2].split()[1:]], np.int64)
        surv = np.array([int(x) for x in lines[3].split()[1:]], np.int64)
        np.testing.assert_array_equal(got_ids, np.sort(ids[g[f"gsky_grid_{P}"]]))
        np.testing.assert_array_equal(lsz, g[f"lsz_grid_{P}"])
        np.testing.assert_array_equal(surv, g[f"surv_grid_{P}"])
        opt = sum(surv[i] / lsz[i] for i in range(P) if lsz[i] > 0) / P
        assert lines[0].split('"optimality": ')[1].split(",")[0] == java_format_4f(opt)
        k_line = [ln for ln in r.stderr.split("\n") if ln.startswith("stats K ")][-1].split()
        K, nl = int(k_line[2]), int(k_line[4])
        kmax = int(max(P, int(g[f"keys_grid_{P}"].max()) + 1))
        assert K == nl == kmax
        seen_k_ne_p |= K != P
    assert seen_k_ne_p, "no merge with K != P on this stream"
