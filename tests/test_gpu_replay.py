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
