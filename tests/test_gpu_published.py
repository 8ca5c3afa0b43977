"""The one output number the reference publishes for a configured workload: local optimality
0.25 at 4D for MR-Dim, MR-Grid and MR-Angle (/root/reference/python/graph_paper_figures.py:38-42,
Figure 7's 4D point; Flink parallelism 2 -> P = 4 partitions, FlinkSkyline.java:76).

On the reference's anti-correlated formula (python/unified_producer.py:89-123) at D >= 4 the
global skyline is exactly the all-zero tuples, and every all-zero tuple lands in
key 0 under all three partitioners; key 0's local skyline is those tuples (survivors_0 = |L_0|)
and every other key's local skyline is dominated by them (survivors_k = 0), so optimality =
(1/P) sum_k survivors_k / |L_k| (FlinkSkyline.java:593-608) = 1/4, printed by Java's
String.format(Locale.US, "%.4f") as "0.2500".  Asserted on the HIP path's sky_global_stats, and
through the C replay of the Java operators' call sequence (tests/operator_replay.c)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, golden_streams, load_golden

pytestmark = pytest.mark.gpu

BIN = os.path.join(REPO, "flink-skyline-qos_amd", "build", "operator_replay")
ALGO = {"mr-dim": 0, "mr-grid": 1, "mr-angle": 2}
N = 1_000_000
P = 4


def java_format_4f(x):
    import decimal
    d = decimal.Decimal(repr(float(x)))
    return str(d.quantize(decimal.Decimal("0.0001"), rounding=decimal.ROUND_HALF_UP))


def optimality(ls, sv, P_):
    """GlobalSkylineAggregator (FlinkSkyline.java:593-608): mean over the P partitions of
    survivors_k / |L_k| (a partition with an empty local skyline adds 0)."""
    return sum(sv[k] / ls[k] for k in range(P_) if ls[k] > 0) / P_


@pytest.fixture(scope="module")
def stream_4d(oracle):
    vals = oracle.synth(2, 4, N, seed=2026)          # the reference anti-correlated formula, 4D
    ids = np.arange(N, dtype=np.int64)
    return ids, vals


@pytest.mark.parametrize("algo", ["mr-dim", "mr-grid", "mr-angle"])
def test_published_4d_optimality_on_the_hip_path(algo, stream_4d, gpu_engine_factory, oracle):
    ids, vals = stream_4d
    eng = gpu_engine_factory(4, P, algo)
    gids, org = eng.query(vals, ids)
    ls, sv = eng.stats()
    eng.close()
    zeros = np.nonzero(~vals.any(axis=1))[0]
    assert len(zeros) > 0
    np.testing.assert_array_equal(gids, ids[zeros])          # the skyline = the all-zero tuples
    assert (org == 0).all()                                  # all of them in key 0
    _, _, els, esv, _ = oracle.query_sfs_chunked(algo[3:], vals, P)
    np.testing.assert_array_equal(ls, els)
    np.testing.assert_array_equal(sv, esv)
    assert sv[0] == ls[0] == len(zeros) and (sv[1:] == 0).all()
    assert java_format_4f(optimality(ls, sv, P)) == "0.2500"


def test_published_4d_optimality_on_the_golden_reference_stream(gpu_engine_factory):
    """The golden 4D stream is the reference generator's own output (tests/golden/make_golden.py)."""
    path = [p for p in golden_streams() if "anti_correlated_4d" in p][0]
    g = load_golden(path)
    for algo in ALGO:
        eng = gpu_engine_factory(4, P, algo)
        eng.query(g["values"], g["ids"].astype(np.int64))
        ls, sv = eng.stats()
        eng.close()
        assert java_format_4f(optimality(ls, sv, P)) == "0.2500", algo


@pytest.mark.parametrize("algo", ["mr-dim", "mr-grid", "mr-angle"])
def test_published_4d_optimality_through_the_java_sequence(algo, stream_4d, tmp_path):
    """The Java operators' calls (per-key 5000-tuple buffers, drainFull groups of 8,
    sky_part_snapshot_reps messages, sky_global_merge_reps, sky_global_stats) print the JSON
    line of FlinkSkyline.java:631-648 with "optimality": 0.2500."""
    assert os.path.exists(BIN), "build/operator_replay missing: run __graft_entry__.build()"
    ids, vals = stream_4d
    csv = tmp_path / "stream.csv"
    with open(csv, "w") as f:                                # the producers' payload, :174
        f.write("".join(f"{i},{a},{b},{c},{d}\n" for i, (a, b, c, d) in zip(ids.tolist(), vals.astype(np.int64).tolist())))
    r = subprocess.run([BIN, str(csv), "4", str(P // 2), str(ALGO[algo]), "1000.0", "-1", "8", "0"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    line = r.stdout.strip().split("\n")[0]
    assert line.split('"optimality": ')[1].split(",")[0] == "0.2500", line
    js = json.loads(line)
    assert js["record_count"] == N and js["skyline_size"] == int((~vals.any(axis=1)).sum())
