"""GPU parity of the device CSV decoder (k_csv.hip, sky_parse_csv[_dev]) against the
oracle restatement of ServiceTuple.fromString + filter(nonNull) + Long.parseLong
(oracle/csv_oracle.c; ServiceTuple.java:89-104, FlinkSkyline.java:103,276).
Bar: per-record status codes identical, accepted ids and value bits identical."""
import math
import random

import numpy as np
import pytest
import torch

from conftest import golden_streams, load_golden

pytestmark = pytest.mark.gpu


def _field(rng):
    k = rng.randrange(20)
    if k < 8:
        return str(rng.randrange(0, 10001))
    if k < 10:
        return "%d.%d" % (rng.randrange(0, 1000), rng.randrange(0, 1000))
    if k == 10:
        nd = rng.randrange(15, 45)
        d = "".join(rng.choice("0123456789") for _ in range(nd))
        p = rng.randrange(0, nd)
        return d[:p] + "." + d[p:] + "e%d" % rng.randrange(-340, 320)
    if k == 11:
        return rng.choice(["NaN", "-Infinity", "Infinity", "1e400", "-0", "4.9e-324", "2.2250738585072011e-308",
                           "0x1.8p1", "-0x.8p-1074", "0x1.fffffffffffff8p1023", "1.5f", " 7 ", "\t8\r", "+.5",
                           "1.e2", "9007199254740993", "123456789012345678901234567890"])
    if k == 12:
        return rng.choice(["", "x", "1e", ".", "--1", "inf", "1.2.3", "0x1.8", "1 2", "0x", "NaNx", "1ee5"])
    if k == 13:
        return "%de%d" % (rng.randrange(1, 10 ** 6), rng.randrange(-30, 30))
    return str(rng.randrange(-1000, 1000))


def _record(rng, D):
    k = rng.randrange(30)
    if k == 0:
        return ""
    n = D if k > 3 else rng.choice([0, 1, D - 1, D + 1])
    idk = rng.randrange(40)
    if idk == 0:
        idf = rng.choice(["", " 5", "x", "9223372036854775808", "-9223372036854775808", "+3", "-"])
    else:
        idf = str(rng.randrange(0, 10 ** 12))
    fields = [idf] + [_field(rng) for _ in range(max(n, 0))]
    s = ",".join(fields)
    if rng.randrange(15) == 0:
        s += "," * rng.randrange(1, 3)
    if rng.randrange(20) == 0:
        s += "\r"
    return s


def _check(eng, oracle, text, D, offset=0):
    st_o, ids_o, vals_o = oracle.parse_csv(text, D)
    buf = torch.zeros(len(text) + offset + 16, dtype=torch.uint8, device="cuda")
    if len(text):
        buf[offset:offset + len(text)] = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    dtext = buf[offset:]
    R = len(st_o)
    ids = torch.empty(max(R, 1), dtype=torch.int64, device="cuda")
    vals = torch.empty((max(R, 1), D), dtype=torch.float64, device="cuda")
    stat = torch.empty(max(R, 1), dtype=torch.uint8, device="cuda")
    n, cnt = eng.parse_csv_dev(dtext, len(text), ids, vals, R, stat)
    assert cnt[0] == R
    st = stat[:R].cpu().numpy()
    np.testing.assert_array_equal(st, st_o)
    ok = st_o == 0
    assert n == int(ok.sum())
    for c in (1, 2, 3):
        assert cnt[c] == int((st_o == c).sum())
    gi = ids[:n].cpu().numpy()
    gv = vals[:n].cpu().numpy()
    np.testing.assert_array_equal(gi, ids_o[ok])
    # bit-exact values (NaN: the canonical quiet NaN on both sides)
    np.testing.assert_array_equal(gv.view(np.int64), vals_o[ok].view(np.int64))
    return n


@pytest.mark.parametrize("route", ["chunks", "groups"])
@pytest.mark.parametrize("D", [1, 2, 4, 8])
def test_csv_fuzz_matches_oracle(gpu_engine_factory, oracle, monkeypatch, D, route):
    """Both parse routes: the group route (the default, SKY_CSV_CHUNKS=0) and byte chunks (=1)."""
    monkeypatch.setenv("SKY_CSV_CHUNKS", "1" if route == "chunks" else "0")
    rng = random.Random(100 + D)
    text = ("\n".join(_record(rng, D) for _ in range(20000))).encode()
    eng = gpu_engine_factory(D, 8)
    n = _check(eng, oracle, text, D)
    assert n > 5000
    eng.close()


def _plain_record(rng, D, i, rate):
    """The producer's shape (ids and values as plain digit strings, unified_producer.py:174),
    with a rare perturbation that the lane-per-record fast path must hand to the general path:
    9-digit fields, decimals, signs, empty / missing / extra fields, '\\r', a trailing comma."""
    vals = [str(rng.randrange(0, 10 ** rng.choice([1, 4, 8]))) for _ in range(D)]
    rec = [str(i % 10 ** 8)] + vals
    if rng.random() < rate:
        k = rng.randrange(10)
        c = rng.randrange(D + 1)
        if k == 0:
            rec[c] = "123456789"                    # 9 digits: the 64-bit SWAR path
        elif k == 1:
            rec[c] = "99999999"                     # 8 digits: still the fast path
        elif k == 2:
            rec[c] = "1.5"
        elif k == 3:
            rec[c] = "-7" if c else "+7"
        elif k == 4:
            rec[c] = ""
        elif k == 5:
            rec.pop()
        elif k == 6:
            rec.append("3")
        elif k == 7:
            rec[-1] += "\r"
        elif k == 8:
            rec[-1] += ","
        else:
            rec[c] = "00000042"
    return ",".join(rec)


@pytest.mark.parametrize("route", ["chunks", "groups"])
@pytest.mark.parametrize("D,rate,tail", [(1, 0.001, True), (2, 0.0005, False), (3, 0.002, True), (4, 0.0, False),
                                         (7, 0.001, False), (8, 0.0005, True), (8, 0.0, False), (9, 0.001, True)])
def test_csv_producer_shape_mixed(gpu_engine_factory, oracle, monkeypatch, D, rate, tail, route):
    """Workgroups of plain records take the lane-per-record fast path (D <= 8), a workgroup with
    one perturbed record takes the general path on the same staged text; both against the oracle,
    with and without a final newline."""
    monkeypatch.setenv("SKY_CSV_CHUNKS", "1" if route == "chunks" else "0")
    rng = random.Random(7 * D + int(rate * 10000))
    text = "\n".join(_plain_record(rng, D, i, rate) for i in range(60000))
    text = (text + ("" if tail else "\n")).encode()
    eng = gpu_engine_factory(D, 8)
    n = _check(eng, oracle, text, D)
    assert n >= 60000 * (1 - 2 * rate) - 50
    eng.close()


@pytest.mark.parametrize("route", ["chunks", "groups"])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 256, 257, 20000, 65537])
def test_csv_block_aligned_records(gpu_engine_factory, oracle, monkeypatch, route, n):
    """16-byte records: every '\n' is the last byte of a 16-byte unit, so group ends fall exactly on
    1 KB / 4 KB count-block boundaries (k_csv_group_pos picks the quarter by its count), and the
    record counts straddle the group size."""
    monkeypatch.setenv("SKY_CSV_CHUNKS", "1" if route == "chunks" else "0")
    text = "".join("%08d,%06d\n" % (i, (i * 7919) % 1000000) for i in range(n)).encode()
    assert len(text) == 16 * n
    eng = gpu_engine_factory(1, 8)
    assert _check(eng, oracle, text, 1) == n
    eng.close()


@pytest.mark.parametrize("route", ["chunks", "groups"])
@pytest.mark.parametrize("offset", [1, 2, 3, 5])
def test_csv_unaligned_buffer(gpu_engine_factory, oracle, monkeypatch, offset, route):
    monkeypatch.setenv("SKY_CSV_CHUNKS", "1" if route == "chunks" else "0")
    rng = random.Random(offset)
    text = ("\n".join(_record(rng, 3) for _ in range(3000)) + "\n").encode()
    eng = gpu_engine_factory(3, 8)
    _check(eng, oracle, text, 3, offset)
    eng.close()


def test_csv_long_records_and_numbers(gpu_engine_factory, oracle):
    """Records far longer than the LDS staging window (global-memory path) and
    significands of hundreds of digits (exact big-integer path, sticky digits)."""
    rng = random.Random(3)
    lines = []
    for i in range(600):
        vals = []
        for _ in range(2):
            nd = rng.choice([20, 300, 790, 801, 1200])
            d = str(rng.randrange(1, 10)) + "".join(rng.choice("0123456789") for _ in range(nd - 1))
            p = rng.randrange(0, nd)
            vals.append(d[:p] + "." + d[p:] + "e%d" % rng.randrange(-1200, 40))
        lines.append(f"{i}," + ",".join(vals))
    text = ("\n".join(lines) + "\n").encode()
    eng = gpu_engine_factory(2, 8)
    assert _check(eng, oracle, text, 2) == 600
    eng.close()


@pytest.mark.parametrize("chunks", ["0", "1"])
def test_csv_exact_reparse_path(chunks):
    """More exact conversions than the queue holds: every record is re-parsed on the exact
    path (groups of 256 records, boundaries found by the fallback workgroups).  The queue
    size is read once per process, so this runs in a child process with a 4-entry queue.
    chunks=1: the byte-chunk route, which never sizes the group array itself -- the exact
    re-parse must size it (round 3 faulted here: an illegal address in the re-parse)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = r"""
import random, sys
sys.path.insert(0, %r); sys.path.insert(0, %r)
import skyline
from conftest import Oracle
from test_gpu_csv import _check
rng = random.Random(5)
lines = []
for i in range(3000):
    vals = []
    for _ in range(2):
        nd = rng.choice([3, 25, 40])
        d = str(rng.randrange(1, 10)) + "".join(rng.choice("0123456789") for _ in range(nd - 1))
        vals.append(d[:1] + "." + d[1:] + "e%%d" %% rng.randrange(-30, 30))
    lines.append(("%%d," %% i) + ",".join(vals) if i %% 97 else "bad,1,2")
text = ("\n".join(lines) + "\n").encode()
eng = skyline.SkylineEngine(2, 8, "mr-angle", 1000.0, 0)
_check(eng, Oracle(), text, 2)
_check(eng, Oracle(), text[:-1], 2)          # tail record without a newline
print("ok")
""" % (os.path.join(os.path.dirname(here), "flink-skyline-qos_amd"), here)
    env = dict(os.environ, SKY_CSV_SLOW_CAP="4", SKY_CSV_CHUNKS=chunks)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_csv_chunks_listed_spans(gpu_engine_factory, oracle, monkeypatch):
    """Byte-chunk parse (SKY_CSV_CHUNKS=1; the default is the group route): chunks sized from the text's average record, each
    workgroup finding its own records; chunks that do not fit go to the fallback as spans: > 256
    record starts (tiny records), a record running past the staged tail (mid-text and the text's
    last, with and without a newline), > 2048 fields.  Same results as the group-pass parse."""
    rng = random.Random(21)
    D = 3
    head = [f"{10 ** 6 + i}," + ",".join(str(rng.randrange(10 ** 5, 10 ** 6)) for _ in range(3)) for i in range(8000)]
    tiny = ["7"] * 2000 + ["1,2,3,4"] * 1500
    # > 10 KB (past any chunk's staged tail), every field < 8 KB (the oracle's field limit)
    longrec = ["5," + ",".join(str(rng.randrange(10 ** 9)) for _ in range(3)) + "," + "1" * 7000 + ",2" + "0" * 4000]
    wide = ["9," + ",".join(["1"] * 3000)] * 3
    tail = [f"{i},{i % 7}00000,{i % 5}00000,{i % 3}00000" for i in range(3000)]
    for body in (head + tiny + longrec + head + wide + tail, head + longrec, head + wide):
        for end in ("", "\n"):
            text = ("\n".join(body) + end).encode()
            assert len(text) / len(body) >= 512 / (0.8 * 256)       # chunk mode is chosen
            eng = gpu_engine_factory(D, 8)
            monkeypatch.setenv("SKY_CSV_CHUNKS", "1")
            n1 = _check(eng, oracle, text, D)
            monkeypatch.setenv("SKY_CSV_CHUNKS", "0")
            n0 = _check(eng, oracle, text, D)
            monkeypatch.delenv("SKY_CSV_CHUNKS")
            assert n1 == n0
            eng.close()


def test_csv_halfway_values(gpu_engine_factory, oracle):
    from fractions import Fraction
    rng = random.Random(9)
    lines = []
    for i in range(2000):
        e = rng.randrange(-1074, 970)
        m = rng.randrange(1 << 52, 1 << 53)
        h = Fraction(2 * m + 1) * Fraction(2) ** (e - 1)
        den = h.denominator
        k = den.bit_length() - 1
        s = str(h.numerator * 5 ** k)
        if k:
            s = s.rjust(k + 1, "0")
            s = s[:-k] + "." + s[-k:]
        tweak = rng.choice(["", "1", "0001"])
        lines.append(f"{i},{s}{tweak if '.' in s else ''}")
    text = ("\n".join(lines)).encode()
    eng = gpu_engine_factory(1, 4)
    assert _check(eng, oracle, text, 1) == 2000
    eng.close()


def test_csv_edge_buffers(gpu_engine_factory, oracle):
    eng = gpu_engine_factory(2, 8)
    for text in [b"", b"\n", b"\n\n\n", b"1,2,3", b"1,2,3\n", b"1,2", b"x" * 50000, b"1,2,3\n" * 5000 + b"4,5"]:
        _check(eng, oracle, text, 2)
    # host-buffer entry point and capacity errors
    ids, vals, cnt = eng.parse_csv(b"1,2,3\n4,5,6\nbad\n")
    assert ids.tolist() == [1, 4] and vals.tolist() == [[2, 3], [5, 6]] and cnt.tolist() == [3, 1, 0, 0]
    from skyline._abi import SkylineError
    d = torch.frombuffer(bytearray(b"1,2,3\n4,5,6\n"), dtype=torch.uint8).cuda()
    o_i = torch.empty(1, dtype=torch.int64, device="cuda")
    o_v = torch.empty((1, 2), dtype=torch.float64, device="cuda")
    with pytest.raises(SkylineError) as ei:
        eng.parse_csv_dev(d, 12, o_i, o_v, 1)
    assert ei.value.code == -3
    eng.close()


@pytest.mark.parametrize("path", golden_streams(), ids=lambda p: p.split("stream_")[-1][:-4])
def test_format_matches_reference_payload_and_roundtrips(gpu_engine_factory, path):
    """sky_format_csv_dev writes the producer's payload byte for byte
    (unified_producer.py:174), and the decoder reads it back exactly."""
    g = load_golden(path)
    vals, ids = g["values"], g["ids"].astype(np.int64)
    n, D = vals.shape
    eng = gpu_engine_factory(D, 8)
    dv = torch.from_numpy(vals).cuda()
    di = torch.from_numpy(ids).cuda()
    nb = eng.format_csv_dev(di, dv, n)
    text = torch.empty(nb, dtype=torch.uint8, device="cuda")
    assert eng.format_csv_dev(di, dv, n, text, nb) == nb
    ref = "".join(f"{i}," + ",".join(map(str, map(int, row))) + "\n" for i, row in zip(ids.tolist(), vals.tolist()))
    assert bytes(text.cpu().numpy()) == ref.encode()
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    ov = torch.empty((n, D), dtype=torch.float64, device="cuda")
    m, cnt = eng.parse_csv_dev(text, nb, oi, ov, n)
    assert m == n and cnt.tolist() == [n, 0, 0, 0]
    assert torch.equal(oi, di) and torch.equal(ov, dv)
    eng.close()


def test_csv_roundtrip_full_size(gpu_engine_factory):
    """Size-independent property at the benchmark's shape: 8D reference anti-correlated
    stream, 20M records, format -> parse is the identity; then the query on the decoded
    rows equals the query on the original rows."""
    n, D = 20_000_000, 8
    eng = gpu_engine_factory(D, 16)
    dv = torch.empty((n, D), dtype=torch.float64, device="cuda")
    di = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_dev("anti_correlated", n, dv, di, seed=77)
    nb = eng.format_csv_dev(di, dv, n)
    text = torch.empty(nb, dtype=torch.uint8, device="cuda")
    eng.format_csv_dev(di, dv, n, text, nb)
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    ov = torch.empty((n, D), dtype=torch.float64, device="cuda")
    m, cnt = eng.parse_csv_dev(text, nb, oi, ov, n)
    assert m == n and cnt.tolist() == [n, 0, 0, 0]
    assert torch.equal(oi, di) and torch.equal(ov, dv)
    a_i = torch.empty(n, dtype=torch.int64, device="cuda")
    a_o = torch.empty(n, dtype=torch.int32, device="cuda")
    b_i = torch.empty(n, dtype=torch.int64, device="cuda")
    b_o = torch.empty(n, dtype=torch.int32, device="cuda")
    ga = eng.query_dev(di, dv, a_i, a_o, n)
    gb = eng.query_dev(oi, ov, b_i, b_o, n)
    assert ga == gb and torch.equal(a_i[:ga], b_i[:gb])
    eng.close()
