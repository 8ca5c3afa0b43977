"""CPU tests of the CSV-ingest oracle (oracle/csv_oracle.c), the checker of the device
decoder (k_csv.hip).  It restates ServiceTuple.fromString (ServiceTuple.java:89-104),
the nonNull filter (FlinkSkyline.java:103) and Long.parseLong(id) (:276).

Pins: (1) values against Python's float() — an independent correctly rounded
decimal conversion (David Gay) — on every string both grammars accept; (2) the
JDK's documented Double.parseDouble grammar through a hand table; (3) the
reference producer's payload format (unified_producer.py:174) over the golden
streams, which must decode back to the generator's values.  The JVM itself cannot
run here (no JDK): parity against the JVM binary is unpinned.
"""
import math
import random
import struct

import numpy as np
import pytest

from conftest import golden_streams, load_golden


def bits(x):
    return struct.unpack("<q", struct.pack("<d", x))[0]


# (string, expected) per the JDK 11 Double.parseDouble / FloatingDecimal grammar; None = NumberFormatException
JAVA_TABLE = [
    ("0", 0.0), ("-0", -0.0), ("+7", 7.0), ("12.5", 12.5), (" 12 ", 12.0), ("\t3\r", 3.0),
    ("1.5f", 1.5), ("1.5F", 1.5), ("2d", 2.0), ("2D", 2.0), ("1e3", 1000.0), ("1E+3", 1000.0),
    ("1e-3", 0.001), ("1.e2", 100.0), (".5", 0.5), ("+.5", 0.5), ("-.5e1", -5.0), ("0005", 5.0),
    ("NaN", math.nan), ("-NaN", math.nan), ("+NaN", math.nan), ("Infinity", math.inf),
    ("-Infinity", -math.inf), ("+Infinity", math.inf), ("1e400", math.inf), ("-1e400", -math.inf),
    ("1e-400", 0.0), ("4.9e-324", 5e-324), ("0x1p3", 8.0), ("0X1P3", 8.0), ("0x1.8p1", 3.0),
    ("-0x.8p1", -1.0), ("0x10p-4", 1.0), ("0x1p3d", 8.0), ("0x1.fffffffffffff8p0", 2.0),
    ("0x1.fffffffffffff7p0", float.fromhex("0x1.fffffffffffffp0")), ("0x1p-1075", 0.0),
    ("0x1.0000000000001p-1075", 5e-324), ("0x1p1024", math.inf),
    ("", None), ("   ", None), (".", None), ("e5", None), ("1e", None), ("1e+", None), ("1ee5", None),
    ("--1", None), ("+-1", None), ("1.2.3", None), ("1,5", None), ("inf", None), ("nan", None),
    ("infinity", None), ("NaNx", None), ("Infinit", None), ("1_000", None), ("0x", None),
    ("0x1.8", None), ("0xp1", None), ("0x1p", None), ("1.5ff", None), ("1.5 f", None), ("f", None),
    ("1d5", None), ("0b101", None), ("１", None),
]


@pytest.mark.parametrize("s,exp", JAVA_TABLE)
def test_java_parse_double_table(oracle, s, exp):
    got = oracle.java_parse_double(s)
    if exp is None:
        assert got is None, s
    elif math.isnan(exp):
        assert got is not None and math.isnan(got)
    else:
        assert got is not None and bits(got) == bits(exp), (s, got, exp)


def _rand_decimal(rng):
    kind = rng.randrange(6)
    sign = rng.choice(["", "-", "+"])
    if kind == 0:       # producer-style integers
        return sign + str(rng.randrange(0, 100000))
    if kind == 1:       # short decimals
        return sign + "%d.%0*d" % (rng.randrange(0, 10000), rng.randrange(1, 6), rng.randrange(0, 10 ** 5) % 10 ** 5)
    nd = rng.randrange(1, 40)
    digits = "".join(rng.choice("0123456789") for _ in range(nd))
    pt = rng.randrange(0, nd + 1)
    mant = digits[:pt] + "." + digits[pt:] if rng.random() < 0.7 else digits
    if mant in (".",):
        mant = "0"
    exp = "" if kind == 2 else "e%d" % rng.randrange(-345, 330)
    return sign + mant + exp


def test_decimal_values_match_python_float(oracle):
    """Correct rounding: the oracle equals Python's float() bit for bit on 40k strings,
    including 17-40 digit significands and the subnormal / overflow ranges."""
    rng = random.Random(11)
    n = 0
    for _ in range(40000):
        s = _rand_decimal(rng)
        try:
            exp = float(s)
        except ValueError:
            continue
        got = oracle.java_parse_double(s)
        assert got is not None and bits(got) == bits(exp), (s, got, exp)
        n += 1
    assert n > 39000


def test_halfway_cases(oracle):
    """Exact halfway points (ties to even) and their neighbours, built with exact decimal
    expansions of binary fractions: the hard cases of correct rounding."""
    from fractions import Fraction
    rng = random.Random(5)
    for _ in range(300):
        e = rng.randrange(-1074, 970)
        m = rng.randrange(1 << 52, 1 << 53)
        for h in (Fraction(2 * m + 1) * Fraction(2) ** (e - 1), Fraction(2 * m + 1) * Fraction(2) ** (e - 1)
                  + Fraction(1, 10 ** 800), Fraction(2 * m + 1) * Fraction(2) ** (e - 1) - Fraction(1, 10 ** 800)):
            # exact decimal string of h (finite: denominator is a power of two)
            num, den = h.numerator, h.denominator
            k = den.bit_length() - 1 if den & (den - 1) == 0 else None
            if k is None:
                continue
            s = str(num * 5 ** k)
            if k:
                s = s.rjust(k + 1, "0")
                s = s[:-k] + "." + s[-k:]
            exp = float(s)
            got = oracle.java_parse_double(s)
            assert bits(got) == bits(exp), s[:40]


def test_parse_long_and_split_semantics(oracle):
    text = (b"5,1,2\n"                # ok
            b"6,1,2,\n"               # trailing empty field dropped by split -> ok
            b"7,1,2,,,\n"             # several trailing empties -> ok
            b"8,1,,2\n"               # interior empty -> parseDouble("") -> null
            b",1,2\n"                 # empty id -> Long.parseLong("") fails
            b" 9,1,2\n"               # Long.parseLong does not trim
            b"10,1\n"                 # well-formed, one value: wrong arity for D = 2
            b"11,1,2,3\n"             # three values
            b"12\n"                   # p.length < 2 -> null
            b"\n"                     # empty record -> null
            b",,,\n"                  # split gives [] -> null
            b"9223372036854775807,0,0\n"
            b"9223372036854775808,0,0\n"   # long overflow
            b"-9223372036854775808,0,0\n"
            b"+13, 1 ,2\r\n"          # trim on values, CR trimmed
            b"14,1,x\n"
            b"15,1e400,-0")           # unterminated tail is a record
    st, ids, vals = oracle.parse_csv(text, 2)
    assert st.tolist() == [0, 0, 0, 1, 2, 2, 3, 3, 1, 1, 1, 0, 2, 0, 0, 1, 0]
    ok = st == 0
    assert ids[ok].tolist() == [5, 6, 7, 9223372036854775807, -9223372036854775808, 13, 15]
    assert vals[ok][-1][0] == math.inf and bits(vals[ok][-1][1]) == bits(-0.0)


@pytest.mark.parametrize("path", golden_streams()[:6], ids=lambda p: p.split("stream_")[-1][:-4])
def test_reference_payload_roundtrip(oracle, path):
    """The reference producer's payload format (unified_producer.py:174: f"{id}," +
    ",".join(map(str, data))) over a golden stream decodes back to its values and ids."""
    g = load_golden(path)
    vals, ids = g["values"], g["ids"]
    lines = [f"{i}," + ",".join(map(str, map(int, row))) for i, row in zip(ids.tolist(), vals.tolist())]
    text = ("\n".join(lines) + "\n").encode()
    st, pid, pv = oracle.parse_csv(text, vals.shape[1])
    assert (st == 0).all() and len(st) == len(vals)
    assert (pid == ids).all() and np.array_equal(pv, vals)
