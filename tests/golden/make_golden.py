"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the authoring container (it reads /root/reference, which does not
exist on the GPU box).  Nothing under tests/ imports this script.

1. Input streams come from the reference's OWN generator functions
   (/root/reference/python/unified_producer.py:50-123), imported with stub
   `kafka` / `faker` modules (neither is installed; the stubs mirror Faker's
   `random_int = randrange(min, max+1)` and its `random` Random instance).  The
   generator is unseeded in the reference; here both RNG streams are seeded.
2. Expected operator outputs come from the C restatement in oracle/ (the Java
   operators cannot run here: no JDK — SURVEY.md §8c), cross-checked in this
   script against brute force.
3. atan2 vectors come from node's Math.atan2 (V8's port of FreeBSD msun
   e_atan2.c, itself fdlibm) — an independent fdlibm implementation that pins
   the fdlibm restatement used by MR-Angle.

Usage:  python tests/golden/make_golden.py
"""
import ctypes
import json
import os
import random
import struct
import subprocess
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True


def load_reference_generator():
    stub_dir = tempfile.mkdtemp(prefix="skyline_stubs_")
    os.makedirs(os.path.join(stub_dir, "kafka"))
    os.makedirs(os.path.join(stub_dir, "faker"))
    with open(os.path.join(stub_dir, "kafka", "__init__.py"), "w") as f:
        f.write("class KafkaProducer:\n    def __init__(self, *a, **k):\n        raise RuntimeError('stub')\n")
    with open(os.path.join(stub_dir, "faker", "__init__.py"), "w") as f:
        f.write(
            "import random as _r\n"
            "class Faker:\n"
            "    def __init__(self, seed=0):\n"
            "        self.random = _r.Random(seed)\n"
            "    def random_int(self, min=0, max=9999, step=1):\n"
            "        return self.random.randrange(min, max + 1, step)\n")
    sys.path.insert(0, stub_dir)
    sys.path.insert(0, "/root/reference/python")
    import unified_producer  # noqa: E402  (reference module, generator functions only)
    import faker  # noqa: E402  (our stub)
    return unified_producer, faker


def ref_stream(up, faker_mod, dist, D, n, seed, dmin=0, dmax=1000):
    random.seed(seed)                       # module-level random used by uniform()/correlated
    fk = faker_mod.Faker(seed + 7919)       # Faker's own Random (random_int, .random)
    gen = {"uniform": up.generate_uniform_data,
           "correlated": up.generate_correlated_data,
           "anti_correlated": up.generate_anti_correlated_data}[dist]
    rows = [gen(fk, D, dmin, dmax) for _ in range(n)]
    return np.asarray(rows, dtype=np.float64).reshape(n, D)


def load_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    c_dp = ctypes.POINTER(ctypes.c_double)
    c_i64p = ctypes.POINTER(ctypes.c_int64)
    c_i32p = ctypes.POINTER(ctypes.c_int32)
    c_u8p = ctypes.POINTER(ctypes.c_uint8)
    L.orc_query_bnl.restype = ctypes.c_int64
    L.orc_query_bnl.argtypes = [ctypes.c_int, c_dp, c_i64p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_double, ctypes.c_int, ctypes.c_int, c_i64p, c_i32p,
                                ctypes.c_int64, c_i64p, c_i64p]
    L.orc_keys.argtypes = [ctypes.c_int, c_dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                           ctypes.c_double, c_i32p]
    L.orc_skyline_brute.argtypes = [c_dp, ctypes.c_int64, ctypes.c_int, c_u8p]
    return L


def ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


ALGOS = {"dim": 0, "grid": 1, "angle": 2}


def oracle_query(L, algo, vals, ids, P, domain, sem=0):
    n, D = vals.shape
    K = P if not (algo == "grid" and sem == 1) else max(P, 1 << D)
    out_ids = np.zeros(max(n, 1), np.int64)
    out_org = np.zeros(max(n, 1), np.int32)
    lsz = np.zeros(K, np.int64)
    surv = np.zeros(K, np.int64)
    g = L.orc_query_bnl(ALGOS[algo], ptr(vals, ctypes.c_double), ptr(ids, ctypes.c_int64), n, D, P,
                        domain, 5000, sem, ptr(out_ids, ctypes.c_int64), ptr(out_org, ctypes.c_int32),
                        n, ptr(lsz, ctypes.c_int64), ptr(surv, ctypes.c_int64))
    assert g >= 0
    return out_ids[:g].copy(), out_org[:g].copy(), lsz, surv


def main():
    up, fk = load_reference_generator()
    L = load_oracle()
    summary = {"streams": [], "generator": "reference unified_producer.py (stub kafka/faker, seeded)"}
    n_small = 3000
    for dist in ("uniform", "correlated", "anti_correlated"):
        for D in (2, 3, 4, 6, 8):
            seed = 1234 + D + {"uniform": 0, "correlated": 100, "anti_correlated": 200}[dist]
            vals = np.ascontiguousarray(ref_stream(up, fk, dist, D, n_small, seed))
            ids = np.arange(n_small, dtype=np.int64)
            rec = {"values": vals.astype(np.int16) if np.all(vals == np.round(vals)) and vals.max() < 32767 else vals,
                   "ids": ids}
            # brute-force definition check of the BNL restatement (global, 'complete' grid == all data)
            brute = np.zeros(n_small, np.uint8)
            L.orc_skyline_brute(ptr(vals, ctypes.c_double), n_small, D, ptr(brute, ctypes.c_uint8))
            for algo in ("dim", "grid", "angle"):
                for P in (4, 8, 16):
                    keys = np.zeros(n_small, np.int32)
                    L.orc_keys(ALGOS[algo], ptr(vals, ctypes.c_double), n_small, D, P, 1000.0,
                               ptr(keys, ctypes.c_int32))
                    gids, gorg, lsz, surv = oracle_query(L, algo, vals, ids, P, 1000.0)
                    if algo != "grid" or (1 << D) <= P:
                        assert set(gids.tolist()) == set(np.nonzero(brute)[0].tolist()), (dist, D, algo, P)
                    rec[f"keys_{algo}_{P}"] = keys.astype(np.int16)
                    rec[f"gsky_{algo}_{P}"] = np.sort(gids).astype(np.int32)
                    rec[f"lsz_{algo}_{P}"] = lsz
                    rec[f"surv_{algo}_{P}"] = surv
            fn = f"stream_{dist}_{D}d.npz"
            np.savez_compressed(os.path.join(HERE, fn), **rec)
            summary["streams"].append({"file": fn, "dist": dist, "D": D, "n": n_small, "seed": seed,
                                       "skyline_size_brute": int(brute.sum())})
            print(fn, "skyline", int(brute.sum()))

    # PDF p.15 §5.1 generator KAT config (2D, domain 0-10000): correlated skyline is all [0,0]
    # duplicates; committed as a 20k-tuple stream (the PDF's 200k is unseeded, statistical only).
    vals = np.ascontiguousarray(ref_stream(up, fk, "correlated", 2, 20000, 4242, 0, 10000))
    np.savez_compressed(os.path.join(HERE, "kat_pdf15_correlated_2d.npz"), values=vals.astype(np.int16))
    brute = np.zeros(len(vals), np.uint8)
    L.orc_skyline_brute(ptr(vals, ctypes.c_double), len(vals), 2, ptr(brute, ctypes.c_uint8))
    sky = vals[brute.astype(bool)]
    summary["kat_pdf15_correlated_2d"] = {"n": 20000, "skyline_size": int(brute.sum()),
                                         "all_zero": bool(np.all(sky == 0))}

    # atan2 vectors from V8's fdlibm port (node)
    r = random.Random(99)
    pairs = []
    for _ in range(6000):
        pairs.append((float(r.randint(0, 1000)), float(r.randint(0, 1000))))
    for _ in range(3000):
        pairs.append((float(r.randint(0, 10000)), float(r.randint(-10000, 10000))))
    for _ in range(3000):
        pairs.append((r.uniform(0, 1e3) * 10 ** r.randint(-5, 5), r.uniform(-1e3, 1e3) * 10 ** r.randint(-5, 5)))
    pairs += [(0.0, 0.0), (-0.0, 0.0), (0.0, -0.0), (1.0, 1.0), (1e300, 1.0), (1.0, 1e300),
              (float("inf"), 1.0), (1.0, float("-inf")), (float("inf"), float("inf"))]
    inp = "\n".join(f"{struct.pack('<d', y).hex()} {struct.pack('<d', x).hex()}" for y, x in pairs)
    js = (r"const l=require('fs').readFileSync(0,'utf8').trim().split('\n');const o=[];"
          r"for(const s of l){const [a,b]=s.split(' ');const y=Buffer.from(a,'hex').readDoubleLE(0),"
          r"x=Buffer.from(b,'hex').readDoubleLE(0);const r=Buffer.alloc(8);r.writeDoubleLE(Math.atan2(y,x));"
          r"o.push(r.toString('hex'));}console.log(o.join('\n'));")
    res = subprocess.run(["node", "-e", js], input=inp, capture_output=True, text=True, check=True).stdout.split()
    yx = np.array(pairs, np.float64)
    out = np.array([struct.unpack("<d", bytes.fromhex(h))[0] for h in res], np.float64)
    node_ver = subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip()
    np.savez_compressed(os.path.join(HERE, "atan2_v8_fdlibm.npz"), yx=yx, atan2=out)
    summary["atan2"] = {"n": len(pairs), "source": f"node {node_ver} Math.atan2 (V8 ieee754::atan2)"}
    with open(os.path.join(HERE, "SUMMARY.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary["kat_pdf15_correlated_2d"]))


if __name__ == "__main__":
    main()
