#!/usr/bin/env python3
"""CPU simulation of k_mbr_pairs' pruning for different orders of the reps (no GPU).

Reps: the distinct (partition, vector) pairs of the local skylines of the std-anti 8D stream
(MR-Angle P=16), as the oracle computes them (~the set the pruned pass sees).  The reps are
cut into 64-row tiles (16-row sub-boxes) in the given order; for a sample of y reps we count
the x tiles whose min corner <= y (tiles reaching the row stage), the sub-boxes whose min corner
<= y (entries; 16 pair tests each) and the tiles passing the y tile's max-corner test.
Early exit (a y dominated by its own partition stops) is ignored: an upper bound, the same
for every order.  Usage: python tools/mbr_sim.py [n] [samples]"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
from conftest import Oracle  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
D, P = 8, 16
orc = Oracle()
t0 = time.time()
cache = f"/tmp/mbr_sim_reps_{n}.npz"
vals = orc.synth(3, D, n, seed=1234 + D)
if os.environ.get("SIM_ALL"):                # every tuple as a rep (no SFS: fast, ~the same geometry)
    keys = orc.keys("angle", vals, P)
    inl = np.ones(n, bool)
elif os.path.exists(cache):
    z = np.load(cache)
    keys, inl = z["keys"], z["inl"]
else:
    _, keys, _, _, inl = orc.query_sfs_chunked("angle", vals, P)
    np.savez(cache, keys=keys, inl=inl)
inl = inl.astype(bool)
kv = np.column_stack([keys[inl].astype(np.float64), vals[inl]])
kv = np.unique(kv, axis=0)
key = kv[:, 0].astype(np.int64)
X = kv[:, 1:].astype(np.int64)          # integral values: the u16 image orders the same way
m = len(X)
print(f"reps {m} (local-skyline tuples {inl.sum()}) in {time.time() - t0:.1f} s", flush=True)


def morton(q, bits):
    assert bits * D <= 63
    c = np.zeros(len(q), np.uint64)
    for b in range(bits - 1, -1, -1):
        for d in range(D):
            c = (c << np.uint64(1)) | ((q[:, d] >> b) & 1).astype(np.uint64)
    return c


def quant(bits):
    lo, hi = X.min(0), X.max(0)
    return ((X - lo) << bits) // (hi - lo + 1)


def hilbert(q, bits):
    """Skilling's transpose algorithm (AIP Conf. Proc. 707, 2004), vectorised."""
    x = q.copy().astype(np.int64)
    M = 1 << (bits - 1)
    Q = M
    while Q > 1:
        Pm = Q - 1
        for i in range(D):
            hi = (x[:, i] & Q) != 0
            x[hi, 0] ^= Pm
            t = (x[~hi, 0] ^ x[~hi, i]) & Pm
            x[~hi, 0] ^= t
            x[~hi, i] ^= t
        Q >>= 1
    for i in range(1, D):
        x[:, i] ^= x[:, i - 1]
    t = np.zeros(len(x), np.int64)
    Q = M
    while Q > 1:
        t[(x[:, D - 1] & Q) != 0] ^= Q - 1
        Q >>= 1
    for i in range(D):
        x[:, i] ^= t
    return morton(x, bits)          # interleave the transposed bits


def kd_order(idx, depth=0):
    """k-d leaves of <= 64 rows: split at the median of the widest dimension."""
    out = []
    stack = [idx]
    while stack:
        s = stack.pop()
        if len(s) <= 64:
            out.append(s)
            continue
        sub = X[s]
        d = int(np.argmax(sub.max(0) - sub.min(0)))
        h = ((len(s) + 127) // 128) * 64        # left part a multiple of 64 rows
        part = np.argpartition(sub[:, d], h - 1)
        stack.append(s[part[h:]])
        stack.append(s[part[:h]])
    return np.concatenate(out[::-1]) if out else idx


def order_by(name):
    if name.startswith("morton"):
        bits = int(name[6:])
        c = morton(quant(bits), bits)
        return np.lexsort((c, key))
    if name.startswith("hilbert"):
        bits = int(name[7:])
        c = hilbert(quant(bits), bits)
        return np.lexsort((c, key))
    if name == "kd":
        parts = [kd_order(np.nonzero(key == k)[0]) for k in np.unique(key)]
        return np.concatenate(parts)
    raise ValueError(name)


def stats(order, name, rng):
    Xo = X[order]
    nt = (m + 63) // 64
    pad = nt * 64 - m
    big = np.iinfo(np.int64).max
    Xp = np.concatenate([Xo, np.full((pad, D), big)]) if pad else Xo
    T = Xp.reshape(nt, 64, D)
    tmin = T.min(1)
    Xq = np.concatenate([Xo, np.full((pad, D), -1)]) if pad else Xo
    tmax = Xq.reshape(nt, 64, D).max(1)
    smin = T.reshape(nt, 4, 16, D).min(2).reshape(nt * 4, D)
    smin8 = T.reshape(nt, 8, 8, D).min(2).reshape(nt * 8, D)
    ys = rng.choice(m, S, replace=False)
    tiles = subs = cand = subs8 = 0
    ytiles = {}
    for j in ys:
        y = Xo[j]
        tiles += int((tmin <= y).all(1).sum())
        subs += int((smin <= y).all(1).sum())
        subs8 += int((smin8 <= y).all(1).sum())
        cand += int((tmin <= tmax[j // 64]).all(1).sum())
    # box extent: mean over tiles of the sum of per-dimension extents
    ext = float((tmax - tmin.clip(None, 10 ** 9)).sum(1).mean())
    print(f"{name:10s} tiles/y {tiles / S:8.1f}  cand tiles/ytile {cand / S:8.1f}  entries/y {subs / S:8.1f}  "
          f"pairs/y {16 * subs / S:9.1f}  8-row entries/y {subs8 / S:8.1f} pairs/y {8 * subs8 / S:9.1f}  "
          f"mean extent {ext:8.1f}", flush=True)
    # per y tile: x tiles some lane reaches (the tiles tested), groups of 64 tiles passing
    gmin = np.concatenate([tmin, np.full(((-nt) % 64, D), big)]).reshape(-1, 64, D).min(1)
    yts = rng.choice(nt, 60, replace=False)
    tt = gg = 0
    for yt in yts:
        Y = Xo[yt * 64:(yt + 1) * 64]
        reach = np.zeros(nt, bool)
        for y in Y:
            reach |= (tmin <= y).all(1)
        tt += int(reach.sum())
        gg += int((gmin <= tmax[yt]).all(1).sum())
    print(f"{'':10s} tested tiles/ytile {tt / len(yts):8.1f}  groups/ytile {gg / len(yts):6.1f} of {len(gmin)}",
          flush=True)


for name in sys.argv[3:] or ["morton4", "morton6", "hilbert4", "hilbert6", "kd"]:
    t0 = time.time()
    o = order_by(name)
    stats(o, name, np.random.default_rng(7))
    print(f"   ({time.time() - t0:.1f} s)", flush=True)
