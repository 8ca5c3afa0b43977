"""World-size-2 gloo test (CPU) of the multi-GPU exchange in skyline/dist.py.

The device phases are stood in for by the oracle (test infrastructure): each
rank reduces its shard to the distinct vectors of its local skylines with
multiplicities, the ranks exchange them with skyline.dist.allgather_varlen /
pack_export / unpack_union over gloo, and each rank finishes the union.  The
result must equal the single-process answer (the decomposition the GPU path
uses: SKY(u SKY(shard_r)) = SKY(u shard_r))."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_export(orc, vals, P):
    """distinct vectors of the local skylines of one shard, with partition + multiplicity"""
    sky, keys, _, _ = orc.query_sfs("angle", vals, P)
    inl = np.zeros(len(vals), bool)
    # local skylines (all partitions): run per partition via 'complete' trick -> use SFS per key
    for k in np.unique(keys):
        idx = np.nonzero(keys == k)[0]
        loc = orc.brute(vals[idx])
        inl[idx[loc]] = True
    rows = vals[inl]
    ks = keys[inl]
    uniq, inv, cnt = np.unique(np.column_stack([ks, rows]), axis=0, return_inverse=True, return_counts=True)
    return uniq[:, 1:].copy(), uniq[:, 0].astype(np.int32), cnt.astype(np.int64)


def _worker(rank, world, port, shards, P, D, ret):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "flink-skyline-qos_amd"))
    import torch.distributed as dist
    from conftest import Oracle
    from skyline.dist import allgather_varlen, pack_export, unpack_union
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    orc = Oracle()
    rows, keys, mult = _local_export(orc, shards[rank], P)
    packed = pack_export(torch.from_numpy(rows), torch.from_numpy(keys), torch.from_numpy(mult))
    gathered, counts = allgather_varlen(packed)
    urows, ukeys, umult = unpack_union(gathered, counts, D)
    assert sum(counts) == urows.shape[0]
    assert torch.equal(urows[sum(counts[:rank]):sum(counts[:rank]) + counts[rank]], torch.from_numpy(rows))
    # finish on the union: global skyline vectors and their total multiplicity
    u = urows.numpy()
    g = orc.brute(u)
    gset = {tuple(r) for r in u[g]}
    total = int(umult.numpy()[g].sum())
    ret[rank] = (sorted(gset), total)
    dist.destroy_process_group()


def test_two_rank_exchange_equals_single_process(oracle):
    n, D, P = 6000, 4, 8
    vals = oracle.synth(2, D, n, seed=3)
    shards = [vals[: n // 2], vals[n // 2:]]
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shards, P, D, ret)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    exp = oracle.brute(vals)
    exp_set = sorted({tuple(r) for r in vals[exp]})
    for r in range(2):
        got_set, total = ret[r]
        assert got_set == exp_set
        assert total == len(exp)          # every skyline tuple counted exactly once


def test_pack_unpack_roundtrip():
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "flink-skyline-qos_amd"))
    from skyline.dist import pack_export, unpack_union
    rows = torch.tensor([[0.0, -0.0, 1e300], [float("inf"), 2.5, -3.0]], dtype=torch.float64)
    keys = torch.tensor([3, 15], dtype=torch.int32)
    mult = torch.tensor([7, 1], dtype=torch.int64)
    pk = pack_export(rows, keys, mult)
    stacked = torch.stack([pk, torch.zeros_like(pk)])
    r, k, m = unpack_union(stacked, [2, 0], 3)
    assert torch.equal(r.view(torch.int64), rows.view(torch.int64))   # bit-preserving (keeps -0.0)
    assert k.tolist() == [3, 15] and m.tolist() == [7, 1]
