"""gloo tests (CPU, world sizes 2 and 4) of the multi-GPU exchange in skyline/dist.py.

The device phases are stood in for by the oracle (test infrastructure): each rank reduces
its shard to the distinct vectors of its local skylines with partition + multiplicity
(sky_export_local_dev), the ranks exchange them with skyline.dist.allgather_varlen /
pack_export / unpack_union over gloo, each rank decides the fate of ITS OWN vectors
against the union (sky_import_union_dev's rule: in L_k iff no union vector of key k
dominates it, in G iff no union vector dominates it), and the per-rank shares of |L_k| /
survivors_k are summed by skyline.dist.allreduce_stats.  The result must equal the
single-process answer, and each rank's global-phase work must be its share (|own| x
|union|, about 1/G of the |union|^2 a replicated merge would cost)."""
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
    _, keys, _, _, inl = orc.query_sfs_chunked("angle", vals, P)
    inl = inl.astype(bool)
    rows = vals[inl]
    ks = keys[inl]
    uniq, cnt = np.unique(np.column_stack([ks, rows]), axis=0, return_counts=True)
    return uniq[:, 1:].copy(), uniq[:, 0].astype(np.int32), cnt.astype(np.int64)


def _dominates(a, b):
    return bool((a <= b).all() and (a < b).any())


def _worker(rank, world, port, shards, P, D, ret):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "flink-skyline-qos_amd"))
    import torch.distributed as dist
    from conftest import Oracle
    from skyline.dist import allgather_varlen, allreduce_stats, pack_export, unpack_union
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    orc = Oracle()
    rows, keys, mult = _local_export(orc, shards[rank], P)
    packed = pack_export(torch.from_numpy(rows), torch.from_numpy(keys), torch.from_numpy(mult))
    gathered, counts = allgather_varlen(packed)
    urows, ukeys, umult = unpack_union(gathered, counts, D)
    assert sum(counts) == urows.shape[0]
    off = sum(counts[:rank])
    assert torch.equal(urows[off:off + counts[rank]], torch.from_numpy(rows))
    u, uk = urows.numpy(), ukeys.numpy()
    ls = np.zeros(P, np.int64)
    sv = np.zeros(P, np.int64)
    gvecs = []
    pairs = 0
    for j in range(counts[rank]):               # own vectors only, each against the whole union
        y, ky = u[off + j], uk[off + j]
        dom_l = dom_g = False
        for i in range(len(u)):
            pairs += 1
            if _dominates(u[i], y):
                dom_g = True
                if uk[i] == ky:
                    dom_l = True
                    break
        if not dom_l:
            ls[ky] += mult[j]
        if not dom_g:
            sv[ky] += mult[j]
            gvecs.append(tuple(y))
    tls, tsv = allreduce_stats(ls, sv, torch.device("cpu"))
    ret[rank] = (sorted(gvecs), tls.tolist(), tsv.tolist(), pairs, len(u))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_rank_exchange_equals_single_process(world, oracle):
    n, D, P = 8000, 4, 8
    vals = oracle.synth(0, D, n, seed=3 + world)
    bounds = np.linspace(0, n, world + 1).astype(int)
    shards = [vals[bounds[r]:bounds[r + 1]] for r in range(world)]
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shards, P, D, ret)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    exp, keys, els, esv = oracle.query_sfs("angle", vals, P)
    exp_set = sorted({tuple(r) for r in vals[exp]})
    got_set = sorted({v for r in range(world) for v in ret[r][0]})
    assert got_set == exp_set
    n_union = ret[0][4]
    for r in range(world):
        assert ret[r][1] == els.tolist()          # job-wide integers after the all-reduce
        assert ret[r][2] == esv.tolist()
        # global-phase work of one rank: its own vectors against the union, ~1/G of |U|^2
        assert ret[r][3] <= 1.6 * n_union * n_union / world
    assert sum(ret[r][3] for r in range(world)) <= n_union * n_union


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
