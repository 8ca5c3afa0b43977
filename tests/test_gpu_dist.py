"""Two real processes on the MI355X running skyline.dist.distributed_query (the
bench's multi-GPU step) over a gloo group: export -> all-gather -> import through
libskyline_hip in each rank.  Both ranks share cuda:0 (a one-GPU box); the RCCL
transport itself is exercised only by the driver's 8-GPU run.  The union of the
ranks' ids and the optimality integers must equal one single-process query."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "flink-skyline-qos_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, vals, D, P, ret):
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    import skyline
    from skyline.dist import distributed_query
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    n = len(vals) // world
    shard = vals[rank * n:(rank + 1) * n]
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
    dv = torch.from_numpy(np.ascontiguousarray(shard)).cuda()
    di = torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64, device="cuda")
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    g = distributed_query(eng, di, dv, oi, oo, n)
    eng.sync()
    ls, sv = eng.stats()
    ret[rank] = (oi[:g].cpu().numpy().tolist(), oo[:g].cpu().numpy().tolist(), ls.tolist(), sv.tolist())
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("dist_id,D", [(2, 8), (3, 4), (0, 4)])
def test_two_process_distributed_query(dist_id, D, gpu_engine_factory, oracle):
    n, P = 40000, 16
    vals = oracle.synth(dist_id, D, 2 * n, seed=31 + D)
    eng = gpu_engine_factory(D, P, "mr-angle")
    exp_ids, exp_org = eng.query(vals, np.arange(2 * n))
    exp_ls, exp_sv = eng.stats()
    eng.close()
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, vals, D, P, ret)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    got = sorted(ret[0][0] + ret[1][0])
    assert got == sorted(exp_ids.tolist())
    org = dict(zip(ret[0][0] + ret[1][0], ret[0][1] + ret[1][1]))
    assert [org[i] for i in exp_ids.tolist()] == exp_org.tolist()
    for r in range(2):                       # every rank reports the job-wide integers
        assert ret[r][2] == exp_ls.tolist()
        assert ret[r][3] == exp_sv.tolist()
