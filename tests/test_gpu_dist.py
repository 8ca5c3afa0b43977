"""Real processes on the MI355X running skyline.dist.distributed_query (the bench's
multi-GPU step: sky_dist_export -> all-gather -> sky_dist_merge -> all-reduce ->
sky_dist_finish through libskyline_hip in each rank): two ranks over a gloo group sharing
cuda:0 (a one-GPU box), and one rank in an "nccl" (RCCL) group, which runs the device-resident
collectives of the 8-GPU path.  The union of the ranks' ids and the optimality integers must
equal one single-process query."""
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


def _nccl_worker(port, vals, D, P, ret):
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    import skyline
    from skyline.dist import distributed_query
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    n = len(vals)
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
    dv = torch.from_numpy(np.ascontiguousarray(vals)).cuda()
    di = torch.arange(n, dtype=torch.int64, device="cuda")
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    out = []
    for _ in range(3):
        g = distributed_query(eng, di, dv, oi, oo, n)
        torch.cuda.synchronize()
        ls, sv = eng.stats()
        out.append((oi[:g].cpu().numpy().tolist(), oo[:g].cpu().numpy().tolist(), ls.tolist(), sv.tolist(),
                    eng.last_dist_stats["host_syncs"]))
    ret[0] = out
    eng.close()
    dist.destroy_process_group()


def test_rccl_transport_single_rank(gpu_engine_factory, oracle):
    """The RCCL branch of skyline.dist (all_gather_into_tensor / all_reduce on device tensors,
    stream-ordered with the library's stream) in a world-1 "nccl" group on the one GPU: every
    step equals one query, and steps after the first make one host read."""
    n, D, P = 200000, 8, 16
    vals = oracle.synth(2, D, n, seed=5)
    eng = gpu_engine_factory(D, P, "mr-angle")
    exp_ids, exp_org = eng.query(vals, np.arange(n))
    exp_ls, exp_sv = eng.stats()
    eng.close()
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), vals, D, P, ret))
    p.start()
    p.join(180)
    assert p.exitcode == 0
    for ids, org, ls, sv, syncs in ret[0]:
        assert ids == exp_ids.tolist() and org == exp_org.tolist()
        assert ls == exp_ls.tolist() and sv == exp_sv.tolist()
    assert [x[4] for x in ret[0][1:]] == [1, 1]
