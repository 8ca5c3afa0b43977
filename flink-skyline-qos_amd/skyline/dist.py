"""Multi-GPU skyline: one process per GPU, shards of the tuple stream per rank.

Exactness: SKY(u_k SKY(P_k)) = SKY(u P_k) for ANY split, so:
  1. each rank reduces its own shard to the distinct vectors of its local skylines, with
     partition key and multiplicity (sky_export_local_dev);
  2. the ranks exchange those vectors with ONE all-gather (RCCL over xGMI when the process
     group is "nccl"; gloo on CPU for tests), counts first;
  3. each rank decides the fate of ITS OWN vectors against the gathered union
     (sky_import_union_dev: in L_k iff no union vector of key k dominates it, in G iff no
     union vector dominates it) -- |own| x |union| pair tests per rank, so the global phase
     shrinks with the number of ranks instead of being replicated on every rank;
  4. the per-rank shares of |L_k| and survivors_k are summed with one all-reduce of 2K
     integers (the optimality inputs, FlinkSkyline.java:593-608).
Tuple ids never leave their rank: each rank emits its own global-skyline ids.

Wire format of one exported vector (int64 words): D value words (f64 bits),
1 partition key, 1 multiplicity  ->  [count, D+2] int64 per rank, padded to the
largest count (counts are all-gathered first).
"""
import time

import numpy as np
import torch
import torch.distributed as dist


def pack_export(rows_f64, keys_i32, mult_i64):
    """[n,D] f64, [n] i32, [n] i64 -> [n, D+2] i64 (bit-preserving)."""
    n, D = rows_f64.shape
    out = torch.empty((n, D + 2), dtype=torch.int64, device=rows_f64.device)
    out[:, :D] = rows_f64.contiguous().view(torch.int64)
    out[:, D] = keys_i32.to(torch.int64)
    out[:, D + 1] = mult_i64
    return out


def unpack_union(packed, counts, D):
    """all-gathered [W, maxc, D+2] + per-rank counts -> contiguous union tensors."""
    parts = [packed[r, :int(c)] for r, c in enumerate(counts)]
    u = torch.cat(parts, 0) if parts else packed.new_empty((0, D + 2))
    rows = u[:, :D].contiguous().view(torch.float64)
    keys = u[:, D].to(torch.int32).contiguous()
    mult = u[:, D + 1].contiguous()
    return rows, keys, mult


def allgather_varlen(packed, group=None):
    """Gather a [n, W] int64 tensor of per-rank length n from every rank.
    Returns (stacked [world, maxn, W], counts list).  With a gloo group (CPU
    collectives: tests, or rehearsing several ranks on one GPU) device tensors are
    staged through host memory; with nccl (RCCL) they stay in HBM."""
    world = dist.get_world_size(group)
    if packed.device.type == "cuda" and dist.get_backend(group) == "gloo":
        out, counts = allgather_varlen(packed.cpu(), group)
        return out.to(packed.device), counts
    dev = packed.device
    cnt = torch.tensor([packed.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    maxc = max(max(counts), 1)
    W = packed.shape[1]
    buf = torch.zeros((maxc, W), dtype=torch.int64, device=dev)
    buf[:packed.shape[0]] = packed
    out = torch.empty((world, maxc, W), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out.view(world * maxc, W), buf, group=group)
    return out, counts


def allreduce_stats(ls, sv, device, group=None):
    """Sum the per-rank |L_k| / survivors_k shares over the ranks (one all-reduce)."""
    K = len(ls)
    backend = dist.get_backend(group)
    dev = device if (backend != "gloo" and device.type == "cuda") else torch.device("cpu")
    t = torch.from_numpy(np.concatenate([ls, sv]).astype(np.int64)).to(dev)
    dist.all_reduce(t, group=group)
    t = t.cpu().numpy()
    return t[:K], t[K:]


def distributed_query(engine, d_ids, d_vals, d_ids_out, d_origin_out, cap, group=None):
    """One query over the union of every rank's shard.  Returns this rank's
    number of global-skyline ids written to d_ids_out (stream order); afterwards
    engine.stats() holds the job-wide |L_k| / survivors_k and engine.last_dist_stats
    the exchange's sizes and phase times."""
    D = engine.dims
    dev = d_vals.device
    t0 = time.perf_counter()
    ne = engine.export_local_dev(d_ids, d_vals)
    rows = torch.empty((max(ne, 1), D), dtype=torch.float64, device=dev)
    keys = torch.empty(max(ne, 1), dtype=torch.int32, device=dev)
    mult = torch.empty(max(ne, 1), dtype=torch.int64, device=dev)
    if ne:
        engine.export_copy_dev(rows, keys, mult, ne)
    engine.sync()
    t1 = time.perf_counter()
    packed = pack_export(rows[:ne], keys[:ne], mult[:ne])
    gathered, counts = allgather_varlen(packed, group)
    urows, ukeys, umult = unpack_union(gathered, counts, D)
    rank = dist.get_rank(group)
    self_off = sum(counts[:rank])
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    g = engine.import_union_dev(urows, ukeys, umult, urows.shape[0], self_off, d_ids_out, d_origin_out, cap)
    ls, sv = engine.stats()                      # this rank's share
    t3 = time.perf_counter()
    ls, sv = allreduce_stats(ls, sv, dev, group)
    engine.set_stats(ls, sv)
    t4 = time.perf_counter()
    n_union = int(urows.shape[0])
    engine.last_dist_stats = {
        "world": dist.get_world_size(group), "union_vectors": n_union, "own_vectors": ne,
        "exchange_bytes_per_rank": int(gathered.numel() * 8),
        "own_x_union_pair_tests": ne * n_union,
        "ms": {"export": (t1 - t0) * 1e3, "allgather": (t2 - t1) * 1e3, "import": (t3 - t2) * 1e3,
               "stats_allreduce": (t4 - t3) * 1e3}}
    return g
