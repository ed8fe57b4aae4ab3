"""Multi-GPU sharding of history batches.

Histories are independent, so a batch is split into contiguous shards, one
per rank (one process per GPU); no data moves between ranks during the
search.  The only collective is one all-reduce of the qsmd_totals counters
(SUM) -- over RCCL/xGMI on the GPUs (torch.distributed "nccl" backend), over
gloo in the CPU tests -- plus a MAX of the early-stop flag.

The per-rank checker is a callable so the same driver runs the HIP search on
a GPU (``device_checker``) and is exercised on CPU with gloo in the tests.
"""

from __future__ import annotations

import numpy as np

TOTAL_FIELDS = ("checked", "linearisable", "nonlinearisable", "model_errors", "encode_errors",
                "budget", "skipped", "nodes")


def shard(n_total: int, rank: int, world: int):
    """Contiguous shard [first, first + count) of n_total items for rank."""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def totals_from_status(status, nodes):
    """qsmd_totals of one shard from its per-history outputs."""
    st = np.asarray(status)
    t = np.zeros(len(TOTAL_FIELDS), dtype=np.int64)
    t[1] = int((st == 1).sum())
    t[2] = int((st == 0).sum())
    t[3] = int((st == 2).sum())
    t[4] = int((st == 3).sum())
    t[5] = int((st == 4).sum())
    t[6] = int((st == 5).sum())
    t[0] = t[1] + t[2] + t[3]
    t[7] = int(np.asarray(nodes, dtype=np.int64).sum())
    return t


def allreduce_totals(local_totals, stop_flag=0, group=None):
    """SUM the counters and MAX the early-stop flag across ranks.  Works with
    a CPU (gloo) or CUDA (nccl = RCCL) tensor; returns numpy int64[8], flag."""
    import torch
    import torch.distributed as dist

    if isinstance(local_totals, torch.Tensor):
        t = local_totals
    else:
        t = torch.as_tensor(np.asarray(local_totals, dtype=np.int64))
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        f = torch.tensor([int(stop_flag)], dtype=torch.int64, device=t.device)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
        stop_flag = int(f.item())
    return t.cpu().numpy().astype(np.int64), int(stop_flag)


def check_sharded(checker, gen_params, n_total, rank, world, group=None):
    """Generate this rank's shard of a seeded synthetic stream, check it with
    ``checker(model_id, hdr, events) -> (status, nodes)`` and all-reduce the
    totals.  Returns (global totals, (first, count), status, nodes)."""
    from . import gen

    first, count = shard(n_total, rank, world)
    hdr, events, _ = gen.generate(gen_params, first, count)
    status, nodes = checker(gen_params.model_id, hdr, events)
    local = totals_from_status(status, nodes)
    stop = int((np.asarray(status) == 0).any() or (np.asarray(status) == 2).any())
    tot, stop = allreduce_totals(local, stop, group)
    return tot, stop, (first, count), status, nodes


def device_checker(ctx, max_nodes=0):
    """Checker running the HIP search through the C ABI (host buffers)."""
    def run(model_id, hdr, events):
        st, nd, _, _ = ctx.check_arrays(model_id, hdr, events, max_nodes=max_nodes)
        return st, nd
    return run
