"""Multi-GPU sharding of history batches.

Histories are independent, so a batch is split into contiguous shards, one
per rank (one process per GPU); no data moves between ranks during the
search.  The only collective is one all-reduce of the qsmd_totals counters
(SUM) -- over RCCL/xGMI on the GPUs (torch.distributed "nccl" backend), over
gloo in the CPU tests -- plus the early-stop flag: with early exit, a MIN
of the first failing history's index after every chunk, so ranks stop
searching once every history left to them lies after it.

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
        t = local_totals.to(torch.int64)
    else:
        t = torch.as_tensor(np.asarray(local_totals, dtype=np.int64))
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = t.to(_collective_device(group))            # RCCL: device tensors only
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        f = torch.tensor([int(stop_flag)], dtype=torch.int64, device=t.device)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
        stop_flag = int(f.item())
    return t.cpu().numpy().astype(np.int64), int(stop_flag)


def _collective_device(group=None):
    """Where a collective's tensors must live: the current GPU under the nccl
    backend (RCCL over xGMI takes device tensors only), the host under gloo."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def check_sharded(checker, gen_params, n_total, rank, world, group=None, early_exit=False, chunk=65536):
    """Generate this rank's shard of a seeded synthetic stream, check it with
    ``checker(model_id, hdr, events) -> (status, nodes)`` and all-reduce the
    totals.  Returns (global totals, stop flag, (first, count), status, nodes).

    ``early_exit``: QuickCheck's stop at the first failing test
    (/root/reference/test/TicketDispenser.hs:284-322, ``expectFailure``)
    across ranks -- see check_shard_early_exit; the checker is then called
    as ``checker(model_id, hdr, events, early=True)``."""
    from . import gen

    first, count = shard(n_total, rank, world)
    hdr, events, _ = gen.generate(gen_params, first, count)
    if early_exit:
        status, nodes, info = check_shard_early_exit(checker, gen_params.model_id, hdr, events, n_total, rank,
                                                     world, chunk=chunk, group=group)
        tot, _ = allreduce_totals(totals_from_status(status, nodes), 0, group)
        return tot, int(info["first_fail"] < n_total), (first, count), status, nodes
    status, nodes = checker(gen_params.model_id, hdr, events)
    local = totals_from_status(status, nodes)
    stop = int((np.asarray(status) == 0).any() or (np.asarray(status) == 2).any())
    tot, stop = allreduce_totals(local, stop, group)
    return tot, stop, (first, count), status, nodes


def chunk_slice(hdr, events, a, b):
    """Histories [a, b) of a batch as a batch of their own: headers rebased
    onto the events they span (one copy of those events per chunk, not of
    the shard's)."""
    h = np.array(hdr[a:b], copy=True)
    if len(h) == 0:
        return h, events[:0]
    lo = int(h["ev_off"].min())
    hi = int((h["ev_off"].astype(np.int64) + h["n_ev"].astype(np.int64)).max())
    h["ev_off"] -= lo
    return h, events[lo:hi]


def early_chunks(n_max, chunk, first_chunk=None, growth=4):
    """The chunk schedule of the sharded early exit: round k checks offsets
    [a_k, b_k) of every rank's shard (the same offsets on every rank, so each
    rank can tell when all of them are done).  Geometric by default: the
    first round checks ``first_chunk`` histories per rank and every round
    ``growth`` times more, up to ``chunk`` -- a batch whose first failure
    comes early (config 3's injected bugs: most do) is decided after a
    small first round instead of a full chunk, while a batch without one
    still takes only a few more rounds.  first_chunk None or >= chunk: fixed
    chunks of ``chunk``."""
    assert chunk > 0
    w = chunk if not first_chunk or first_chunk >= chunk else max(1, int(first_chunk))
    out, a = [], 0
    while a < n_max:
        out.append((a, min(n_max, a + w)))
        a += w
        w = min(chunk, w * max(1, growth))
    return out


def check_shard_early_exit(checker, model_id, hdr, events, n_total, rank, world, chunk=65536, group=None,
                           first_chunk=None):
    """QSMD_FLAG_EARLY_EXIT_BATCH over a sharded batch ("a MAX
    on the early-stop flag"; here the flag carries the smallest global index
    of a failing history, a MIN all-reduce).

    Each rank checks its contiguous shard in chunks (early_chunks: of
    ``chunk`` histories, or growing from ``first_chunk`` up to it), each
    with the device's early exit (everything after the chunk's first
    non-linearisable or raising history is SKIPPED).  After every chunk one
    MIN all-reduce publishes the global index of the first failing history
    found so far; a rank stops once its next chunk starts after it.  Every
    rank runs the same number of rounds (each computes every rank's chunk
    schedule, so all take the same decision to stop).  Afterwards the
    histories after the global first failure are SKIPPED with 0 nodes, so
    status, nodes and totals equal one context's QSMD_FLAG_EARLY_EXIT_BATCH
    over the concatenated batch: every history up to the first failure is
    searched in full (its chunk started before it, and a chunk only skips
    after its own first failure, which is never earlier).

    Returns (status, nodes, info) for this rank's shard; info holds the
    global first failure (n_total if none), the rounds and the histories
    this rank searched (not SKIPPED by the device, in chunks it ran)."""
    import torch.distributed as dist

    first, count = shard(n_total, rank, world)
    assert len(hdr) == count
    status = np.full(count, 5, dtype=np.uint8)                 # SKIPPED until searched
    nodes = np.zeros(count, dtype=np.uint64)
    starts = [shard(n_total, r, world) for r in range(world)]  # (first, count) of every rank
    sched = early_chunks(max(c for _, c in starts) if n_total else 0, chunk, first_chunk)
    best = n_total                                             # global first failure (none: n_total)
    searched = 0
    rounds = 0
    for a, b in sched:
        # does any rank still have a chunk that starts before the first failure?
        if not any(a < c and f + a < best for f, c in starts):
            break
        local = best
        if a < count and first + a < best:
            b = min(count, b)
            h, e = chunk_slice(hdr, events, a, b)
            st, nd = checker(model_id, h, e, early=True)
            st = np.asarray(st, dtype=np.uint8)
            status[a:b] = st
            nodes[a:b] = np.asarray(nd, dtype=np.uint64)
            searched += int((st != 5).sum())
            fails = np.nonzero((st == 0) | (st == 2))[0]
            if len(fails):
                local = min(local, first + a + int(fails[0]))
        best = int(_allreduce(np.array([local]), dist.ReduceOp.MIN, group)[0])
        rounds += 1
    cut = best - first                                         # local index of the global first failure
    if cut < count:
        after = max(0, cut + 1)
        status[after:] = 5
        nodes[after:] = 0
    return status, nodes, dict(first_fail=best, rounds=rounds, searched=searched)


def check_shard_early_exit_device(ctx, model_id, d_hdr, d_ev, n_events, n_total, rank, world, chunk=262144,
                                  group=None, max_nodes=0, first_chunk=None):
    """check_shard_early_exit on DEVICE-resident buffers (the
    reference's parallel property stops at its first failing test,
    /root/reference/test/TicketDispenser.hs:284-322).

    d_hdr / d_ev: this rank's shard as uint8 torch tensors on its GPU (the
    include/qsmd.h records; ev_off relative to d_ev).  Each round checks the
    rank's next chunk (early_chunks) in place through qsmd_check_batch_device
    with QSMD_FLAG_EARLY_EXIT_BATCH (headers at the chunk's offset, the
    shard's whole event buffer, outputs into the shard's status / node
    arrays).  The chunk's first failure comes from its device totals -- with
    the flag every history after it is SKIPPED, so it is the chunk's last
    history minus the skipped count; the 64-byte totals row is the only
    thing read back per round, and one MIN all-reduce per round (RCCL on a
    device tensor under nccl) publishes the global first failure.  Status
    and node arrays stay on the device; the totals are the rounds' rows
    summed on the host, with every history after the global first failure
    SKIPPED (no status is read back for that: see _early_rounds).  The
    calls and copies run on a stream of their own, ordered after the
    caller's.  Same rounds, stopping rule and
    final SKIPPED marking as the host version, so status, nodes and totals
    equal one context's early exit over the concatenated batch.

    Returns (status u8 tensor, nodes i64 tensor, info) for this rank's shard;
    info: first_fail (n_total if none), rounds, searched (histories the
    device did not skip), totals (this rank's, an int64[8] host tensor) --
    all-reduce them with allreduce_totals for the batch's."""
    import torch
    import torch.distributed as dist

    first, count = shard(n_total, rank, world)
    dev = d_hdr.device
    starts = [shard(n_total, r, world) for r in range(world)]
    sched = early_chunks(max(c for _, c in starts) if n_total else 0, chunk, first_chunk)
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    cdev = _collective_device(group) if multi else dev
    # the calls and the torch ops below on one stream of their own (torch's
    # default stream is handle 0, which the C ABI reads as "the context's
    # stream": nothing would order the two), joined to the caller's at the end
    # (the outputs allocated on the caller's stream, which waits for the side
    # stream before it returns: the caching allocator never sees them freed
    # while the side stream still writes them)
    status = torch.empty(count, dtype=torch.uint8, device=dev)   # written by the calls, the rest filled
    nodes = torch.empty(count, dtype=torch.int64, device=dev)
    caller = torch.cuda.current_stream(dev)
    st_ = _side_stream(dev)
    st_.wait_stream(caller)
    with torch.cuda.stream(st_):
        out = _early_rounds(ctx, model_id, d_hdr, d_ev, n_events, n_total, first, count, starts, sched, multi, cdev,
                            group, max_nodes, st_.cuda_stream, status, nodes)
    caller.wait_stream(st_)
    return out


_SIDE_STREAMS = {}


def _side_stream(dev):
    """One side stream per device for the early-exit rounds (creating a HIP
    stream per call cost more than the rounds themselves)."""
    import torch

    k = dev.index if dev.index is not None else torch.cuda.current_device()
    if k not in _SIDE_STREAMS:
        _SIDE_STREAMS[k] = torch.cuda.Stream(dev)
    return _SIDE_STREAMS[k]


def _early_rounds(ctx, model_id, d_hdr, d_ev, n_events, n_total, first, count, starts, sched, multi, cdev, group,
                  max_nodes, s, status, nodes):
    import torch
    import torch.distributed as dist

    from . import device

    dev = d_hdr.device
    flags = device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_EARLY_EXIT_BATCH
    tot = torch.empty((max(len(sched), 1), 8), dtype=torch.int64, device=dev)
    acc = np.zeros(8, dtype=np.int64)                          # the rounds' totals rows
    best, rounds, searched, end = n_total, 0, 0, 0             # [0, end): the histories this rank checked
    for k, (a, b) in enumerate(sched):
        if not any(a < c and f + a < best for f, c in starts):
            break
        local = best
        if a < count and first + a < best:
            b = min(count, b)
            ctx.check_device(model_id, d_hdr.data_ptr() + 16 * a, b - a, d_ev.data_ptr(), n_events,
                             status.data_ptr() + a, nodes.data_ptr() + 8 * a, None, tot[k].data_ptr(),
                             flags=flags, max_nodes=max_nodes, stream=s)
            t = tot[k].cpu().numpy()                           # (waits for the call: s is the current stream)
            acc += t
            end = b
            searched += (b - a) - int(t[6])
            if t[2] + t[3] > 0:                                # the chunk's first failure
                local = min(local, first + b - 1 - int(t[6]))
        if multi:
            r = torch.full((1,), local, dtype=torch.int64, device=cdev)
            dist.all_reduce(r, op=dist.ReduceOp.MIN, group=group)
            best = int(r.item())
        else:
            best = local
        rounds += 1
    # The statuses after the global first failure end SKIPPED with 0 nodes.
    # Before this rank's shard (cut < 0): all of it.  In it: the failure is
    # this rank's own, found in the last chunk it checked (a rank stops at
    # its first), whose early exit already SKIPPED the rest of that chunk --
    # so the rows hold, and only the chunks never checked are left.
    cut = best - first
    lo = 0 if cut < 0 else end
    if cut < 0:
        acc[:] = 0
    acc[6] += count - lo
    if lo < count:
        status[lo:] = 5
        nodes[lo:] = 0
    return status, nodes, dict(first_fail=best, rounds=rounds, searched=searched, totals=torch.from_numpy(acc))


def device_checker(ctx, max_nodes=0):
    """Checker running the HIP search through the C ABI (host buffers);
    early=True adds QSMD_FLAG_EARLY_EXIT_BATCH."""
    from . import device

    def run(model_id, hdr, events, early=False):
        flags = device.QSMD_FLAG_EXHAUSTIVE | (device.QSMD_FLAG_EARLY_EXIT_BATCH if early else 0)
        st, nd, _, _ = ctx.check_arrays(model_id, hdr, events, flags=flags, max_nodes=max_nodes)
        return st, nd
    return run


# --------------------------------------------------------------------------
# One very large history across ranks (BASELINE config 4).

_NO_TASK = np.iinfo(np.int64).max


def _allreduce(arr, op, group=None):
    import torch
    import torch.distributed as dist

    t = torch.tensor(np.asarray(arr, dtype=np.int64))        # a copy: gloo reduces in place
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = t.to(_collective_device(group))
        dist.all_reduce(t, op=op, group=group)
    return t.cpu().numpy().astype(np.int64)


def round_windows(n, world, round_tasks=None, first_per_rank=2):
    """The task windows [c0, c1) of check_single_split's rounds: a fixed
    window of ``round_tasks`` tasks, or by default a geometric schedule --
    ``first_per_rank`` tasks per rank in the first round, doubling every
    round -- so an early deciding task (the first subtree of a linearisable
    history usually holds its witness) stops every rank after a few tasks,
    while an exhausted history still takes only ~log2(n / world) rounds."""
    out, c0 = [], 0
    w = round_tasks or max(1, first_per_rank) * world
    while c0 < n:
        out.append((c0, min(n, c0 + w)))
        c0 += w
        if not round_tasks:
            w *= 2
    return out


def check_single_split(checker, model_id, hdr, events, rank, world, model0=None, flags=1,
                       max_nodes=0, tasks_per_rank=64, round_tasks=None, group=None):
    """Search ONE history with every rank.

    Each rank cuts the search at the same frontier (checker.split_frontier
    is deterministic), so no task list is exchanged; rank r searches the
    tasks t = r, r + world, ... (round-robin in DFS order).  Work goes in
    rounds over windows of the task list (round_windows: geometric by
    default, or ``round_tasks`` per round); after each round one MIN
    all-reduce publishes the first task found deciding (True or Map.!) --
    the early-termination flag of §8e -- and no rank searches a task after
    it: every task before it has been searched in full by its owner, so the
    node count stays exact.  Then one SUM all-reduce gathers the per-task
    results (each rank contributes only its own entries) and every rank
    folds them in DFS order.

    checker: qsmd.device.Context (or anything with split_frontier /
    check_tasks).  Returns (status, nodes, witness path or None, info dict).
    """
    import torch.distributed as dist

    from . import device

    fr, tasks, w_top = checker.split_frontier(model_id, hdr, events, model0, flags, max_nodes,
                                              min_tasks=world * tasks_per_rank,
                                              max_tasks=max(4096, 2 * world * tasks_per_rank),
                                              witness=True)
    n = len(tasks)
    st_local = np.zeros(n, dtype=np.int64)           # status + 1 where searched here
    nd_local = np.zeros(n, dtype=np.int64)
    rows = {}
    best = _NO_TASK
    rounds = 0
    for c0, c1 in round_windows(n, world, round_tasks):
        sel = np.arange(c0 + (rank - c0) % world, c1, world)     # this rank's tasks t = rank (mod world)
        sel = sel[sel < best]
        if len(sel):
            s, nd, w = checker.check_tasks(model_id, hdr, events, tasks[sel], model0, flags, max_nodes,
                                           witness=True)
            st_local[sel] = s.astype(np.int64) + 1
            nd_local[sel] = nd.astype(np.int64)
            dec = sel[(s == 1) | (s == 2)]
            for t in sel[s == 1]:
                rows[int(t)] = w[int(np.nonzero(sel == t)[0][0])]
            if len(dec):
                best = min(best, int(dec.min()))
        best = int(_allreduce(np.array([best]), dist.ReduceOp.MIN, group)[0])
        rounds += 1
        if best != _NO_TASK:
            break
    st_all = _allreduce(st_local, dist.ReduceOp.SUM, group)
    nd_all = _allreduce(nd_local, dist.ReduceOp.SUM, group)
    status = np.where(st_all > 0, st_all - 1, 5).astype(np.uint8)     # unsearched: SKIPPED
    st_f, nodes, win = device.combine_tasks(fr, tasks, status, nd_all.astype(np.uint64), max_nodes)
    witness = None
    if st_f == 1:
        if win >= 0:
            mine = rows[win].astype(np.int64) + 1 if win in rows else np.zeros(64, dtype=np.int64)
            row = _allreduce(mine, dist.ReduceOp.SUM, group) - 1
            end = np.nonzero(row == 0xFF)[0]
            witness = row[: int(end[0]) if len(end) else 64].astype(np.uint8)
        else:
            end = np.nonzero(w_top == 0xFF)[0]
            witness = w_top[: int(end[0]) if len(end) else len(w_top)]
    info = dict(n_tasks=n, depth=int(fr.depth), top_nodes=int(fr.top_nodes), rounds=rounds,
                searched_here=int((st_local > 0).sum()), winner=win)
    return st_f, nodes, witness, info
