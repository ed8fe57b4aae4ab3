#!/usr/bin/env python3
"""BASELINE config 4: one adversarial TicketDispenser history (8 clients x
64 ops, shared pid, heavy overlap, a bug at the end) searched by every GPU
with state memoisation (QSMD_FLAG_MEMO) and the root-frontier split of
SURVEY.md §8e (qsmd.dist.check_single_split: same frontier on every rank,
round-robin tasks, RCCL MIN all-reduce of the first deciding task, SUM
gather, ordered fold).

    python tools/bench_single.py [--steps K] [--warmup W] [--no-bug] [--exhaustive]
    torchrun --nproc-per-node N tools/bench_single.py ...

Prints one JSON line on rank 0: seconds per single-history check (lower is
better) and the verdict, checked against the memo oracle on rank 0.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from qsmd import device, gen, models  # noqa: E402
from qsmd import dist as qdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--ops", type=int, default=64)
    ap.add_argument("--no-bug", action="store_true")
    ap.add_argument("--exhaustive", action="store_true", help="no memo (feasible only for small sizes)")
    ap.add_argument("--tasks-per-rank", type=int, default=64)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    h, e, _ = gen.adversarial_ticket(args.clients, args.ops, bug=not args.no_bug)
    flags = device.QSMD_FLAG_EXHAUSTIVE | (0 if args.exhaustive else device.QSMD_FLAG_MEMO)
    ctx = device.Context(local)

    def step():
        return qdist.check_single_split(ctx, models.MODEL_TICKET, h, e, rank, world, flags=flags,
                                        tasks_per_rank=args.tasks_per_rank)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    times = []
    res = None
    for _ in range(args.steps):
        t = time.perf_counter()
        res = step()
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t)
    el = float(np.mean(times))
    if world > 1:
        x = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())
    st, nodes, w, info = res
    out = {"metric": "single adversarial history check time (BASELINE config 4)", "value": el * 1e3,
           "unit": "ms", "higher_is_better": False, "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "mode": "exhaustive" if args.exhaustive else "memo",
           "config": {"workload": f"ticket_{args.clients}x{args.ops}_adversarial", "bug": not args.no_bug,
                      "events": int(h[0]["n_ev"])},
           "status": int(st), "nodes_explored": int(nodes), "split": info}
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_c
        st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_TICKET, h, e, memo=not args.exhaustive)
        out["oracle_status"] = int(st_o[0])
        out["oracle_nodes"] = int(nd_o[0])
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
