#!/usr/bin/env python3
"""Benchmark: histories checked per second (and search nodes per second) for
BASELINE.json config 2 -- 1M synthetic 4-client x 16-op Bank histories per GPU
(weak scaling: every rank checks its own 1M-history shard of one global
stream; the histories are independent).

One step = one full pass of the hot path (the linearisability search,
src/Linearisability.hs:52-69) over the resident batch + the RCCL all-reduce of
the verdict/node counters (the only collective).  Inputs are resident in HBM
before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Rank 0 prints one JSON line.  The cpu_baseline leg (N=1, rank 0) times the C
oracle (oracle/ref_cpu.c, the reference restated with the same semantics) on a
bounded sample of the same batch on the host's cores.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "quickcheck-state-machine-distributed_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: our library shares torch's HIP runtime)
import torch.distributed as dist  # noqa: E402

from qsmd import codec, device, gen  # noqa: E402

METRIC = ("histories checked/sec (whole node) + search nodes/sec, "
          "4×16-op Bank, 1/2/4/8 GPU")
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def alg_bytes(hdr, nodes):
    """SURVEY.md §8d algorithmic bytes: per history 16 B header + 16 B per
    operation (2 events x 8 B) + 16 B result + 16 B per explored node."""
    n_ev = hdr["n_ev"].astype(np.int64)
    return int((16 + 8 * n_ev + 16).sum() + 16 * nodes.astype(np.int64).sum())


def hbm_bytes(hdr):
    """Bytes that must cross HBM: header + events in, status + nodes out."""
    return int((16 + 8 * hdr["n_ev"].astype(np.int64) + 1 + 8).sum())


def cpu_baseline(hdr, ev, model_id, target_s):
    """Time the C oracle on the rank-0 batch, single thread, repeating whole
    passes until at least target_s seconds of CPU work have been measured."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    oracle_c.lib()
    passes, dt, nodes = 0, 0.0, 0.0
    st = nd = None
    while dt < target_s or passes == 0:
        t = time.perf_counter()
        st, nd, _ = oracle_c.check_batch(model_id, hdr, ev, threads=1)
        dt += time.perf_counter() - t
        nodes += float(nd.astype(np.float64).sum())
        passes += 1
    n = len(hdr) * passes
    # SURVEY.md §8d also asks for the same port on every host core (history shards per thread)
    threads = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    oracle_c.check_batch(model_id, hdr, ev, threads=threads)
    dt_mt = time.perf_counter() - t
    return {"value": n / dt, "unit": "histories/s", "cores": 1, "kind": "port",
            "sample": f"{passes} pass(es) over the {len(hdr)} rank-0 histories, 1 thread, {dt:.1f} s, "
                      f"oracle/ref_cpu.c -O3 (reference semantics, no memo)",
            "nodes_per_sec": nodes / dt,
            "multi_thread": {"value": len(hdr) / dt_mt, "cores": threads,
                             "sample": f"1 pass over the {len(hdr)} histories, {threads} threads, {dt_mt:.2f} s"}}, \
        st, nd, len(hdr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="bank_4x16", choices=sorted(gen.CONFIGS))
    ap.add_argument("--n-hist", type=int, default=1_000_000, help="histories per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split-budget", type=int, default=None,
                    help="per-lane node budget before the split stage (library default if unset)")
    ap.add_argument("--stage0-budget", type=int, default=None,
                    help="fixed stage-0 node budget (the rest go to the memo stage); default 40 with calls in "
                         "flight (the next batch hides the memo stage; tools/gpu/inflight_budget*.sh, "
                         "profiles/r01/v7/inflight_budget_sweep.json), the adaptive cascade one call at a time; -1 = adaptive")
    ap.add_argument("--param", action="append", default=[], metavar="NAME=VALUE",
                    help="qsmd_set_param on every context (tuning; repeatable)")
    ap.add_argument("--memo", action="store_true", help="QSMD_FLAG_MEMO (node counts become 'explored')")
    ap.add_argument("--inflight", type=int, default=0,
                    help="calls in flight (one context + stream each): the next step's search overlaps the tail of "
                         "the previous one; 0 = 3 on one GPU, 2 with RCCL (its stream takes one of the 4 hardware queues)")
    ap.add_argument("--ar-rounds", type=int, default=16,
                    help="rounds of in-flight steps whose counters one RCCL all-reduce carries (N > 1)")
    ap.add_argument("--device-gen", action="store_true",
                    help="generate the batch on the GPU (qsmd_gen_batch_device; same histories as the host generator)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC summary written by profiles/profile.sh (for roofline.traffic)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # the counter all-reduce (QSMD_BENCH_DIST=1 exercises it on one rank too)
    use_dist = world > 1 or os.environ.get("QSMD_BENCH_DIST") == "1"
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)

    cfg = dict(gen.CONFIGS[args.config])
    model_id = cfg["model_id"]
    n = args.n_hist
    ctx = device.Context(local)
    t = time.perf_counter()
    if args.device_gen:                   # on-device generation (csrc/gen.hip), same stream as the host's
        per = 2 * cfg["n_ops"]
        d_hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        d_ev = torch.empty(n * per * 8, dtype=torch.uint8, device=dev)
        ctx.gen_device(gen.params(**cfg), rank * n, n, d_hdr.data_ptr(), d_ev.data_ptr(),
                       stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        hdr = d_hdr.cpu().numpy().view(codec.HDR_DTYPE)
        ev = d_ev.cpu().numpy().view(codec.EV_DTYPE)
    else:
        hdr, ev, bug = gen.generate(gen.params(**cfg), rank * n, n, threads=min(16, os.cpu_count() or 1))
        d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
        d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    log(f"[rank {rank}] generated {n} histories ({'device' if args.device_gen else 'host'}) "
        f"in {time.perf_counter() - t:.2f}s")

    # S calls in flight (--inflight): one context, stream and output set per
    # slot; step k runs on slot k % S, so the next batch's stage 0 fills the
    # compute units the previous call's tail leaves idle.  Each step is the
    # full search of the batch; a slot's steps are ordered on its stream.
    S = args.inflight if args.inflight > 0 else (2 if use_dist else 3)
    ctxs = [ctx] + [device.Context(local) for _ in range(S - 1)]
    budget0 = args.stage0_budget if args.stage0_budget is not None else (40 if S > 1 else -1)
    for c in ctxs:
        if args.split_budget is not None:
            c.set_split_budget(args.split_budget)
        if budget0 >= 0:
            c.set_stage0_budget(budget0)
        for kv in args.param:
            name, value = kv.split("=")
            c.set_param(name, int(value))
    flags = device.QSMD_FLAG_EXHAUSTIVE | (device.QSMD_FLAG_MEMO if args.memo else 0)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    outs = [(torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int64, device=dev))
            for _ in range(S)]
    # counters: [block parity][step of the block][8]; a block is R rounds of S
    # steps (--ar-rounds), all-reduced together (one bucketed RCCL all-reduce
    # per block, overlapping the next block; a row is reused two blocks later,
    # after it)
    R = max(1, args.ar_rounds)
    B = R * S
    tot = torch.zeros(2, B, 8, dtype=torch.int64, device=dev)
    # (the round's all-reduce runs on the last slot's stream: RCCL adds its own
    # stream, and more streams than hardware queues serialise each other)
    comm = streams[S - 1] if use_dist else None
    do_ar = use_dist and os.environ.get("QSMD_BENCH_NOAR") != "1"   # (diagnostic: group without collectives)
    done = [None, None]                   # per parity: the round's all-reduce finished
    k_step = [0]

    def step():
        k = k_step[0]
        k_step[0] += 1
        i, row, par = k % S, k % B, (k // B) % 2
        d_st_i, d_nd_i = outs[i]
        with torch.cuda.stream(streams[i]):
            if done[par] is not None:
                streams[i].wait_event(done[par])
            ctxs[i].check_device(model_id, d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st_i.data_ptr(),
                                 d_nd_i.data_ptr(), None, tot[par, row].data_ptr(), flags=flags,
                                 stream=streams[i].cuda_stream)
        if do_ar and row == B - 1:        # the block is enqueued: its counters all-reduced together
            for st_ in streams[:-1]:
                comm.wait_stream(st_)
            with torch.cuda.stream(comm):
                dist.all_reduce(tot[par], op=dist.ReduceOp.SUM)
                done[par] = torch.cuda.Event()
                done[par].record(comm)
        return row, par

    def drain():
        if k_step[0] % B:                 # a partial last block: reduce it, start the next one fresh
            if do_ar:
                par = ((k_step[0] - 1) // B) % 2
                for st_ in streams[:-1]:
                    comm.wait_stream(st_)
                with torch.cuda.stream(comm):
                    dist.all_reduce(tot[par], op=dist.ReduceOp.SUM)
                    done[par] = torch.cuda.Event()
                    done[par].record(comm)
            k_step[0] = (k_step[0] + B - 1) // B * B

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    drain()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if use_dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    s0_ms, call_ms = ctx.timing_read()
    d_st, d_nd = outs[last[0] % S]
    st = d_st.cpu().numpy()
    nd = d_nd.cpu().numpy()
    tot = tot[last[1], last[0]].cpu().numpy()   # global totals of the last step
    ms_per_step = elapsed / args.steps * 1e3
    total_hist = n * world
    value = total_hist * args.steps / elapsed
    nodes_total = int(tot[7])
    assert int(tot[0]) + int(tot[4]) + int(tot[5]) == total_hist, tot

    # roofline of the dominant kernel (stage 0 search), rank-local
    s0_mean = float(np.mean(s0_ms)) if len(s0_ms) else float("nan")
    # (with a fixed stage-0 budget the kernel stops a history at that many
    # nodes and the memo stage searches it again: stage 0's own node work is
    # min(nodes, budget) per history)
    a_bytes = alg_bytes(hdr, np.minimum(nd, budget0) if budget0 > 0 else nd)
    achieved = a_bytes / (s0_mean * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        with open(args.traffic) as f:
            tr = json.load(f)
        if tr.get("config") == args.config and tr.get("n_hist") == n:
            traffic = tr.get("hbm_bytes_per_launch")

    out = {
        "metric": METRIC, "value": value, "unit": "histories/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded scheduler-policy generator, include/qsmd_gen.h" +
                (", generated on the GPU)" if args.device_gen else ")"),
        "config": {"workload": args.config, "histories_per_gpu": n,
                   "clients": cfg["n_clients"], "ops": cfg["n_ops"],
                   "events_per_history": 2 * cfg["n_ops"], "parallelism": f"shard{world}", "calls_in_flight": S,
                   "stage0_budget": budget0 if budget0 >= 0 else "adaptive",
                   "allreduce_every_steps": B if use_dist else None, "mode": "memo" if args.memo else "exhaustive"},
        "nodes_per_sec": nodes_total * args.steps / elapsed,
        "verdicts": {"checked": int(tot[0]), "linearisable": int(tot[1]),
                     "nonlinearisable": int(tot[2]), "model_errors": int(tot[3]),
                     "budget": int(tot[5])},
        "device_ms": {"stage0_mean": s0_mean, "call_mean": float(np.mean(call_ms)) if len(call_ms) else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "alg_bytes_per_launch": a_bytes, "hbm_io_bytes_per_launch": hbm_bytes(hdr),
                     "kernel": "compact_search<Bank> (stage 0)"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, st_o, nd_o, sample = cpu_baseline(hdr, ev, model_id, args.cpu_seconds)
        out["cpu_baseline"] = cb
        out["mismatches_vs_oracle"] = int(((st_o != st[:sample]) | (nd_o != nd[:sample].astype(np.uint64))).sum())
        out["checked_vs_oracle"] = sample
    if rank == 0:
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
