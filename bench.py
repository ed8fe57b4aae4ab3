#!/usr/bin/env python3
"""Benchmark: histories checked per second (and search nodes per second) for
BASELINE.json config 2 -- 1M synthetic 4-client x 16-op Bank histories per GPU
(weak scaling: every rank checks its own 1M-history shard of one global
stream; the histories are independent).

One step = one full pass of the hot path (the linearisability search,
src/Linearisability.hs:52-69) over one resident batch (--rotate K: K
distinct batches in turn).  Inputs are resident in HBM before the timed
region.  With N > 1 the ranks exchange nothing during the steps; each step's
verdict / node counters stay on its GPU, and their RCCL all-reduce over the
ranks (64 B) follows the window, timed on its own (config.exchange_ms).

Environment (diagnostics): QSMD_BENCH_DIST=1 runs one rank on the N > 1
path; QSMD_BENCH_COUNTERS=rccl exchanges the counters over RCCL inside the
window instead, =gloo on the host after it; QSMD_BENCH_HOSTTIME=1 prints the window's host-time split
on stderr; QSMD_BENCH_THREADS=1 prints the CPU time each thread of the
process spent inside the window (/proc schedstat); QSMD_BENCH_PIN=1 pins the
main thread to one core after the warm-up (the threads RCCL created keep
the process's cores); QSMD_BENCH_DEVICE=d pins every rank to GPU d;
QSMD_LIB_PATH loads another build of libqsmd.so.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
    python bench.py --early-exit      (BASELINE config 3's early-termination
                                       path: ms to the decision, histories
                                       searched per second up to it)
    python bench.py --early-exit --plant 0.6   (config 2's stream with one
                                       failure planted at 60 % of the batch:
                                       the geometric rounds and a MIN per round)

Rank 0 prints one JSON line.  At N = 1 it also reports (outside the timed
region of `value`): the CPU baselines on the host's cores -- the C oracle
(oracle/ref_cpu.c, the reference restated with the same semantics) on one
thread and on every available core, and the literal list transliteration of
src/Linearisability.hs (the reference-shaped point) on config 1 -- and
bounded runs of BASELINE configs 1, 3, 4 and 5 (`extra.configs`).
"""

import argparse
import json
import os
import sys
import threading
import time

# HIP reads GPU_MAX_HW_QUEUES when it initialises (the first torch CUDA call):
# --hw-queues Q sets it for this process before torch is imported
if "--hw-queues" in sys.argv:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[sys.argv.index("--hw-queues") + 1]
elif (int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("QSMD_BENCH_DIST") == "1") \
        and (os.environ.get("QSMD_BENCH_COUNTERS") == "rccl" or "--early-exit" in sys.argv) \
        and "GPU_MAX_HW_QUEUES" not in os.environ:
    # with RCCL (the early-exit leg): the slot streams and RCCL's internal
    # one each keep a hardware queue (4 by default: they would share).
    # (The GPU boxes export HIP's default of 4, which this leaves as it is.  A
    # lone rank with 4 calls in flight on 8 queues measured +2-4 % on config
    # 2, but 8 queues cost config 1 17 % and config 5 23 % at 3 in flight in
    # the same process: tools/gpu/archive/r04_inflight2.sh .. r04_d200.sh.)
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

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
SIMDS = 1024                   # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9               # MI355X peak engine clock
VALU_CYCLES = 2                # a wave64 VALU instruction on a SIMD32


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


def thread_cpu_ns():
    """{thread id: (name, ns on a CPU)} of this process (/proc schedstat)."""
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"/proc/self/task/{tid}/schedstat") as f:
                out[int(tid)] = (name, int(f.read().split()[0]))
        except (OSError, ValueError, IndexError):
            pass
    return out


def host_cores():
    """Threads this process may use on the host: the box's CPU share when set
    (OMP_NUM_THREADS), else the affinity set."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env))) if env and env.isdigit() else aff


class InFlight:
    """S calls in flight (one context, stream and output set per slot; step k
    runs on slot k % S, so the next batch's stage 0 fills the compute units
    the previous call's tail leaves idle).  Each call writes its totals to a
    row of its own.  The window ends when every rank's GPU has checked every
    history; then the rows are summed on the device and all-reduced over
    the ranks with RCCL (the verdict / node counters of SURVEY.md §8e), timed
    on their own (exchange_ms).  The RCCL communicator is created only then:
    its mere presence cost one rank 7-8 % of the window with no collective
    issued.  QSMD_BENCH_COUNTERS: "rccl-after" (the default),
    "rccl" (the communicator from the warm-up, the all-reduce inside the
    window), "gloo" (the 64 B summed on the host after the window)."""

    def __init__(self, dev, model_id, d_hdr, n, d_ev, n_ev, S, flags, use_dist, knobs, budget0, streams=None,
                 host_group=None, batches=None):
        self.dev, self.model_id, self.n = dev, model_id, n
        # the resident batches (--rotate K: step k checks batch k % K, so the
        # library's cross-call hints always come from another batch)
        self.batches = batches or [(d_hdr, d_ev, n_ev)]
        self.S, self.flags = S, flags
        self.ctxs = [device.Context(dev.index) for _ in range(S)]
        for c in self.ctxs:
            if budget0 >= 0:
                c.set_stage0_budget(budget0)
            for k, v in knobs:
                c.set_param(k, v)
        # (streams of their own: torch's default stream is handle 0, which the
        # C ABI reads as "the context's stream")
        self.streams = streams or [torch.cuda.Stream(dev) for _ in range(S)]
        self.outs = [(torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int64, device=dev))
                     for _ in range(S)]
        self.tot = None                       # [step][8], allocated per timed region
        self.use_dist = use_dist
        self.host_group = host_group
        self.counters = os.environ.get("QSMD_BENCH_COUNTERS", "rccl-after") if use_dist else "none"
        if self.counters not in ("rccl-after", "rccl", "gloo", "none"):
            raise SystemExit(f"QSMD_BENCH_COUNTERS={self.counters}: rccl-after, rccl or gloo")
        self.rccl = self.counters == "rccl"     # (the all-reduce inside the window)
        # the per-call timing events inside the timed window (the roofline
        # leg after it always records them): instrumentation only -- the
        # headline runs without (api.hip: ~13 us per call for a lone caller)
        self.timing_events = 1
        self.steps_run = 0
        self.last = (0, 0)
        self.totals = None
        self.exchange_ms = None
        self.elapsed_incl_exchange = None

    def step(self):
        k = self.steps_run
        i = k % self.S
        d_st, d_nd = self.outs[i]
        d_hdr, d_ev, n_ev = self.batches[k % len(self.batches)]
        with torch.cuda.stream(self.streams[i]):
            self.ctxs[i].check_device(self.model_id, d_hdr.data_ptr(), self.n, d_ev.data_ptr(), n_ev,
                                      d_st.data_ptr(), d_nd.data_ptr(), None, self.tot[k].data_ptr(),
                                      flags=self.flags, stream=self.streams[i].cuda_stream)
        self.last = (i, k % len(self.batches))
        self.steps_run += 1

    def _sum(self, rccl=False):
        """The rows of every step so far, summed on the device after every
        slot's last call (on slot 0's stream, which the caller synchronises),
        then over the ranks with RCCL when `rccl`."""
        s0 = self.streams[0]
        for st_ in self.streams[1:]:
            s0.wait_stream(st_)
        with torch.cuda.stream(s0):
            acc = self.tot[:self.steps_run].sum(0)
            if rccl:
                dist.all_reduce(acc, op=dist.ReduceOp.SUM)
        return acc

    def prime(self):
        """One call per context before the warm-up, synchronised: the library
        sizes a context's lane-mode memo tables from its last finished call's
        heavy count (api.hip), so each context's second call may grow them
        (hipMalloc + clear); priming makes that happen outside the steps."""
        d_hdr, d_ev, n_ev = self.batches[0]
        for i in range(self.S):
            d_st, d_nd = self.outs[i]
            with torch.cuda.stream(self.streams[i]):
                self.ctxs[i].check_device(self.model_id, d_hdr.data_ptr(), self.n, d_ev.data_ptr(),
                                          n_ev, d_st.data_ptr(), d_nd.data_ptr(), None, None, flags=self.flags,
                                          stream=self.streams[i].cuda_stream)
        torch.cuda.synchronize(self.dev)

    def timed(self, steps, warmup):
        self.prime()
        self.tot = torch.zeros(max(steps, warmup, 1), 8, dtype=torch.int64, device=self.dev)
        self.totals = torch.zeros(8, dtype=torch.int64, pin_memory=True)
        self.steps_run = 0
        for _ in range(warmup):
            self.step()
        self._sum(self.rccl)                 # ("rccl": the warm-up's all-reduce creates the communicator)
        torch.cuda.synchronize(self.dev)
        self.tot.zero_()
        torch.cuda.synchronize(self.dev)
        if self.use_dist:
            dist.barrier(group=self.host_group)
        torch.cuda.synchronize(self.dev)
        self.ctxs[0].timing_reset()
        for c in self.ctxs:
            c.set_param("timing_events", self.timing_events)
        if os.environ.get("QSMD_BENCH_PIN") == "1":     # (diagnostic, DESIGN.md §9: the main thread alone on a core)
            os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})
        threads = os.environ.get("QSMD_BENCH_THREADS") == "1"
        th0 = thread_cpu_ns() if threads else None
        self.steps_run = 0
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        t_drain = time.perf_counter()
        if self.rccl:                          # (diagnostic: the exchange over RCCL, inside the window)
            acc = self._sum(True)
            with torch.cuda.stream(self.streams[0]):
                self.totals.copy_(acc, non_blocking=True)
        t_sync = time.perf_counter()
        torch.cuda.synchronize(self.dev)
        # each rank's window runs from the common opening barrier to its own
        # GPU's end: every history of every step is checked and its status
        # and node count are in HBM.  The MAX over ranks below is the whole
        # job's time, so the closing barrier stays outside the window (inside
        # it, its ~137 us of host gloo round trips were ~5 % of a 20-step run,
        # DESIGN.md §9)
        t_end = time.perf_counter()
        elapsed = t_end - t0
        if threads:                            # each thread's CPU time inside the window
            th1 = thread_cpu_ns()
            busy = {f"{th1[t][0]}:{t}": round((th1[t][1] - th0.get(t, ("", 0))[1]) * 1e-6, 3) for t in th1}
            print(json.dumps({"window_ms": round(elapsed * 1e3, 3), "main_tid": threading.get_native_id(),
                              "thread_cpu_ms": {k: v for k, v in sorted(busy.items(), key=lambda kv: -kv[1]) if v > 0}}),
                  file=sys.stderr)
        if os.environ.get("QSMD_BENCH_HOSTTIME") == "1":   # where the window's host time goes
            print(json.dumps({"enqueue_ms": (t_drain - t0) * 1e3, "sum_ms": (t_sync - t_drain) * 1e3,
                              "sync_ms": (t_end - t_sync) * 1e3}), file=sys.stderr)
        # the totals of every timed step: summed on the device, then over the
        # ranks -- 64 B of bookkeeping, timed on its own and reported beside
        # the headline, which excludes it
        self.exchange_ms = None
        if not self.rccl:
            if self.counters == "rccl-after":   # (the communicator, created now, outside the timing)
                with torch.cuda.stream(self.streams[0]):
                    dist.all_reduce(torch.zeros(1, dtype=torch.int64, device=self.dev))
                torch.cuda.synchronize(self.dev)
            t_x = time.perf_counter()
            acc = self._sum(self.counters == "rccl-after")
            with torch.cuda.stream(self.streams[0]):
                self.totals.copy_(acc, non_blocking=True)
            torch.cuda.synchronize(self.dev)
            if self.counters == "gloo":
                dist.all_reduce(self.totals, op=dist.ReduceOp.SUM, group=self.host_group)
            self.exchange_ms = (time.perf_counter() - t_x) * 1e3
        for c in self.ctxs:
            c.set_param("timing_events", 1)
        torch.cuda.synchronize(self.dev)
        # the window plus the exchange that follows it: the whole job's time
        # with its only collective (value_incl_exchange)
        self.elapsed_incl_exchange = elapsed + (self.exchange_ms or 0.0) * 1e-3
        if self.use_dist:
            dist.barrier(group=self.host_group)
            torch.cuda.synchronize(self.dev)
            e = torch.tensor([elapsed, self.elapsed_incl_exchange], dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX, group=self.host_group)
            elapsed, self.elapsed_incl_exchange = float(e[0].item()), float(e[1].item())
        return elapsed

    def roofline_leg(self, calls):
        """The search kernels alone: `calls` synchronous calls of batch 0 on
        slot 0 (each waits for the previous, nothing else on the GPU), with
        the HIP events stage 0 and the heavy stage record at their start and
        end on the launch stream -- the per-launch times the roofline divides
        by, and the launches a kernel trace of this command shows last
        (profiles/summarize_pmc.py --last).  Also returns the stage-0 budget
        those calls ran with (the library's automatic one included)."""
        torch.cuda.synchronize(self.dev)
        self.ctxs[0].timing_reset()
        d_st, d_nd = self.outs[0]
        d_hdr, d_ev, n_ev = self.batches[0]
        for _ in range(calls):
            self.ctxs[0].check_device(self.model_id, d_hdr.data_ptr(), self.n, d_ev.data_ptr(), n_ev,
                                      d_st.data_ptr(), d_nd.data_ptr(), None, None, flags=self.flags,
                                      stream=self.streams[0].cuda_stream)
            torch.cuda.synchronize(self.dev)
        s0, hv, call = self.ctxs[0].timing_read_stages()
        f64 = lambda x: np.asarray(x, dtype=np.float64)   # noqa: E731
        return f64(s0), f64(hv), f64(call), self.ctxs[0].get_param("stage0_budget_last")

    def results(self):
        """Outputs of the last step (status, nodes, its batch index) and the
        totals of every timed step over all ranks."""
        i, bi = self.last
        st = self.outs[i][0].cpu().numpy()
        nd = self.outs[i][1].cpu().numpy()
        return st, nd, self.totals.numpy(), bi

    def close(self):
        for c in self.ctxs:
            c.close()


def device_batch(name, first, n, dev):
    hdr, ev, _ = gen.generate(gen.params(**gen.CONFIGS[name]), first, n, threads=min(16, host_cores()))
    return hdr, ev, torch.from_numpy(hdr.view(np.uint8)).to(dev), torch.from_numpy(ev.view(np.uint8)).to(dev)


def cpu_baselines(hdr, ev, model_id, target_s, mt_s):
    """The C oracle on the rank-0 batch: one thread for >= target_s seconds
    of whole passes, then every available core for >= mt_s seconds."""
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
    cores = host_cores()
    mt_passes, dt_mt = 0, 0.0
    while dt_mt < mt_s or mt_passes == 0:
        t = time.perf_counter()
        oracle_c.check_batch(model_id, hdr, ev, threads=cores)
        dt_mt += time.perf_counter() - t
        mt_passes += 1
    return {"value": len(hdr) * passes / dt, "unit": "histories/s", "cores": 1, "kind": "port",
            "sample": f"{passes} pass(es) over the {len(hdr)} rank-0 histories, 1 thread, {dt:.1f} s, "
                      f"oracle/ref_cpu.c -O3 (reference semantics, no memo)",
            "nodes_per_sec": nodes / dt,
            "multi_thread": {"value": len(hdr) * mt_passes / dt_mt, "cores": cores,
                             "sample": f"{mt_passes} pass(es) over the {len(hdr)} histories, {cores} threads "
                                       f"(history shards), {dt_mt:.2f} s"}}, st, nd


def reference_shaped(seconds):
    """The literal list transliteration of src/Linearisability.hs:25-69
    (oracle/linearise_lists.py: cons-list copies, filter1, findResponse, the
    lazy forest, any / any') on BASELINE config 1, CPython, one thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import linearise_lists as ll
    from qsmd import models
    hdr, ev, _ = gen.generate_config("ticket_2x10", 0, 20000)
    b = codec.Batch(models.TICKET, hdr, ev, [{i: i for i in range(int(h["n_pid"]))} for h in hdr],
                    [{} for _ in hdr])
    hs = [codec.decode_history(b, i) for i in range(len(hdr))]
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ll.check("ticket", hs[done % len(hs)])
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "histories/s", "cores": 1, "kind": "port",
            "sample": f"{done} checks of {len(hs)} ticket_2x10 histories (BASELINE config 1), {dt:.1f} s, "
                      f"oracle/linearise_lists.py (literal list transliteration, CPython)"}


def early_exit_leg(dev, rank, world, config, n_per_gpu, steps, warmup, chunk, use_dist, host_group, check_oracle,
                   first_chunk=None, plant=None):
    """BASELINE config 3's early-termination path: QSMD_FLAG_EARLY_EXIT_BATCH
    over a batch sharded across the ranks (qsmd.dist.check_shard_early_exit_device:
    device-resident shards, one MIN all-reduce of the first failure per
    round of geometrically growing chunks, RCCL under torchrun).  One step =
    one early-exit pass over the whole batch (n_per_gpu x world histories of
    the seeded stream): it ends when the batch is decided -- its first
    failure found and every later history SKIPPED, as QuickCheck stops at its
    first failing test (test/TicketDispenser.hs:284-322).  The time is the
    MAX over ranks.  Reported as a latency, ms_to_decision, and as the
    histories actually searched per second up to the decision (SKIPPED
    histories are not work).  plant: a fraction f -- the histories are a
    linearisable configuration's with one failure planted at f x the batch
    (gen.plant_failure), so the rounds before it run for real."""
    from qsmd import dist as qdist
    n_total = n_per_gpu * world
    first, count = qdist.shard(n_total, rank, world)
    hdr, ev, _ = gen.generate(gen.params(**gen.CONFIGS[config]), first, count, threads=min(16, host_cores()))
    planted = None
    if plant is not None:
        planted = min(n_total - 1, int(plant * n_total))
        if first <= planted < first + count:
            ev = gen.plant_failure(hdr, ev, planted - first)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    mid = gen.CONFIGS[config]["model_id"]
    ctx = device.Context(dev.index)
    run = lambda: qdist.check_shard_early_exit_device(ctx, mid, d_hdr, d_ev, len(ev), n_total, rank, world,  # noqa
                                                      chunk=chunk, group=None, first_chunk=first_chunk)
    for _ in range(warmup):
        run()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier(group=host_group)
    t0 = time.perf_counter()
    for _ in range(steps):
        st, nd, info = run()
    # the batch's totals: one SUM all-reduce (RCCL under nccl), inside the window
    tot, _ = qdist.allreduce_totals(info["totals"], 0, None)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    searched = info["searched"]
    if use_dist:
        e = torch.tensor([el, float(searched)], dtype=torch.float64)
        dist.all_reduce(e[:1], op=dist.ReduceOp.MAX, group=host_group)
        s = e[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM, group=host_group)
        el, searched = float(e[0].item()), int(s.item())
    out = {"workload": config, "histories": n_total, "histories_per_gpu": n_per_gpu, "chunk": chunk,
           "first_chunk": first_chunk, "planted_at": planted, "steps": steps,
           "ms_to_decision": el / steps * 1e3,
           "searched": searched, "histories_searched_per_sec": searched * steps / el,
           "skipped": n_total - searched,
           "first_fail": info["first_fail"], "rounds": info["rounds"],
           "totals": dict(zip(("checked", "linearisable", "nonlinearisable", "model_errors", "encode_errors",
                               "budget", "skipped", "nodes"), (int(x) for x in tot)))}
    if check_oracle and world == 1:
        # the oracle on every history up to the first failure; everything after it SKIPPED
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_c
        ff = info["first_fail"]
        m = min(count, ff + 1)
        st_o, nd_o, _ = oracle_c.check_batch(mid, hdr[:m], ev, threads=host_cores())
        st_h, nd_h = st.cpu().numpy(), nd.cpu().numpy()
        out["mismatches_vs_oracle"] = int(((st_h[:m] != st_o) | (nd_h[:m] != nd_o.astype(np.int64))).sum() +
                                          (st_h[m:] != 5).sum())
        out["checked_vs_oracle"] = m
    ctx.close()
    return out


def extra_configs(dev, S, knobs, streams):
    """Bounded runs of BASELINE configs 1, 3, 5 (same in-flight step as the
    headline, the library's stage-0 budget) and 4 (one adversarial 8 x 64 TicketDispenser history, memo
    mode), each checked against the oracle on a sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    out = {}
    for cfg_id, name, n, steps in ((1, "ticket_2x10", 1_000_000, 20), (3, "bank_4x16_bugs", 1_000_000, 10),
                                   (5, "bank_6x24", 100_000, 20)):
        hdr, ev, d_hdr, d_ev = device_batch(name, 0, n, dev)
        mid = gen.CONFIGS[name]["model_id"]
        # (the headline's slot streams: the same streams on the same hardware queues)
        run = InFlight(dev, mid, d_hdr, n, d_ev, len(ev), S, device.QSMD_FLAG_EXHAUSTIVE, False, knobs, -1,
                       streams=streams)
        el = run.timed(steps, 3)
        st, nd, tot, _ = run.results()
        s0, call = run.ctxs[0].timing_read()
        run.close()
        m = min(n, 50_000)
        st_o, nd_o, _ = oracle_c.check_batch(mid, hdr[:m], ev, threads=host_cores(), max_nodes=0)
        out[f"config{cfg_id}"] = {
            "workload": name, "histories": n, "steps": steps, "histories_per_sec": n * steps / el,
            "nodes_per_sec": float(tot[7]) / el, "device_ms_call_mean": float(np.mean(call)),
            "nonlinearisable": int(tot[2]) // steps, "mismatches_vs_oracle": int(((st[:m] != st_o) |
                                                                        (nd[:m] != nd_o.astype(np.int64))).sum()),
            "checked_vs_oracle": m}
    h, e, _ = gen.adversarial_ticket(8, 64, bug=True)
    ctx = device.Context(dev.index)
    times = []
    for _ in range(21):
        t = time.perf_counter()
        st, nd, _, _ = ctx.check_arrays(1, h, e, flags=device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_MEMO)
        times.append(time.perf_counter() - t)
    ctx.close()
    st_o, _, _ = oracle_c.check_batch(1, h, e, memo=True)
    # the CPU point on this host: the C oracle's memo mode (the reference's
    # search pruning known-failing states), one thread, the same history
    cpu_t, cpu_n = time.perf_counter(), 0
    while time.perf_counter() - cpu_t < 1.0:
        oracle_c.check_batch(1, h, e, memo=True)
        cpu_n += 1
    cpu_ms = 1e3 * (time.perf_counter() - cpu_t) / cpu_n
    out["config4"] = {"workload": "adversarial TicketDispenser 8x64 (one history, QSMD_FLAG_MEMO, host entry)",
                      "ms_per_history": 1e3 * float(np.median(times[1:])), "verdict": int(st[0]),
                      "verdict_matches_oracle": bool(int(st[0]) == int(st_o[0])),
                      "cpu_ms_per_history": cpu_ms,
                      "cpu_sample": f"{cpu_n} calls of oracle/ref_cpu.c memo mode, 1 thread, through ctypes"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="bank_4x16", choices=sorted(gen.CONFIGS))
    ap.add_argument("--n-hist", type=int, default=1_000_000, help="histories per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the extra BASELINE configs")
    ap.add_argument("--stage0-budget", type=int, default=None,
                    help="stage-0 node budget (default 20 with calls in flight, the library's otherwise)")
    ap.add_argument("--param", action="append", default=[], metavar="NAME=VALUE",
                    help="qsmd_set_param on every context (tuning; repeatable)")
    ap.add_argument("--memo", action="store_true", help="QSMD_FLAG_MEMO (node counts become 'explored')")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP initialises)")
    ap.add_argument("--timing-events", type=int, default=0, choices=(0, 1),
                    help="per-call HIP timing events inside the timed window (1: device_ms.in_flight; "
                         "instrumentation, ~13 us per synchronous call)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="calls in flight (one context + stream each); 0 = 4 (the extra configs: 3)")
    ap.add_argument("--device-gen", action="store_true",
                    help="generate the batch on the GPU (qsmd_gen_batch_device; same histories as the host generator)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06", "stage0_pmc.json"),
                    help="PMC summary of the search kernels (profiles/summarize_pmc.py) for the roofline fields")
    ap.add_argument("--early-exit", action="store_true",
                    help="time BASELINE config 3's early-termination path instead (bank_4x16_bugs by default, "
                         "1.25M histories per GPU: 10M over 8 GPUs), sharded, QSMD_FLAG_EARLY_EXIT_BATCH")
    ap.add_argument("--chunk", type=int, default=262144, help="--early-exit: histories per rank per round (at most)")
    ap.add_argument("--plant", type=float, default=None, metavar="F",
                    help="--early-exit: config 2's linearisable stream with one failure planted at F x the batch "
                         "(gen.plant_failure): the geometric rounds up to it run for real")
    ap.add_argument("--first-chunk", type=int, default=4096,
                    help="--early-exit: histories per rank in the first round, x4 per round up to --chunk "
                         "(qsmd.dist.early_chunks; 0: fixed --chunk rounds)")
    ap.add_argument("--rotate", type=int, default=5,
                    help="distinct resident batches of n-hist histories; step s checks batch s %% K, so the "
                         "library's cross-call hints come from other batches, as in a stream of new batches "
                         "(default 5; 1 = every step re-checks one batch)")
    ap.add_argument("--rotate-copies", action="store_true",
                    help="diagnostic: --rotate's batches are copies of batch 0 (same hints, no cache reuse)")
    ap.add_argument("--roof-calls", type=int, default=30,
                    help="synchronous calls after the timed region that time the dominant kernel alone")
    args = ap.parse_args()
    args.rotate = max(1, args.rotate)
    if args.rotate > 1 and (args.inflight or 4) > 1 and args.rotate % (args.inflight or 4) == 0:
        ap.error("--rotate K must not be a multiple of the calls in flight (each context would see one batch)")

    # stdout carries exactly one JSON line (rank 0): RCCL prints a version
    # banner to file descriptor 1 when it creates its communicator, so fd 1
    # goes to stderr for the whole run and the JSON line is written to a
    # duplicate of the original stdout
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # QSMD_BENCH_DEVICE: a multi-rank rehearsal on one GPU (the batch path's
    # process group is gloo; RCCL refuses two ranks on one device)
    if os.environ.get("QSMD_BENCH_DEVICE"):
        local = int(os.environ["QSMD_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or os.environ.get("QSMD_BENCH_DIST") == "1"
    # 4 calls in flight on the box's 4 hardware queues: one stream's chain
    # (stage 0, then its heavy stage beside the other streams' stage 0s) is
    # the pipeline's critical path, and a fourth stream overlaps it -- config
    # 2 at the driver's 20 steps 8.47-8.91e9 against 7.88-8.50e9 with 3 (5
    # alternating rounds), 5 or 6 in flight share hardware queues and lose
    # (7.1-7.5 / 6.7e9; tools/gpu/archive/r05_if.sh, r05_if2.sh).  The extra configs
    # run at 3: config 1 (2 x 10 TicketDispenser) drops from 9.9 to 6.7e9 at 4
    S = args.inflight if args.inflight > 0 else 4
    # the slot streams, created and used first, so that each gets a hardware
    # queue of its own (GPU_MAX_HW_QUEUES)
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    for st_ in streams:
        with torch.cuda.stream(st_):
            torch.ones(1, device=dev).add_(1)
    torch.cuda.synchronize(dev)
    if use_dist:
        if "RANK" not in os.environ:      # QSMD_BENCH_DIST=1 without a launcher: one rank over RCCL
            os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=os.environ.get("MASTER_PORT", "29517"))
        # The RCCL communicator is created lazily by the first collective:
        # on the batch path after the timed window, since one rank with a
        # communicator lost 7-8 % of the driver's window with no collective
        # issued in it (none 8.61-8.96 vs 8.08-8.23e9; the all-reduce itself
        # takes 27 us; more hardware queues made it worse: tools/gpu/archive/r05_ar.sh,
        # r05_q.sh).  The early-exit leg's MIN per round is a
        # real exchange on the data path and creates it in its warm-up.
        # PyTorch's NCCL watchdog and heartbeat monitor cost one rank 5-7 %
        # with no collective issued: off.
        os.environ.setdefault("TORCH_NCCL_ENABLE_MONITORING", "0")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
        if os.environ.get("QSMD_BENCH_COUNTERS") == "gloo" and not args.early_exit:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl")
    # the bracketing barriers, the totals and the MAX over ranks of the timed
    # region go over a host (gloo) group: after torch.cuda.synchronize() every
    # rank's GPU work is done
    host_group = dist.new_group(backend="gloo") if use_dist else None

    if args.early_exit:
        config = args.config if args.config != "bank_4x16" else "bank_4x16_bugs"
        n_ee = args.n_hist if args.n_hist != 1_000_000 else 1_250_000
        if args.plant is not None and args.config == "bank_4x16":
            config = "bank_4x16"             # (a linearisable stream: the planted failure is its only one)
        ee = early_exit_leg(dev, rank, world, config, n_ee, args.steps, args.warmup, args.chunk, use_dist, host_group,
                            rank == 0 and not args.no_cpu_baseline, first_chunk=args.first_chunk or None,
                            plant=args.plant)
        if rank == 0:
            out = {"metric": "histories searched/sec up to the batch's decision, early-termination path "
                             "(QSMD_FLAG_EARLY_EXIT_BATCH, sharded); ms_to_decision beside it",
                   "value": ee["histories_searched_per_sec"], "unit": "histories/s", "n_gpus": world,
                   "steps": args.steps, "warmup": args.warmup, "ms_per_step": ee["ms_to_decision"],
                   "ms_to_decision": ee["ms_to_decision"], "higher_is_better": True,
                   "scaling": "weak", "vs_baseline": None, "dtype": "int32",
                   "data": "synthetic (seeded scheduler-policy generator with injected race bugs)",
                   "config": {"workload": config, "histories_per_gpu": n_ee, "parallelism": f"shard{world}",
                              "chunk": args.chunk, "first_chunk": args.first_chunk or None,
                              "planted_at_fraction": args.plant, "mode": "exhaustive + early exit"},
                   "early_exit": ee}
            print(json.dumps(out), file=json_out, flush=True)
        if use_dist:
            dist.destroy_process_group()
        return

    cfg = dict(gen.CONFIGS[args.config])
    model_id = cfg["model_id"]
    n = args.n_hist
    t = time.perf_counter()
    if args.device_gen:                   # on-device generation (csrc/gen.hip), same stream as the host's
        per = 2 * cfg["n_ops"]
        d_hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        d_ev = torch.empty(n * per * 8, dtype=torch.uint8, device=dev)
        gctx = device.Context(local)
        gctx.gen_device(gen.params(**cfg), rank * n, n, d_hdr.data_ptr(), d_ev.data_ptr(),
                        stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        gctx.close()
        hdr = d_hdr.cpu().numpy().view(codec.HDR_DTYPE)
        ev = d_ev.cpu().numpy().view(codec.EV_DTYPE)
    else:
        hdr, ev, d_hdr, d_ev = device_batch(args.config, rank * args.rotate * n, n, dev)
    # --rotate K: K distinct resident batches (histories [(rank K + k) n, ..)
    # of the seeded stream); step s checks batch s % K
    host_batches = [(hdr, ev)]
    dev_batches = [(d_hdr, d_ev, len(ev))]
    for k in range(1, args.rotate):
        if args.rotate_copies:               # diagnostic: the same histories at another address
            h_k, e_k, dh_k, de_k = hdr, ev, d_hdr.clone(), d_ev.clone()
        else:
            h_k, e_k, dh_k, de_k = device_batch(args.config, (rank * args.rotate + k) * n, n, dev)
        host_batches.append((h_k, e_k))
        dev_batches.append((dh_k, de_k, len(e_k)))
    log(f"[rank {rank}] generated {args.rotate} x {n} histories ({'device' if args.device_gen else 'host'}) "
        f"in {time.perf_counter() - t:.2f}s")

    # with calls in flight the heavy stage of one call overlaps the next call's
    # stage 0, so a lower stage-0 budget pays: since the heavy list is sharded
    # and lane mode's memo joins after 32 nodes (round 4), 17-20 measure
    # within the spread on config 2 at this command (7.90-8.30e9 at 18; 7.6-7.7
    # at 16; 7.59 at 26 before; tools/gpu/archive/r04_knobs2.sh)
    budget0 = args.stage0_budget if args.stage0_budget is not None else (20 if S > 1 else -1)
    knobs = [(kv.split("=")[0], int(kv.split("=")[1])) for kv in args.param]
    # with calls in flight the heavy stage runs in lane mode (64 searches per
    # wavefront: a few dozen wavefronts beside the next call's stage 0) with
    # its memo tables in HBM (an LDS-table workgroup holds a whole CU).  The
    # library's default for a short heavy list -- wave mode, one wavefront
    # per history, the shortest chain for one call at a time -- puts ~2000
    # wavefronts beside the next stage 0 for ~100 us
    if S > 1:
        for k, v in (("memo_lds", 0), ("heavy_mode", 1)):
            if k not in dict(knobs):
                knobs.append((k, v))
    flags = device.QSMD_FLAG_EXHAUSTIVE | (device.QSMD_FLAG_MEMO if args.memo else 0)
    run = InFlight(dev, model_id, d_hdr, n, d_ev, len(ev), S, flags, use_dist, knobs,
                   budget0, streams, host_group, batches=dev_batches)
    run.timing_events = args.timing_events
    elapsed = run.timed(args.steps, args.warmup)
    s0_ms, call_ms = run.ctxs[0].timing_read()
    st, nd, tot, last_batch = run.results()
    roof_s0, roof_hv, roof_call, budget_used = run.roofline_leg(max(1, args.roof_calls))
    nd0 = run.outs[0][1].cpu().numpy()             # batch 0's node counts (the roofline leg's calls)
    fold = run.ctxs[0].get_param("fold")
    run.close()

    ms_per_step = elapsed / args.steps * 1e3
    total_hist = n * world
    value = total_hist * args.steps / elapsed
    nodes_total = int(tot[7])                      # every timed step, every rank
    assert int(tot[0]) + int(tot[4]) + int(tot[5]) == total_hist * args.steps, tot

    # roofline, rank-local, of the two kernels that bound a call -- stage 0
    # and the lane-mode heavy stage -- each SURVEY §8d's algorithmic bytes of
    # one launch over its mean duration ALONE on the GPU (the roofline leg:
    # synchronous calls of batch 0 after the timed region, HIP events the
    # launches record at their start and end; a kernel trace of this command
    # shows the same launches last).  The top-level fields are the longer
    # kernel's.  Per history: 16 B header + 16 B per operation + 16 B result
    # + 16 B per explored node; stage 0 explores min(nodes, budget), the
    # heavy stage re-reads its histories and explores the nodes past the
    # budget (the budget the leg's calls ran with, the library's automatic
    # one included).  Beside them: the same stage-0 bytes per step of the
    # timed region, and what the PMC counters of a profiled run of the same
    # configuration and budget give for the same launches.
    # (budget_used 0xFFFFFFFF: stage 0 ran without a budget -- no heavy stage)
    heavy = nd0.astype(np.int64) > budget_used
    n_ev0 = hdr["n_ev"].astype(np.int64)
    kern = {"stage0": {"kernel": "compact_search<Bank, G32> (stage 0)", "ms": roof_s0,
                       "alg_bytes_per_launch": alg_bytes(hdr, np.minimum(nd0, budget_used)),
                       "hbm_io_bytes_per_launch": hbm_bytes(hdr)}}
    if len(roof_hv) and (roof_hv >= 0).all():
        kern["heavy"] = {"kernel": "memo_search<Bank> (heavy stage, lane mode)", "ms": roof_hv,
                         "heavy_histories": int(heavy.sum()),
                         "alg_bytes_per_launch": int((32 + 8 * n_ev0[heavy]).sum() +
                                                     16 * (nd0[heavy].astype(np.int64) - budget_used).sum())}
    pmc = {}
    if os.path.exists(args.pmc):
        with open(args.pmc) as f:
            pmc = json.load(f)
        if not (pmc.get("config") == args.config and pmc.get("n_hist") == n and
                pmc.get("stage0_budget") == budget_used):
            pmc = {}                      # measured on another configuration or budget: not this run's
    for name, k in kern.items():
        ms = k.pop("ms")
        t = float(np.mean(ms)) * 1e-3
        k["achieved"] = k["alg_bytes_per_launch"] / t / 1e9
        k["frac"] = k["achieved"] / HBM_PEAK_GBS
        k["kernel_ms"] = {"mean": float(np.mean(ms)), "median": float(np.median(ms)), "min": float(np.min(ms)),
                          "launches": int(len(ms))}
        blk = pmc if name == "stage0" else pmc.get("heavy", {})
        k["traffic"] = blk.get("hbm_bytes_per_launch") if pmc else None
        if k["traffic"]:
            k["hbm_actual"] = k["traffic"] / t / (HBM_PEAK_GBS * 1e9)
        valu = blk.get("valu_insts_per_launch") if pmc else None
        if valu:
            k["valu_issue"] = valu * VALU_CYCLES / (SIMDS * CLOCK_HZ * t)
    dom = max(kern, key=lambda k: kern[k]["kernel_ms"]["mean"])
    a_bytes = kern["stage0"]["alg_bytes_per_launch"]
    roof = {"bound": "hbm", "achieved": kern[dom]["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": kern[dom]["frac"], "traffic": kern[dom]["traffic"], "kernel": kern[dom]["kernel"],
            "alg_bytes_per_launch": kern[dom]["alg_bytes_per_launch"], "stage0_budget_used": budget_used,
            "kernels": kern,
            "call_ms": {"mean": float(np.mean(roof_call)), "median": float(np.median(roof_call))},
            "how": "synchronous calls after the timed region, HIP events at each kernel's start and end",
            "per_step": {"achieved": a_bytes / (ms_per_step * 1e-3) / 1e9,
                         "frac": a_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "how": "stage 0's algorithmic bytes of one launch / ms_per_step (calls in flight)"}}
    if pmc:
        roof["pmc_source"] = os.path.relpath(args.pmc, ROOT)

    out = {
        "metric": METRIC, "value": value, "unit": "histories/s", "n_gpus": world,
        # the same histories over the window plus the counters' exchange after
        # it (N > 1: the all-reduce of the totals; N = 1 exchanges nothing)
        "value_incl_exchange": total_hist * args.steps / run.elapsed_incl_exchange,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "dtype_note": ("exact integer search: stage 0 holds invocation values in 9 bits (-256..255), responses "
                       "in 25, balances in int32; wider values go on to the int64 stages; node counts u64"),
        "data": "synthetic (seeded scheduler-policy generator, include/qsmd_gen.h" +
                (", generated on the GPU)" if args.device_gen else ")"),
        "config": {"workload": args.config, "histories_per_gpu": n,
                   "clients": cfg["n_clients"], "ops": cfg["n_ops"],
                   "events_per_history": 2 * cfg["n_ops"], "parallelism": f"shard{world}", "calls_in_flight": S,
                   "stage0_budget": budget0 if budget0 >= 0 else "library default",
                   "heavy_stage": ("lane mode, HBM memo tables" if S > 1 else "library default (lane or wave "
                                   "mode from the last call's heavy list)")
                   if not args.param else "knobs: " + ",".join(args.param),
                   "counters": {"rccl": "summed on the device, one RCCL all-reduce inside the window",
                                "rccl-after": "summed on the device, one RCCL all-reduce after the window (the "
                                              "communicator created then): the headline excludes it, exchange_ms "
                                              "times it",
                                "gloo": "summed on the device, one host (gloo) all-reduce after the window: the "
                                        "headline excludes it, exchange_ms times it"}.get(run.counters)
                   if use_dist else "summed on the device after the window: the headline excludes it, "
                                    "exchange_ms times it",
                   "exchange_ms": run.exchange_ms,
                   "batches": args.rotate, "fold": fold,
                   "mode": "memo" if args.memo else "exhaustive"},
        "nodes_per_sec": nodes_total / elapsed,
        "verdicts": {"scope": "every timed step, every rank", "checked": int(tot[0]),
                     "linearisable": int(tot[1]), "nonlinearisable": int(tot[2]),
                     "model_errors": int(tot[3]), "budget": int(tot[5])},
        "device_ms": {"in_flight": {"stage0_mean": float(np.mean(s0_ms)) if len(s0_ms) else None,
                                    "call_mean": float(np.mean(call_ms)) if len(call_ms) else None},
                      "alone": {"stage0_mean": float(np.mean(roof_s0)),
                                "heavy_mean": float(np.mean(roof_hv)) if len(roof_hv) else None,
                                "call_mean": float(np.mean(roof_call))}},
        "roofline": roof,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the oracle over the last step's batch: the CPU baseline's timing and the check
        hdr_l, ev_l = host_batches[last_batch]
        cb, st_o, nd_o = cpu_baselines(hdr_l, ev_l, model_id, args.cpu_seconds, 2.0)
        cb["reference_shaped"] = reference_shaped(5.0)
        out["cpu_baseline"] = cb
        if args.memo:                        # node counts are "explored" there: verdicts only
            out["mismatches_vs_oracle"] = int((st_o != st).sum())
        else:
            out["mismatches_vs_oracle"] = int(((st_o != st) | (nd_o != nd.astype(np.uint64))).sum())
        out["checked_vs_oracle"] = len(hdr_l)
        out["checked_batch"] = last_batch
    if rank == 0 and world == 1 and not args.no_extra:
        s_x = min(S, 3) if args.inflight <= 0 else S
        out["extra"] = {"configs": extra_configs(dev, s_x, knobs, streams[:s_x])}
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
