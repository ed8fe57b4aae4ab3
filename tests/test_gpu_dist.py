"""The multi-GPU driver (qsmd/dist.py) on the HIP kernels: two processes on
cuda:0 with the gloo backend, each with its own device.Context -- the batch
shards of SURVEY.md §8e (check_sharded with device_checker) and one history
split at its root frontier over the ranks (check_single_split).  On an
8-GPU node the same code runs one process per GPU over nccl (RCCL); that
scaling run is the driver's, not this test's."""

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _paths():
    sys.path[:0] = [os.path.join(HERE, "..", "quickcheck-state-machine-distributed_amd"),
                    os.path.join(HERE, "..", "oracle"), HERE]


def _heaviest(name, k, n=4000):
    import oracle_c
    from qsmd import gen
    hdr, ev, _ = gen.generate_config(name, 0, n)
    mid = gen.CONFIGS[name]["model_id"]
    st, nd, _ = oracle_c.check_batch(mid, hdr, ev, threads=4, max_nodes=10**7)
    out = []
    for i in np.argsort(-nd.astype(np.int64))[:k]:
        h = hdr[i:i + 1].copy()
        a, m = int(h[0]["ev_off"]), int(h[0]["n_ev"])
        h[0]["ev_off"] = 0
        out.append((mid, h, ev[a:a + m].copy()))
    return out


def _worker(rank, world, port, n_total, out_q):
    _paths()
    import torch
    import torch.distributed as dist

    from qsmd import device, gen
    from qsmd import dist as qdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = device.Context(0, time_limit_ms=60000)
    try:
        res = {}
        p = gen.params(**gen.CONFIGS["bank_4x16_bugs"])
        tot, stop, (first, count), st, nd = qdist.check_sharded(qdist.device_checker(ctx, max_nodes=10**7), p,
                                                                n_total, rank, world)
        res["shard"] = (tot.tolist(), stop, first, count, st.tolist(), [int(x) for x in nd])
        splits = []
        for mid, h, e in _heaviest("bank_4x16_bugs", 3):
            s, nodes, w, info = qdist.check_single_split(ctx, mid, h, e, rank, world, tasks_per_rank=16)
            splits.append((int(s), int(nodes), None if w is None else [int(x) for x in w], info["searched_here"]))
        for bug in (True, False):
            h, e, _ = gen.adversarial_ticket(8, 64, bug=bug)
            s, nodes, w, info = qdist.check_single_split(ctx, 1, h, e, rank, world, tasks_per_rank=16,
                                                         flags=device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_MEMO)
            splits.append((int(s), int(nodes), None if w is None else [int(x) for x in w], info["searched_here"]))
        res["split"] = splits
        # the linearisable 8 x 64 history once more in ONE round over every
        # task (no cross-rank early exit): the same verdict, more tasks searched
        h, e, _ = gen.adversarial_ticket(8, 64, bug=False)
        s, nodes, w, info = qdist.check_single_split(ctx, 1, h, e, rank, world, tasks_per_rank=16,
                                                     round_tasks=10**9,
                                                     flags=device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_MEMO)
        res["one_round"] = (int(s), None if w is None else [int(x) for x in w], info["searched_here"],
                            info["n_tasks"], info["rounds"])
        # QSMD_FLAG_EARLY_EXIT_BATCH over the shards (chunks, MIN all-reduce
        # of the first failure); rank 0 also runs one context's early exit over
        # the concatenated batch
        from test_distributed import planted_stream
        ee = []
        for config, plant in EARLY_CASES:
            hdr, ev = planted_stream(config, n_total, plant)
            mid = gen.CONFIGS[config]["model_id"]
            first, count = qdist.shard(n_total, rank, world)
            h, e = qdist.chunk_slice(hdr, ev, first, first + count)
            st, nd, info = qdist.check_shard_early_exit(qdist.device_checker(ctx, max_nodes=10**7), mid, h, e,
                                                        n_total, rank, world, chunk=2048,
                                                        first_chunk=128)
            # the same on device-resident buffers (one MIN all-reduce per chunk, statuses stay on the GPU)
            d_h = torch.from_numpy(h.view(np.uint8)).cuda()
            d_e = torch.from_numpy(e.view(np.uint8)).cuda()
            dst, dnd, dinfo = qdist.check_shard_early_exit_device(ctx, mid, d_h, d_e, len(e), n_total, rank, world,
                                                                  chunk=2048, max_nodes=10**7, first_chunk=128)
            dtot, _ = qdist.allreduce_totals(dinfo.pop("totals"))
            dev_res = (dst.cpu().tolist(), dnd.cpu().tolist(), dinfo, dtot.tolist())
            one = None
            if rank == 0:
                st1, nd1, _, tot1 = ctx.check_arrays(mid, hdr, ev, max_nodes=10**7, flags=device.QSMD_FLAG_EXHAUSTIVE |
                                                     device.QSMD_FLAG_EARLY_EXIT_BATCH)
                one = (st1.tolist(), [int(x) for x in nd1], tot1)
            ee.append((st.tolist(), [int(x) for x in nd], info, one, dev_res))
        res["early"] = ee
        out_q.put((rank, res))
    finally:
        ctx.close()
        dist.destroy_process_group()


# (config, planted failure): the generated bugs (a failure near the start),
# one failure deep in rank 1's shard, one in rank 0's
EARLY_CASES = [("bank_4x16_bugs", None), ("bank_4x16", 14000), ("bank_4x16", 6500)]


def test_two_processes_on_the_hip_kernels():
    import oracle_c
    from qsmd import dist as qdist
    from qsmd import gen

    world, n_total = 2, 20001
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # batch shards: every rank holds the global totals; the shards are the oracle's
    hdr, ev, _ = gen.generate(gen.params(**gen.CONFIGS["bank_4x16_bugs"]), 0, n_total)
    st_o, nd_o, _ = oracle_c.check_batch(gen.CONFIGS["bank_4x16_bugs"]["model_id"], hdr, ev, threads=8,
                                         max_nodes=10**7)
    want = qdist.totals_from_status(st_o, nd_o).tolist()
    for r in range(world):
        assert results[r]["shard"][0] == want
    cat_st = np.array(results[0]["shard"][4] + results[1]["shard"][4])
    cat_nd = np.array(results[0]["shard"][5] + results[1]["shard"][5])
    assert np.array_equal(cat_st, st_o) and np.array_equal(cat_nd, nd_o.astype(np.int64))
    # single histories split over the two ranks: the single search's verdict,
    # count and witness (exhaustive); the memo mode's verdict for 8 x 64
    for j, (mid, h, e) in enumerate(_heaviest("bank_4x16_bugs", 3)):
        s_o, n_o, w_o = oracle_c.check_batch(mid, h, e, witness=True)
        for r in range(world):
            s, nodes, w, _ = results[r]["split"][j]
            assert (s, nodes) == (int(s_o[0]), int(n_o[0]))
            if s == 1:
                assert w == [int(x) for x in w_o[:len(w)]]
        assert results[0]["split"][j][3] + results[1]["split"][j][3] > 0
    for k, bug in enumerate((True, False)):
        h, e, _ = gen.adversarial_ticket(8, 64, bug=bug)
        s_o, _, w_o = oracle_c.check_batch(1, h, e, memo=True, witness=True)
        for r in range(world):
            s, _, w, _ = results[r]["split"][3 + k]
            assert s == int(s_o[0]) == (0 if bug else 1)
            if not bug:
                assert w == [int(x) for x in w_o[:len(w)]]
    # cross-rank early exit (§8e): the geometric rounds stop both ranks at
    # the first deciding task; one round over all tasks searches them all
    early = sum(results[r]["split"][4][3] for r in range(world))
    full = sum(results[r]["one_round"][2] for r in range(world))
    for r in range(world):
        assert results[r]["one_round"][0] == results[r]["split"][4][0] == 1
        assert results[r]["one_round"][1] == results[r]["split"][4][2]
        assert results[r]["one_round"][4] == 1
    assert results[0]["one_round"][3] > 2 * world and early < full, (early, full)
    # sharded early exit == one context's early exit over the whole batch,
    # with fewer histories searched than the batch (without the flag: all)
    for j, (config, plant) in enumerate(EARLY_CASES):
        cat_st = np.array(results[0]["early"][j][0] + results[1]["early"][j][0], dtype=np.uint8)
        cat_nd = np.array(results[0]["early"][j][1] + results[1]["early"][j][1], dtype=np.uint64)
        st1, nd1, tot1 = results[0]["early"][j][3]
        assert np.array_equal(cat_st, np.array(st1, dtype=np.uint8)), config
        assert np.array_equal(cat_nd, np.array(nd1, dtype=np.uint64)), config
        assert qdist.totals_from_status(cat_st, cat_nd).tolist()[:8] == [
            tot1[k] for k in ("checked", "linearisable", "nonlinearisable", "model_errors", "encode_errors",
                              "budget", "skipped", "nodes")]
        ff = results[0]["early"][j][2]["first_fail"]
        assert ff == results[1]["early"][j][2]["first_fail"] < n_total
        searched = results[0]["early"][j][2]["searched"] + results[1]["early"][j][2]["searched"]
        assert ff + 1 <= searched < n_total, (config, plant, searched)
        # the device-resident path: status for status, count for count the same,
        # the same rounds and histories searched, the all-reduced totals the batch's
        dev_st = np.array(results[0]["early"][j][4][0] + results[1]["early"][j][4][0], dtype=np.uint8)
        dev_nd = np.array(results[0]["early"][j][4][1] + results[1]["early"][j][4][1], dtype=np.uint64)
        assert np.array_equal(dev_st, np.array(st1, dtype=np.uint8)), config
        assert np.array_equal(dev_nd, np.array(nd1, dtype=np.uint64)), config
        for r in range(world):
            dinfo, dtot = results[r]["early"][j][4][2], results[r]["early"][j][4][3]
            hinfo = results[r]["early"][j][2]
            assert (dinfo["first_fail"], dinfo["rounds"], dinfo["searched"]) == \
                (hinfo["first_fail"], hinfo["rounds"], hinfo["searched"]), (config, r)
            assert dtot == qdist.totals_from_status(dev_st, dev_nd).tolist()


def test_bench_two_ranks_on_one_gpu():
    """bench.py's multi-rank path as the driver launches it (torchrun, one
    process per rank), both ranks on cuda:0 (QSMD_BENCH_DEVICE=0): every
    step's totals summed on the device and exchanged once after the window
    (over gloo here: on one node of GPUs the default is RCCL).  bench.py asserts that the totals of
    all ranks cover n_hist x ranks x steps histories; here, the one JSON
    line of rank 0 and its whole-job figures."""
    import json
    import subprocess
    root = os.path.join(HERE, "..")
    # (RCCL refuses two ranks on one device: the rehearsal's totals go over gloo)
    env = dict(os.environ, QSMD_BENCH_DEVICE="0", QSMD_BENCH_COUNTERS="gloo", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "6", "--warmup", "2", "--n-hist", "20000", "--rotate", "3", "--no-extra",
           "--no-cpu-baseline", "--roof-calls", "2"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 6 and d["value"] > 0
    assert d["verdicts"]["checked"] + d["verdicts"]["budget"] <= 2 * 6 * 20000
    assert "gloo" in d["config"]["counters"] and d["config"]["exchange_ms"] is not None
    # the headline with the exchange inside: the same histories over the
    # window plus exchange_ms (MAX over the ranks of each)
    assert 0 < d["value_incl_exchange"] < d["value"]
    t_win = 2 * 6 * 20000 / d["value"]
    assert abs(2 * 6 * 20000 / d["value_incl_exchange"] - t_win - d["config"]["exchange_ms"] * 1e-3) \
        < 0.5 * t_win + 0.05


@pytest.mark.parametrize("n_total,plant,chunk,first_chunk", [
    (0, None, 4096, 64), (1, None, 4096, 64), (1, 0, 4096, 64), (5, 4, 2, 1), (3000, None, 1000, 4096),
    (3000, 2999, 512, 16), (3000, 0, 512, 16), (3000, 1500, 700, 100)])
def test_device_early_exit_one_rank(n_total, plant, chunk, first_chunk):
    """check_shard_early_exit_device without a process group (one rank): an
    empty batch, one history, a failure at either end or in the middle, no
    failure, a first chunk larger than the chunk; the statuses, counts and
    totals of one context's early exit over the batch, the rounds of the
    schedule up to the failure's chunk."""
    _paths()
    import torch

    import oracle_c
    from test_distributed import early_exit_reference, planted_stream
    from qsmd import device, gen
    from qsmd import dist as qdist

    config = "bank_4x16"
    mid = gen.CONFIGS[config]["model_id"]
    hdr, ev = planted_stream(config, max(n_total, 1), plant)
    if n_total == 0:
        hdr, ev = hdr[:0], ev[:0]
    ctx = device.Context(0)
    try:
        d_h = torch.from_numpy(np.ascontiguousarray(hdr).view(np.uint8)).cuda()
        d_e = torch.from_numpy(np.ascontiguousarray(ev).view(np.uint8)).cuda()
        st, nd, info = qdist.check_shard_early_exit_device(ctx, mid, d_h, d_e, len(ev), n_total, 0, 1, chunk=chunk,
                                                           max_nodes=10**7, first_chunk=first_chunk)
        torch.cuda.synchronize()
        st, nd = st.cpu().numpy(), nd.cpu().numpy().astype(np.uint64)
    finally:
        ctx.close()
    if n_total:
        st_full, nd_full, _ = oracle_c.check_batch(mid, hdr, ev, threads=4, max_nodes=10**7)
    else:
        st_full, nd_full = np.zeros(0, dtype=np.uint8), np.zeros(0, dtype=np.uint64)
    st_ref, nd_ref = early_exit_reference(np.asarray(st_full), np.asarray(nd_full))
    assert np.array_equal(st, st_ref) and np.array_equal(nd, nd_ref)
    assert info["totals"].tolist() == qdist.totals_from_status(st_ref, nd_ref).tolist()
    fails = np.nonzero((np.asarray(st_full) == 0) | (np.asarray(st_full) == 2))[0]
    ff = int(fails[0]) if len(fails) else n_total
    assert info["first_fail"] == ff
    sched = qdist.early_chunks(n_total, chunk, first_chunk)
    assert info["rounds"] == (next(i for i, (a, b) in enumerate(sched) if a <= ff < b) + 1 if ff < n_total
                              else len(sched))
