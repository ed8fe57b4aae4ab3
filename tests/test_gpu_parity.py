"""GPU parity: the HIP search (through the C ABI) against the oracle.

Bar: bit-exact verdicts, node counts and witness paths for every history
(integer search, no tolerance).  Oracles: the C restatement (oracle/ref_cpu.c),
itself pinned to the literal list transliteration and the KATs
(tests/test_oracle.py).
"""

import random

import numpy as np
import pytest

import histgen
import oracle_c
from kats import KATS
from qsmd import codec, gen, models
from qsmd.linearisability import linearisable, linearisable_batch, replay_witness

pytestmark = pytest.mark.gpu


def _compare(ctx, model_id, hdr, events, model0=None, max_nodes=0, threads=8, witness=True):
    st_d, nd_d, w_d, tot = ctx.check_arrays(model_id, hdr, events, model0, max_nodes=max_nodes,
                                            witness=witness)
    st_o, nd_o, w_o = oracle_c.check_batch(model_id, hdr, events, model0, max_nodes, threads,
                                           witness=witness)
    bad = np.nonzero((st_d != st_o) | (nd_d != nd_o))[0]
    assert len(bad) == 0, (f"{len(bad)} mismatches, first {bad[:5]}: "
                           f"dev {st_d[bad[:5]]}/{nd_d[bad[:5]]} oracle {st_o[bad[:5]]}/{nd_o[bad[:5]]}")
    if witness:
        lin = st_d == codec.STATUS_LIN
        for i in np.nonzero(lin)[0]:
            h = hdr[i]
            a, b = int(h["ev_off"]), int(h["ev_off"]) + int(h["n_ev"])
            assert np.array_equal(w_d[a:b], w_o[a:b]), f"witness mismatch at history {i}"
    assert tot["nodes"] == int(nd_d.sum())
    assert tot["linearisable"] == int((st_d == 1).sum())
    assert tot["nonlinearisable"] == int((st_d == 0).sum())
    assert tot["model_errors"] == int((st_d == 2).sum())
    assert tot["encode_errors"] == int((st_d == 3).sum())
    return st_d, nd_d, w_d


def test_kats_on_device(ctx):
    for name, (m, hist, status, nodes) in KATS.items():
        res = linearisable_batch(m, [hist], ctx=ctx, witness=True)
        assert res.verdict(0) == status, name
        assert int(res.nodes[0]) == nodes, name
        if status == "lin":
            assert replay_witness(m, hist, res.witness_of(0)), name


def test_linearisable_signature(ctx):
    """The reference signature: linearisable transition postcondition model0 history."""
    _, h2, _, _ = KATS["KAT2_reference_example"]
    _, h3, _, _ = KATS["KAT3_distinct_pids"]
    T = models.TICKET
    assert linearisable(T.transition, T.postcondition, T.init_model, h2, ctx=ctx) is False
    assert linearisable(T.transition, T.postcondition, T.init_model, h3, ctx=ctx) is True
    _, h8, _, _ = KATS["KAT8_bank_map_error"]
    B = models.BANK
    with pytest.raises(models.ModelError):
        linearisable(B.transition, B.postcondition, B.init_model, h8, ctx=ctx)
    with pytest.raises(NotImplementedError):
        linearisable(lambda m, e: m, lambda m, i, r: True, None, h3, ctx=ctx)


@pytest.mark.parametrize("model", ["ticket", "bank"])
def test_random_any_shape(ctx, model):
    """Ill-formed, shared-pid, pending and stray-response histories."""
    rng = random.Random(1234 if model == "ticket" else 4321)
    hs = []
    for _ in range(6000):
        if rng.random() < 0.5:
            hs.append(histgen.random_history(rng, model, rng.randint(0, 16), rng.randint(1, 5)))
        else:
            hs.append(histgen.wellformed_history(rng, model, rng.randint(0, 10), rng.randint(1, 5)))
    m = models.BY_NAME[model]
    b = codec.encode(m, hs)
    _compare(ctx, m.model_id, b.hdr, b.events, max_nodes=200000)


@pytest.mark.parametrize("n_ev,n_pid", [(40, 3), (64, 6), (96, 4), (128, 8), (60, 20), (128, 100)])
@pytest.mark.parametrize("stage0w", ["on", "off", "coop", "memo", "no_heavy"])
def test_stage_cascade(ctx, n_ev, n_pid, stage0w):
    """Histories beyond stage 0 (32 events / 8 pids) go through stage 0w
    (<= 64 events, <= 8 pids; over its node budget: coop64; off: straight to
    stage 1) and stages 1 and 2.  coop: a 4-node budget sends most of them to
    coop64; no_heavy (the default): stage 0w searches them to the end."""
    rng = random.Random(n_ev * 1000 + n_pid)
    ctx.set_param("stage0w", 0 if stage0w == "off" else 1)
    ctx.set_param("stage0w_budget", {"coop": 4, "memo": 4, "on": 32}.get(stage0w, 0))
    ctx.set_param("memo_stage", 0 if stage0w == "coop" else 1)
    try:
        for model in ("ticket", "bank"):
            hs = [histgen.wellformed_history(rng, model, n_ev // 2, n_pid, p_pending=0.0)[:n_ev]
                  for _ in range(300)]
            hs += [histgen.random_history(rng, model, n_ev, n_pid) for _ in range(300)]
            m = models.BY_NAME[model]
            b = codec.encode(m, hs)
            _compare(ctx, m.model_id, b.hdr, b.events, max_nodes=200000)
    finally:
        ctx.set_param("stage0w", 1)
        ctx.set_param("stage0w_budget", 32)
        ctx.set_param("memo_stage", 1)


@pytest.mark.parametrize("model,n_ev", [("bank", 32), ("bank", 20), ("ticket", 24), ("ticket", 7),
                                        ("bank", 48), ("ticket", 64), ("bank", 33)])
def test_packed_uniform_batches(ctx, model, n_ev):
    """Batches whose histories are packed back to back with one length take the
    coalesced staging path; corrupt some events (encode errors) and widen some
    values (deferral to stage 1) so every outcome goes through that path."""
    rng = random.Random(n_ev * 7 + len(model))
    m = models.BY_NAME[model]
    hs = []
    while len(hs) < 64 * 60:
        h = histgen.wellformed_history(rng, model, (n_ev + 1) // 2, rng.randint(1, 5), p_pending=0.0)
        if len(h) >= n_ev:
            hs.append(h[:n_ev])
    b = codec.encode(m, hs)
    ev = b.events.copy()
    nr = np.random.default_rng(n_ev)
    bad = nr.choice(len(ev), 40, replace=False)
    ev["code"][bad[:20]] = 9                                   # unknown constructor
    ev["val"][bad[20:]] = 1 << 20                              # > 19-bit: deferred
    for hdr in (b.hdr, b.hdr[1:]):                             # even and odd block start
        _compare(ctx, m.model_id, hdr, ev, max_nodes=200000)


def test_mixed_sizes_one_batch(ctx):
    rng = random.Random(7)
    hs = []
    for _ in range(3000):
        n = rng.choice([0, 1, 2, 8, 20, 32, 33, 50, 64, 65, 100, 128])
        hs.append(histgen.random_history(rng, "bank", n, rng.randint(1, 12)))
    b = codec.encode(models.BANK, hs)
    _compare(ctx, models.MODEL_BANK, b.hdr, b.events, max_nodes=100000)


@pytest.mark.parametrize("name,n", [("ticket_2x10", 20000), ("bank_4x16", 50000),
                                    ("bank_4x16_bugs", 50000), ("bank_6x24", 20000)])
@pytest.mark.parametrize("budget", [0, 24])
@pytest.mark.parametrize("kernel", [0, 1, 2])
def test_generated_configs(ctx, name, n, budget, kernel):
    """kernel 0: compact_search (2: with groups from a counter on a
    persistent grid); budget > 0: histories over the stage-0 node budget go
    to the heavy stages.  kernel 1: group_search (in-wave sharing; the budget
    does not apply)."""
    if kernel == 1 and budget:
        pytest.skip("group_search has no stage-0 budget")
    ctx.set_param("stage0_kernel", 1 if kernel == 1 else 0)
    ctx.set_param("stage0_dynamic", 1 if kernel == 2 else 0)
    if kernel == 2:
        ctx.set_param("stage0_grid", 97)
    ctx.set_stage0_budget(budget)
    try:
        hdr, ev, bug = gen.generate_config(name, 0, n)
        st, nd, _ = _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=10**7)
    finally:
        ctx.set_stage0_budget(0)
        ctx.set_param("stage0_auto", 1)
        ctx.set_param("stage0_kernel", 0)
        ctx.set_param("stage0_dynamic", 0)
        ctx.set_param("stage0_grid", 65536)
    if name in ("bank_4x16", "bank_6x24"):
        assert (st == codec.STATUS_LIN).all()


@pytest.mark.parametrize("name,n", [("ticket_2x10", 20000), ("bank_4x16", 50000), ("bank_4x16_bugs", 50000)])
@pytest.mark.parametrize("rerun,budget", [(16, 0), (3, 0), (16, 256), (5, 40)])
def test_rerun_stage(ctx, name, n, rerun, budget):
    """Stage 0r: stage 0 stops at `rerun` nodes and the histories over it are
    searched again from the root (packed, list mode), with the stage-0 heavy
    budget (and the caller's max_nodes: budget 40 < the heavy budget)."""
    ctx.set_param("rerun_budget", rerun)
    ctx.set_stage0_budget(budget)
    try:
        hdr, ev, _ = gen.generate_config(name, 3, n)
        _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=40 if rerun == 5 else 10**7)
    finally:
        ctx.set_param("rerun_budget", 0)
        ctx.set_stage0_budget(0)
        ctx.set_param("stage0_auto", 1)


MEMO_CASES = [("bank_4x16_bugs", 50000, 64, 0), ("bank_4x16_bugs", 20000, 8, 300), ("bank_4x16", 50000, 16, 0),
              ("ticket_2x10", 20000, 4, 0), ("bank_6x24", 20000, 16, 0), ("bank_6x24", 20000, 8, 500)]


@pytest.mark.parametrize("name,n,budget,max_nodes", MEMO_CASES)
@pytest.mark.parametrize("entries", [128, 2])
def test_memo_stage(ctx, name, n, budget, max_nodes, entries):
    """The memo stage (exact-count state memo): histories over the stage-0
    (stage-0w for 48 events) budget are searched with subtree counts reused
    from a per-lane table; verdicts, node counts and witnesses must equal the
    reference's.  2 entries: constant replacement; max_nodes: the budget
    falls inside reused subtrees."""
    ctx.set_param("memo_stage", 1)
    ctx.set_param("memo_lane_entries", entries)
    ctx.set_stage0_budget(budget)
    ctx.set_param("stage0w_budget", budget)
    try:
        hdr, ev, _ = gen.generate_config(name, 5, n)
        _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=max_nodes or 10**7)
    finally:
        ctx.set_param("memo_lane_entries", 128)
        ctx.set_stage0_budget(0)
        ctx.set_param("stage0_auto", 1)
        ctx.set_param("stage0w_budget", 32)
        ctx.set_param("stage0_auto", 1)


@pytest.mark.parametrize("name,n", [("bank_4x16", 50000), ("bank_4x16_bugs", 30000), ("ticket_2x10", 20000),
                                    ("bank_6x24", 20000)])
@pytest.mark.parametrize("cut_k,cut_min", [(2, 16), (8, 4), (63, 4)])
def test_straggler_cut(ctx, name, n, cut_k, cut_min):
    """Straggler cut: once a wavefront has run cut_min iterations with at most
    cut_k lanes still searching, those histories go to the memo stage and are
    searched again from the root (63: nearly every history is cut)."""
    ctx.set_param("cut_k", cut_k)
    ctx.set_param("cut_min", cut_min)
    try:
        hdr, ev, _ = gen.generate_config(name, 13, n)
        for _ in range(2):                       # the cascade's quiet mode, then its decision
            _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=10**7)
        _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=30)
    finally:
        ctx.set_param("cut_k", 0)
        ctx.set_param("cut_min", 16)


def test_memo_tables_too_large_fall_back_to_coop_spread(ctx):
    """Memo tables the device cannot hold switch the context to the coop /
    spread heavy stages: the same results."""
    ctx.set_param("memo_grid", 65536)
    ctx.set_param("memo_lane_entries", 65536)
    try:
        hdr, ev, _ = gen.generate_config("bank_4x16_bugs", 21, 20000)
        for _ in range(2):
            _compare(ctx, models.MODEL_BANK, hdr, ev)
    finally:
        ctx.set_param("memo_grid", 2048)
        ctx.set_param("memo_lane_entries", 256)
        ctx.set_param("memo_stage", 1)


@pytest.mark.parametrize("split_budget", [16, 200])
def test_memo_stage_handoff(ctx, split_budget):
    """Memo-stage searches that reach the giant cap (= split budget
    iterations) go to the split stage and are searched there from the root;
    also the default cascade outside heavy mode (stage 0 budget = split
    budget, then the memo stage)."""
    ctx.set_param("split_budget", split_budget)
    try:
        for name, n in (("bank_4x16_bugs", 30000), ("ticket_2x10", 20000), ("bank_6x24", 5000)):
            hdr, ev, _ = gen.generate_config(name, 9, n)
            ctx.set_param("stage0_auto", 0)
            ctx.set_param("stage0_budget", split_budget)
            _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=10**7)
            ctx.set_param("stage0_auto", 1)
            for _ in range(2):
                _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=10**7)
    finally:
        ctx.set_param("split_budget", 1024)
        ctx.set_param("stage0_auto", 1)


@pytest.mark.parametrize("model", ["ticket", "bank"])
def test_memo_stage_any_shape(ctx, model):
    """Unpaired, shared-pid and pending histories (the general DFS mode) and a
    non-default model0 through the memo stage."""
    rng = random.Random(77 if model == "ticket" else 78)
    hs = []
    for _ in range(4000):
        if rng.random() < 0.5:
            hs.append(histgen.random_history(rng, model, rng.randint(8, 32), rng.randint(1, 5)))
        else:
            hs.append(histgen.wellformed_history(rng, model, rng.randint(6, 16), rng.randint(1, 5)))
    m = models.BY_NAME[model]
    ctx.set_param("memo_stage", 1)
    ctx.set_stage0_budget(4)
    try:
        b = codec.encode(m, hs)
        _compare(ctx, m.model_id, b.hdr, b.events, max_nodes=200000)
        if model == "ticket":
            _compare(ctx, m.model_id, b.hdr, b.events, models.TicketModel(1, 0, 3), max_nodes=200000)
    finally:
        ctx.set_stage0_budget(0)
        ctx.set_param("stage0_auto", 1)


def test_concurrent_contexts_on_streams(ctx):
    """bench.py keeps several calls in flight: one context and stream each,
    running at the same time on one GPU.  Every call's results must be the
    oracle's (contexts share no device state)."""
    torch = pytest.importorskip("torch")
    from qsmd import device
    dev = torch.device("cuda:0")
    batches = [gen.generate_config(name, 31, n) for name, n in
               (("bank_4x16_bugs", 20000), ("bank_4x16", 40000), ("bank_6x24", 8000))]
    ctxs = [ctx, device.Context(0), device.Context(0)]
    streams = [torch.cuda.Stream(dev) for _ in ctxs]
    try:
        bufs = []
        for (hdr, ev, _), c, s in zip(batches, ctxs, streams):
            n = len(hdr)
            b = (torch.from_numpy(hdr.view(np.uint8)).to(dev), torch.from_numpy(ev.view(np.uint8)).to(dev),
                 torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int64, device=dev))
            bufs.append(b)
        torch.cuda.synchronize()
        for _ in range(3):                     # the cascade's quiet mode, then its decision
            for (hdr, ev, _), c, s, b in zip(batches, ctxs, streams, bufs):
                c.check_device(models.MODEL_BANK, b[0].data_ptr(), len(hdr), b[1].data_ptr(), len(ev),
                               b[2].data_ptr(), b[3].data_ptr(), None, None, stream=s.cuda_stream)
        torch.cuda.synchronize()
        for (hdr, ev, _), b in zip(batches, bufs):
            st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, hdr, ev, None, 0, 8, witness=False)
            assert np.array_equal(b[2].cpu().numpy(), st_o)
            assert np.array_equal(b[3].cpu().numpy().astype(np.uint64), nd_o.astype(np.uint64))
    finally:
        for c in ctxs[1:]:
            c.close()


def test_model0(ctx):
    rng = random.Random(99)
    hs = [histgen.wellformed_history(rng, "ticket", rng.randint(1, 6), 2) for _ in range(2000)]
    b = codec.encode(models.TICKET, hs)
    for n0 in (0, 5, -3):
        _compare(ctx, models.MODEL_TICKET, b.hdr, b.events, models.TicketModel(1, 0, n0))
    accts = ["p0", "p1", "p2"]
    model0 = {"p0": 10, "p1": 0, "p2": 3}
    hs = [histgen.wellformed_history(rng, "bank", rng.randint(1, 6), 3) for _ in range(2000)]
    b = codec.encode(models.BANK, hs, model0)
    packed = models.BANK.pack_model0(model0, models.BANK.new_account_map(model0))
    assert packed.exists == 0b111 and list(packed.balance)[:3] == [10, 0, 3]
    _compare(ctx, models.MODEL_BANK, b.hdr, b.events, packed)
    del accts


def test_budget(ctx):
    """The caller's max_nodes through every stage: stage-0 budgets 0/5/50
    (heavy stages), and for 33..64 events stage 0w's budget (32, the default:
    the memo stage; 4 without the memo stage: coop64 with its exploration cap)."""
    rng = random.Random(5)
    for n_ev in (40, 24):
        hs = [histgen.random_history(rng, "ticket", n_ev, 1) for _ in range(500)]
        b = codec.encode(models.TICKET, hs)
        for stage0, w_budget, memo in ((0, 0, 1), (5, 0, 1), (50, 0, 0), (0, 4, 0), (0, 4, 1), (0, 256, 1)):
            ctx.set_stage0_budget(stage0)
            ctx.set_param("stage0w_budget", w_budget)
            ctx.set_param("memo_stage", memo)
            try:
                for budget in (1, 7, 100, 1000):
                    st, nd, _ = _compare(ctx, models.MODEL_TICKET, b.hdr, b.events, max_nodes=budget)
                    assert (nd <= budget).all()
            finally:
                ctx.set_stage0_budget(0)
                ctx.set_param("stage0_auto", 1)
                ctx.set_param("stage0w_budget", 32)
                ctx.set_param("memo_stage", 1)


@pytest.mark.parametrize("name,shift", [("bank_4x16_bugs", 0), ("bank_4x16_bugs", 3000),
                                        ("bank_6x24", 0), ("bank_4x16", 0)])
def test_early_exit_batch(ctx, name, shift):
    """QSMD_FLAG_EARLY_EXIT_BATCH: like QuickCheck stopping at the first
    failing test, everything after the first non-linearisable (or raising)
    history is SKIPPED; everything up to it is exactly the full result."""
    from qsmd import device
    hdr, ev, _ = gen.generate_config(name, shift, 8000)
    mid = gen.CONFIGS[name]["model_id"]
    if name == "bank_6x24":                      # plant one failure deep in the batch
        ev = ev.copy()
        k = int(hdr[5000]["ev_off"]) + 47
        ev["val"][k] += 1 if ev["code"][k] == 7 else 0
        ev["code"][k] = 7 if ev["code"][k] != 7 else 7
    st_o, nd_o, _ = oracle_c.check_batch(mid, hdr, ev, threads=8, max_nodes=10**7)
    fails = np.nonzero((st_o == 0) | (st_o == 2))[0]
    cut = int(fails[0]) if len(fails) else len(hdr)
    ctx.set_stage0_budget(32 if shift else 0)
    try:
        st, nd, _, tot = ctx.check_arrays(mid, hdr, ev, flags=device.QSMD_FLAG_EXHAUSTIVE |
                                          device.QSMD_FLAG_EARLY_EXIT_BATCH, max_nodes=10**7)
    finally:
        ctx.set_stage0_budget(0)
        ctx.set_param("stage0_auto", 1)
    assert np.array_equal(st[:cut + 1], st_o[:cut + 1]) and np.array_equal(nd[:cut + 1], nd_o[:cut + 1])
    assert (st[cut + 1:] == codec.STATUS_SKIPPED).all() and (nd[cut + 1:] == 0).all()
    assert tot["skipped"] == max(0, len(hdr) - cut - 1)
    assert tot["nodes"] == int(nd_o[:cut + 1].sum())
    assert tot["checked"] == int(((st_o[:cut + 1] <= 2)).sum())


def test_encode_errors(ctx):
    hdr = np.zeros(5, dtype=codec.HDR_DTYPE)
    ev = np.zeros(8, dtype=codec.EV_DTYPE)
    hdr[0] = (0, 2, 1, 0xFF, 0, 0)            # wrong model
    hdr[1] = (0, 2, 0, 2, 0, 0)               # pid >= n_pid
    hdr[2] = (0, 200, 1, 2, 0, 0)             # too many events / beyond buffer
    hdr[3] = (6, 2, 1, 2, 0, 0)               # ok shape; bad code below
    hdr[4] = (4, 2, 1, 2, 0, 0)               # valid: Open a / Created
    ev[4] = (0, 0, 0, 0, 0)
    ev[5] = (0x80, 0, 0, 0, 0)
    ev[6] = (0, 9, 0, 0, 0)                   # unknown Bank request
    ev[7] = (0x80, 0, 0, 0, 0)
    st, nd, _, tot = ctx.check_arrays(models.MODEL_BANK, hdr, ev)
    assert list(st) == [3, 3, 3, 3, 1]
    assert tot["encode_errors"] == 4


def test_device_resident_full_size(ctx):
    """BASELINE config 2 at full size (1M histories) through the device entry
    point; size-independent properties (all linearisable by construction,
    totals == sums) plus an exact oracle comparison on a sample."""
    torch = pytest.importorskip("torch")
    n = 1_000_000
    hdr, ev, bug = gen.generate_config("bank_4x16", 0, n)
    dev = torch.device("cuda:0")
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.check_device(models.MODEL_BANK, d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                     d_st.data_ptr(), d_nd.data_ptr(), None, d_tot.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    nd = d_nd.cpu().numpy().astype(np.uint64)
    tot = d_tot.cpu().numpy()
    assert (st == codec.STATUS_LIN).all()
    assert int(tot[0]) == n and int(tot[1]) == n and int(tot[7]) == int(nd.sum())
    assert (nd >= 16).all()
    idx = np.arange(0, n, 50)
    st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, hdr[idx], ev, threads=8)
    assert np.array_equal(st_o, st[idx]) and np.array_equal(nd_o, nd[idx])


@pytest.mark.parametrize("packed", [True, False])
def test_value_ranges_and_pairing(ctx, packed):
    """Stage 0 holds invocation values within 14-bit signed and response
    values within 25-bit signed; anything wider goes to stage 1.  Put values
    on both sides of both bounds into generated Bank histories (packed
    uniform batch and a non-uniform one), and mix paired (every pid
    alternates) with unpaired histories inside one wavefront."""
    hdr, ev, _ = gen.generate_config("bank_4x16_bugs", 7, 64 * 40)
    ev = ev.copy()
    nr = np.random.default_rng(11)
    inv = np.nonzero((ev["kp"] & 0x80) == 0)[0]
    rsp = np.nonzero(((ev["kp"] & 0x80) != 0) & (ev["code"] == 7))[0]        # Balance responses
    iv = np.array([8191, 8192, -8192, -8193, 1 << 20, -(1 << 30)], dtype=np.int32)
    rv = np.array([(1 << 24) - 1, 1 << 24, -(1 << 24), -(1 << 24) - 1, 1 << 30], dtype=np.int32)
    ki = nr.choice(inv, 300, replace=False)
    kr = nr.choice(rsp, 300, replace=False)
    ev["val"][ki] = iv[nr.integers(0, len(iv), len(ki))]
    ev["val"][kr] = rv[nr.integers(0, len(rv), len(kr))]
    # unpaired: give a few histories a second invocation of the same pid
    # before its response (and a stray response) by swapping two events
    for h in nr.choice(len(hdr), 200, replace=False):
        o = int(hdr[h]["ev_off"])
        i = o + int(nr.integers(4, 30))
        ev[[i, i + 1]] = ev[[i + 1, i]]
    if not packed:
        hdr = hdr[nr.permutation(len(hdr))]
    _compare(ctx, models.MODEL_BANK, hdr, ev, max_nodes=10**6)


HEAVY_DEFAULTS = {"memo_stage": 0, "stage0_budget": 0, "heavy_stage": 2, "coop_budget": 16, "spread_budget": 128,
                  "spread_cap": 1 << 22, "coop_max": 4096, "stage0_kernel": 0, "group_budget": 16,
                  "share_idle": 16, "share_nodes": 32}


def _heavy(ctx, **kw):
    for k, v in {**HEAVY_DEFAULTS, **kw}.items():
        ctx.set_param(k, v)


@pytest.mark.parametrize("name,n", [("bank_4x16_bugs", 20000), ("bank_4x16", 20000), ("ticket_2x10", 20000)])
@pytest.mark.parametrize("stage,task_budget,cap", [("coop", 1, 0), ("coop", 4, 0), ("coop", 64, 0),
                                                   ("spread", 4, 1 << 22), ("spread", 128, 1 << 22),
                                                   ("spread", 8, 1024), ("auto-coop", 16, 0),
                                                   ("auto-spread", 64, 1 << 22), ("group", 1, 0),
                                                   ("group", 4, 0), ("group", 16, 0), ("group", 64, 0)])
def test_heavy_stage(ctx, name, n, stage, task_budget, cap):
    """The stages for the histories over the stage-0 node budget: coop (one
    wavefront per history, csrc/coop.hip) and spread (global dynamic split,
    csrc/spread.hip).  Tiny task budgets force deep split trees; a tiny
    spread capacity forces its 'no room: search on' path.  Verdicts, node
    counts and witnesses must be exactly the single DFS's."""
    hdr, ev, _ = gen.generate_config(name, 3, n)
    if stage == "coop":
        _heavy(ctx, stage0_kernel=0, stage0_budget=8, heavy_stage=0, coop_budget=task_budget)
    elif stage == "spread":
        _heavy(ctx, stage0_kernel=0, stage0_budget=8, heavy_stage=1, spread_budget=task_budget, spread_cap=cap)
    elif stage == "group":
        _heavy(ctx, stage0_kernel=1, group_budget=task_budget, share_idle=1 + task_budget % 7, share_nodes=2)
    else:                                        # auto: the count decides (1 history -> spread)
        _heavy(ctx, stage0_kernel=0, stage0_budget=8, heavy_stage=2, coop_budget=task_budget,
               spread_budget=task_budget, coop_max=1 << 20 if stage == "auto-coop" else 0)
    try:
        _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev)
    finally:
        _heavy(ctx, memo_stage=1)


@pytest.mark.parametrize("model", ["ticket", "bank"])
@pytest.mark.parametrize("stage", ["coop", "spread", "group"])
def test_heavy_any_shape(ctx, model, stage):
    """Shared pids, pending invocations, stray responses, Map.! errors and
    node budgets through the heavy stages (general, unpaired search)."""
    rng = random.Random(77 if model == "ticket" else 78)
    hs = []
    for _ in range(4000):
        if rng.random() < 0.5:
            hs.append(histgen.random_history(rng, model, rng.randint(8, 32), rng.randint(1, 3)))
        else:
            hs.append(histgen.wellformed_history(rng, model, rng.randint(6, 16), rng.randint(2, 6)))
    m = models.BY_NAME[model]
    b = codec.encode(m, hs)
    if stage == "coop":
        _heavy(ctx, stage0_kernel=0, stage0_budget=4, heavy_stage=0, coop_budget=2)
    elif stage == "spread":
        _heavy(ctx, stage0_kernel=0, stage0_budget=4, heavy_stage=1, spread_budget=6)
    else:
        _heavy(ctx, stage0_kernel=1, group_budget=3, share_idle=2, share_nodes=3)
    try:
        for max_nodes in (0, 50, 3000):
            _compare(ctx, m.model_id, b.hdr, b.events, max_nodes=max_nodes)
    finally:
        _heavy(ctx, memo_stage=1)


def test_adaptive_cascade(ctx):
    """The default adaptive cascade: a call's probe (histories needing more
    than 256 nodes) decides whether later calls run stage 0 with a node budget
    and the heavy stages.  Results are exact in both modes and across the
    switches (bug-heavy batch, then a clean one, then the bug-heavy again)."""
    ctx.set_param("stage0_auto", 1)
    try:
        b3 = gen.generate_config("bank_4x16_bugs", 11, 30000)
        b2 = gen.generate_config("bank_4x16", 11, 30000)
        for hdr, ev, _ in (b3, b3, b3, b2, b2, b3):
            _compare(ctx, models.MODEL_BANK, hdr, ev)
    finally:
        ctx.set_stage0_budget(0)
        ctx.set_param("stage0_auto", 1)
