"""GPU parity of the split stage (csrc/split.hip) and of QSMD_FLAG_MEMO.

The split stage must be invisible in exhaustive mode: a history searched by
many lanes (frontier -> tasks -> ordered combine) has exactly the verdict,
node count and witness of the single reference DFS (oracle/ref_cpu.c).  The
split budget is lowered so that most histories take that path.  With MEMO,
verdicts and witnesses are exact and node counts never exceed the
exhaustive ones.
"""

import contextlib
import ctypes
import random

import numpy as np
import pytest

import histgen
import oracle_c
from qsmd import codec, device, gen, models
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu

DEFAULT_SPLIT = 1024
EXH = device.QSMD_FLAG_EXHAUSTIVE
MEMO = device.QSMD_FLAG_MEMO


@contextlib.contextmanager
def knobs(ctx, split=None, stage0=None):
    try:
        if split is not None:
            ctx.set_split_budget(split)
        if stage0 is not None:
            ctx.set_stage0_budget(stage0)
        yield
    finally:
        ctx.set_split_budget(DEFAULT_SPLIT)
        ctx.set_stage0_budget(32)


@pytest.mark.parametrize("split", [1, 16, 200])
@pytest.mark.parametrize("name,n", [("bank_4x16_bugs", 20000), ("bank_6x24", 4000), ("ticket_2x10", 5000)])
def test_split_generated(ctx, name, n, split):
    hdr, ev, _ = gen.generate_config(name, 0, n)
    with knobs(ctx, split=split):
        _compare(ctx, gen.CONFIGS[name]["model_id"], hdr, ev, max_nodes=10**7)


@pytest.mark.parametrize("model", ["ticket", "bank"])
def test_split_random_shapes(ctx, model):
    """Both variants (<= 64 events / 8 pids and <= 128 events / 128 pids),
    ill-formed, shared-pid and pending histories."""
    rng = random.Random(77 if model == "ticket" else 78)
    hs = []
    for _ in range(3000):
        n = rng.choice([4, 12, 20, 32, 40, 64, 90, 128])
        if rng.random() < 0.5:
            hs.append(histgen.random_history(rng, model, n, rng.randint(1, 12)))
        else:
            hs.append(histgen.wellformed_history(rng, model, n // 2, rng.randint(1, 12))[:n])
    m = models.BY_NAME[model]
    b = codec.encode(m, hs)
    with knobs(ctx, split=8):
        _compare(ctx, m.model_id, b.hdr, b.events, max_nodes=200000)


def test_split_after_heavy_stage(ctx):
    hdr, ev, _ = gen.generate_config("bank_4x16_bugs", 1000, 20000)
    with knobs(ctx, split=64, stage0=8):
        _compare(ctx, models.MODEL_BANK, hdr, ev, max_nodes=10**7)


def test_split_node_limits(ctx):
    """max_nodes across the cut: BUDGET exactly where the single DFS stops."""
    rng = random.Random(5)
    hs = [histgen.random_history(rng, "ticket", 40, 1) for _ in range(400)]
    hs += [histgen.random_history(rng, "ticket", 24, 2) for _ in range(400)]
    b = codec.encode(models.TICKET, hs)
    with knobs(ctx, split=2):
        for budget in (3, 7, 100, 5000):
            st, nd, _ = _compare(ctx, models.MODEL_TICKET, b.hdr, b.events, max_nodes=budget)
            assert (nd <= budget).all()


def test_split_early_exit(ctx):
    hdr, ev, _ = gen.generate_config("bank_4x16_bugs", 0, 8000)
    st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, hdr, ev, threads=8, max_nodes=10**7)
    fails = np.nonzero((st_o == 0) | (st_o == 2))[0]
    cut = int(fails[0])
    with knobs(ctx, split=4):
        st, nd, _, tot = ctx.check_arrays(models.MODEL_BANK, hdr, ev, max_nodes=10**7,
                                          flags=EXH | device.QSMD_FLAG_EARLY_EXIT_BATCH)
    assert np.array_equal(st[:cut + 1], st_o[:cut + 1]) and np.array_equal(nd[:cut + 1], nd_o[:cut + 1])
    assert (st[cut + 1:] == codec.STATUS_SKIPPED).all()
    assert tot["nodes"] == int(nd_o[:cut + 1].sum())


def _heavy(name, n, k):
    hdr, ev, _ = gen.generate_config(name, 0, n)
    st, nd, _ = oracle_c.check_batch(gen.CONFIGS[name]["model_id"], hdr, ev, threads=8, max_nodes=10**7)
    order = np.argsort(-nd.astype(np.int64))[:k]
    return hdr, ev, order


def _one(hdr, ev, i):
    h = hdr[i:i + 1].copy()
    a, n = int(h[0]["ev_off"]), int(h[0]["n_ev"])
    h[0]["ev_off"] = 0
    return h, ev[a:a + n].copy()


@pytest.mark.parametrize("name", ["bank_4x16_bugs", "bank_6x24"])
def test_split_api_single_history(ctx, name):
    """qsmd_split_frontier + qsmd_check_tasks + qsmd_combine_tasks == the
    single search, for any task count, and for tasks spread round-robin
    over several callers (the multi-GPU split)."""
    mid = gen.CONFIGS[name]["model_id"]
    hdr, ev, order = _heavy(name, 4000, 12)
    for i in order:
        h, e = _one(hdr, ev, int(i))
        st_o, nd_o, w_o = oracle_c.check_batch(mid, h, e, witness=True)
        for min_tasks in (1, 16, 300):
            fr, tasks, w_top = ctx.split_frontier(mid, h, e, min_tasks=min_tasks, witness=True)
            assert fr.status in (0, 1, 2)
            for ranks in (1, 3):
                st = np.zeros(len(tasks), dtype=np.uint8)
                nd = np.zeros(len(tasks), dtype=np.uint64)
                wit = np.full((len(tasks), 64), 0xFF, dtype=np.uint8)
                for r in range(ranks):
                    sub = tasks[r::ranks]
                    s, n_, w = ctx.check_tasks(mid, h, e, sub, witness=True)
                    st[r::ranks], nd[r::ranks], wit[r::ranks] = s, n_, w
                # tasks a caller skipped lie after one it found deciding
                status, nodes, win = device.combine_tasks(fr, tasks, st, nd)
                assert (status, nodes) == (int(st_o[0]), int(nd_o[0])), (i, min_tasks, ranks)
                if status == codec.STATUS_LIN:
                    path = wit[win] if win >= 0 else w_top
                    d = int(np.argmax(np.append(path, 0xFF) == 0xFF))
                    od = int(np.argmax(np.append(w_o, 0xFF) == 0xFF))
                    assert d == od and np.array_equal(path[:d], w_o[:od])


def test_split_api_edge_cases(ctx):
    # empty history: decided above the cut (True, no tasks)
    h = np.zeros(1, dtype=codec.HDR_DTYPE)
    h[0] = (0, 0, 0, models.MODEL_BANK, 0, 0)
    fr, tasks, _ = ctx.split_frontier(models.MODEL_BANK, h, np.zeros(0, dtype=codec.EV_DTYPE))
    assert fr.status == codec.STATUS_LIN and len(tasks) == 0
    # max_tasks = 1: the deepest cut with a single task (or, when even the
    # root has more children, the whole search done by the frontier itself)
    hdr, ev, order = _heavy("bank_4x16_bugs", 2000, 1)
    h, e = _one(hdr, ev, int(order[0]))
    st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, h, e)
    for m0 in (None, models.BankModel(0b1111, 0, (ctypes.c_int64 * 8)(5, 5, 5, 5, 0, 0, 0, 0))):
        st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, h, e, m0)
        fr, tasks, _ = ctx.split_frontier(models.MODEL_BANK, h, e, m0, min_tasks=10**6, max_tasks=1)
        assert len(tasks) <= 1
        st, nd, _ = ctx.check_tasks(models.MODEL_BANK, h, e, tasks, m0)
        assert device.combine_tasks(fr, tasks, st, nd)[:2] == (int(st_o[0]), int(nd_o[0]))
    from kats import L, R
    rng = random.Random(11)
    fallback = 0
    # three concurrent OpenAccounts at the root: more root children than max_tasks
    opens = [(p, L(("OpenAccount", p))) for p in "abc"] + [(p, R("AccountCreated")) for p in "abc"]
    hists = [opens, opens + [("a", L(("CheckBalance", "a"))), ("a", R(("Balance", 1)))]]
    hists += [histgen.random_history(rng, "bank", rng.randint(6, 30), rng.randint(2, 5)) for _ in range(200)]
    for hist in hists:
        b = codec.encode(models.BANK, [hist])
        if b.encode_errors:
            continue
        st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, b.hdr, b.events)
        fr, tasks, _ = ctx.split_frontier(models.MODEL_BANK, b.hdr, b.events, min_tasks=8, max_tasks=1)
        fallback += fr.n_tasks == 0 and fr.depth == 0
        st, nd, _ = ctx.check_tasks(models.MODEL_BANK, b.hdr, b.events, tasks)
        assert device.combine_tasks(fr, tasks, st, nd)[:2] == (int(st_o[0]), int(nd_o[0]))
    assert fallback > 0
    # node limit across the cut
    fr, tasks, _ = ctx.split_frontier(models.MODEL_BANK, h, e, min_tasks=64, max_nodes=50)
    st, nd, _ = ctx.check_tasks(models.MODEL_BANK, h, e, tasks, max_nodes=50)
    st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_BANK, h, e, max_nodes=50)
    assert device.combine_tasks(fr, tasks, st, nd, max_nodes=50)[:2] == (int(st_o[0]), int(nd_o[0]))


@pytest.mark.parametrize("name", ["bank_4x16_bugs", "ticket_2x10"])
def test_memo_verdicts(ctx, name):
    hdr, ev, _ = gen.generate_config(name, 0, 20000)
    mid = gen.CONFIGS[name]["model_id"]
    st_o, nd_o, w_o = oracle_c.check_batch(mid, hdr, ev, threads=8, witness=True, max_nodes=10**7)
    with knobs(ctx, split=16):
        st, nd, w, tot = ctx.check_arrays(mid, hdr, ev, flags=EXH | MEMO, witness=True, max_nodes=10**7)
    assert np.array_equal(st, st_o)
    assert (nd <= nd_o).all()
    for i in np.nonzero(st == codec.STATUS_LIN)[0]:
        a, b = int(hdr[i]["ev_off"]), int(hdr[i]["ev_off"]) + int(hdr[i]["n_ev"])
        assert np.array_equal(w[a:b], w_o[a:b]), i


def test_adversarial_ticket_exhaustive_split(ctx):
    """4 clients x 17 ops with one bug: 923201 reference nodes, searched by
    the split stage with the exact count."""
    h, e, _ = gen.adversarial_ticket(4, 17, bug=True)
    st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_TICKET, h, e)
    assert (int(st_o[0]), int(nd_o[0])) == (codec.STATUS_NONLIN, 923201)
    st, nd, _, _ = ctx.check_arrays(models.MODEL_TICKET, h, e)
    assert (int(st[0]), int(nd[0])) == (codec.STATUS_NONLIN, 923201)


@pytest.mark.parametrize("bug", [True, False])
def test_adversarial_ticket_memo(ctx, bug):
    """BASELINE config 4: 8 clients x 64 ops, shared pid, heavy overlap;
    (8!)^7 paths without memo, a few hundred states with it.  Memo mode's
    node count is the pruning DFS's explored count (oracle/ref_cpu.c: each
    state's children evaluated once): equal to the oracle's (281 with the
    bug)."""
    h, e, _ = gen.adversarial_ticket(8, 64, bug=bug)
    st_o, nd_o, w_o = oracle_c.check_batch(models.MODEL_TICKET, h, e, memo=True, witness=True)
    st, nd, w, _ = ctx.check_arrays(models.MODEL_TICKET, h, e, flags=EXH | MEMO, witness=True)
    assert int(st[0]) == int(st_o[0]) == (codec.STATUS_NONLIN if bug else codec.STATUS_LIN)
    assert int(nd[0]) == int(nd_o[0]), (int(nd[0]), int(nd_o[0]))
    if bug:
        assert int(nd[0]) == 281
    if not bug:
        assert np.array_equal(w, w_o)


@pytest.mark.parametrize("nc,no,status,nodes", [(6, 30, codec.STATUS_NONLIN, 88071120488677),
                                                (4, 17, codec.STATUS_NONLIN, 923201),
                                                (8, 40, codec.STATUS_BUDGET, None)])
def test_adversarial_exhaustive_exact_memo(ctx, nc, no, status, nodes):
    """Exhaustive mode (no QSMD_FLAG_MEMO): the split stage's exact-count memo
    reports the reference's node count of adversarial histories no plain
    search could count (pinned by the memoised transliteration,
    tests/test_oracle.py); a count beyond 2^64 - 1 is a budget."""
    h, e, _ = gen.adversarial_ticket(nc, no, bug=True)
    st, nd, _, _ = ctx.check_arrays(models.MODEL_TICKET, h, e)
    assert int(st[0]) == status
    if nodes is not None:
        assert int(nd[0]) == nodes


@pytest.mark.parametrize("xmemo", [1, 0])
@pytest.mark.parametrize("split", [64, 4096])
def test_ticket_8x64_batch(ctx, xmemo, split):
    """Batches of 8-client x 64-op TicketDispenser histories (128 events:
    straight to the giant stage, most decided by its whole search, a heavy
    tail split into tasks), with and without the giant stage's exact memo:
    the reference's verdicts, counts and witnesses."""
    hdr, ev, _ = gen.generate_config("ticket_8x64", 0, 1500 if xmemo else 400)
    ctx.set_param("split_xmemo", xmemo)
    try:
        with knobs(ctx, split=split):
            _compare(ctx, models.MODEL_TICKET, hdr, ev, max_nodes=10**7)
    finally:
        ctx.set_param("split_xmemo", 1)


def test_time_limit_is_reported(ctx):
    """The safety net (qsmd_set_time_limit_ms) is told apart from max_nodes:
    an adversarial 6 x 30 history without the exact memo (8.8e13 reference
    nodes) cannot finish in 20 ms, so the call reports BUDGET and
    qsmd_timed_out says the time limit fired; the next call, under the
    default limit, finishes and says it did not.  (The state DAG counts that
    history exactly in microseconds -- test_dag_counts_what_the_dfs_cannot --
    so it is off here: the DFS and the split stage run into the limit.)"""
    h, e, _ = gen.adversarial_ticket(6, 30, bug=True)
    ctx.set_param("split_xmemo", 0)
    ctx.set_param("dag_states", 0)
    ctx.set_time_limit_ms(20)
    try:
        st, _, _, _ = ctx.check_arrays(models.MODEL_TICKET, h, e)
        assert int(st[0]) == codec.STATUS_BUDGET
        assert ctx.timed_out()
    finally:
        ctx.set_time_limit_ms(60000)
        ctx.set_param("split_xmemo", 1)
        ctx.set_param("dag_states", 128)
    h2, e2, _ = gen.adversarial_ticket(4, 17, bug=True)
    st, nd, _, _ = ctx.check_arrays(models.MODEL_TICKET, h2, e2)
    assert (int(st[0]), int(nd[0])) == (codec.STATUS_NONLIN, 923201)
    assert not ctx.timed_out()


@pytest.mark.parametrize("nc,no,status,nodes", [(6, 30, codec.STATUS_NONLIN, 88071120488677),
                                                (4, 17, codec.STATUS_NONLIN, 923201),
                                                (8, 40, codec.STATUS_BUDGET, 2**64 - 1)])
def test_dag_counts_what_the_dfs_cannot(ctx, nc, no, status, nodes):
    """The state DAG (wave mode) folds a shared-pid adversarial history's
    (nc!)^k-path tree into a chain of a few dozen states: the exact
    reference count (pinned by the memoised transliteration,
    tests/test_oracle.py; 8 x 40: 3.6e22, beyond 2^64 - 1: BUDGET) without
    the giant stage's exact memo, and the giant stage's result with it."""
    h, e, _ = gen.adversarial_ticket(nc, no, bug=True)
    ctx.set_param("split_xmemo", 0)
    try:
        st, nd, _, _ = ctx.check_arrays(models.MODEL_TICKET, h, e)
    finally:
        ctx.set_param("split_xmemo", 1)
    assert not ctx.timed_out()
    assert (int(st[0]), int(nd[0])) == (status, nodes)
    ctx.set_param("dag_states", 0)                  # the DFS, then the giant stage's exact memo
    try:
        st2, nd2, _, _ = ctx.check_arrays(models.MODEL_TICKET, h, e)
    finally:
        ctx.set_param("dag_states", 128)
    assert (int(st2[0]), int(nd2[0])) == (status, nodes)


def test_stalled_giant_workgroup_reports_budget(ctx):
    """The giant stage's phase waits give up after twice the time limit
    (wait_for's safety net).  A workgroup that gave up may meet frontier
    records and task results another workgroup has not finished (one that
    started late), or that an earlier call left in the reused workspace: the
    giants it combines are BUDGET, never a stale verdict.  Forced here with
    the diagnostic stall of the first frontier chunk's workgroup."""
    hdr, ev, _ = gen.generate_config("ticket_8x64", 0, 400)
    first = (hdr[:200].copy(), ev)
    second = (hdr[200:].copy(), ev)
    st_o, nd_o, _ = oracle_c.check_batch(models.MODEL_TICKET, second[0], second[1], threads=8, max_nodes=10**7)
    ctx.set_param("heavy_mode", 1)          # (lane mode sends every 128-event history to the giant stage)
    try:
        ctx.check_arrays(models.MODEL_TICKET, *first, max_nodes=10**7)      # records of another batch
        ctx.set_time_limit_ms(5)
        ctx.set_param("giant_stall_us", 100000)
        st, nd, _, tot = ctx.check_arrays(models.MODEL_TICKET, *second, max_nodes=10**7)
        assert ctx.timed_out()
    finally:
        ctx.set_param("giant_stall_us", 0)
        ctx.set_time_limit_ms(60000)
        ctx.set_param("heavy_mode", 2)
    budget = st == codec.STATUS_BUDGET
    assert budget.sum() > 0
    ok = ~budget
    assert np.array_equal(st[ok], st_o[ok]) and np.array_equal(nd[ok], nd_o[ok])
    assert tot["budget"] == int(budget.sum())
    # the context is sound afterwards
    _compare(ctx, models.MODEL_TICKET, second[0], second[1], max_nodes=10**7)


def _ticket_chain_like(rng, n_ops, width, n_pid, p_reset=0.1, p_bug=0.3):
    """Config-4-shaped TicketDispenser histories: a Reset, then batches of up
    to `width` pending invocations answered in order (responses numbered as a
    sequential run would), over `n_pid` pids (1: the shared pid of
    test/TicketDispenser.hs:302-309); sometimes a Reset among them or one
    response off by one.  Most are chains of one state per level (the wave
    stage's chain path); a Reset beside a TakeTicket gives two successors."""
    pids = [f"p{i}" for i in range(n_pid)]
    h = [("p0", ("L", "Reset")), ("p0", ("R", "Ok"))]
    n, left = 0, n_ops - 1
    while left > 0:
        w = min(rng.randint(1, width), left)
        ops = ["Reset" if rng.random() < p_reset else "TakeTicket" for _ in range(w)]
        who = [pids[(k + rng.randint(0, n_pid - 1)) % n_pid] if n_pid > 1 else "p0" for k in range(w)]
        h += [(who[k], ("L", ops[k])) for k in range(w)]
        for k in range(w):
            if ops[k] == "Reset":
                h.append((who[k], ("R", "Ok")))
                n = 0
            else:
                n += 1
                h.append((who[k], ("R", ("Number", n))))
        left -= w
    if rng.random() < p_bug:
        k = max(i for i, (_, ev) in enumerate(h) if ev[0] == "R")
        if h[k][1][1] != "Ok":
            h[k] = (h[k][0], ("R", ("Number", h[k][1][1][1] + 1)))
    return h


@pytest.mark.parametrize("bug", [0, 1])
@pytest.mark.parametrize("nc,no", [(8, 64), (4, 17), (6, 30), (3, 10), (8, 40), (1, 9), (2, 64), (64, 64)])
def test_ticket_chain_memo(ctx, nc, no, bug):
    """The wave stage's chain path (wave.hip ticket_chain): adversarial
    histories of several widths and lengths in QSMD_FLAG_MEMO mode --
    verdict, explored count and witness equal to the oracle's memo mode."""
    h, e, _ = gen.adversarial_ticket(nc, no, bug=bool(bug))
    st_o, nd_o, w_o = oracle_c.check_batch(models.MODEL_TICKET, h, e, memo=True, witness=True)
    st, nd, w, _ = ctx.check_arrays(models.MODEL_TICKET, h, e, flags=EXH | MEMO, witness=True)
    assert (int(st[0]), int(nd[0])) == (int(st_o[0]), int(nd_o[0]))
    if int(st[0]) == codec.STATUS_LIN:
        assert np.array_equal(w, w_o)


@pytest.mark.parametrize("nc,no", [(4, 17), (3, 10), (2, 30), (1, 40), (5, 12), (2, 40), (1, 60)])
def test_ticket_chain_exhaustive(ctx, nc, no):
    """The chain's exhaustive count g(S) = deg(S) + nT(S) g(next), against
    the reference DFS's count (oracle, no memo)."""
    for bug in (False, True):
        h, e, _ = gen.adversarial_ticket(nc, no, bug=bug)
        _compare(ctx, models.MODEL_TICKET, h, e, max_nodes=10**9)


@pytest.mark.parametrize("memo", [False, True])
@pytest.mark.parametrize("n_pid", [1, 2, 8])
def test_ticket_chain_like_batches(ctx, n_pid, memo):
    """Chain-shaped histories (and near-chains whose Reset makes two
    successors: the DAG's) of 8..128 events through the host entry and the
    heavy stage's wave mode, with node budgets and model0 variants."""
    rng = random.Random(1000 + n_pid)
    hs = [_ticket_chain_like(rng, rng.randint(4, 64), rng.randint(1, 8), n_pid) for _ in range(400)]
    b = codec.encode(models.TICKET, hs)
    flags = EXH | (MEMO if memo else 0)
    ctx.set_param("heavy_mode", 0)
    ctx.set_stage0_budget(2)
    try:
        # (exhaustive: budgets, since a wide chain's DFS count is (w!)^levels)
        for max_nodes, m0 in ((10**5, None), (40, None), (10**5, models.TicketModel(1, 0, 3)),
                              (10**5, models.TicketModel(0, 0, 0))):
            if memo and max_nodes == 40:
                continue
            if memo:
                max_nodes = 0
            st, nd, w, _ = ctx.check_arrays(models.MODEL_TICKET, b.hdr, b.events, m0, flags=flags,
                                            max_nodes=max_nodes, witness=True)
            st_o, nd_o, w_o = oracle_c.check_batch(models.MODEL_TICKET, b.hdr, b.events, m0, max_nodes, 8,
                                                   witness=True, memo=memo)
            # (memo mode: the compact stages count the reference's nodes, the
            # wave stage the pruning DFS's -- verdicts and witnesses compared)
            diff = (st != st_o) if memo else ((st != st_o) | (nd != nd_o))
            bad = np.nonzero(diff)[0]
            assert len(bad) == 0, (max_nodes, bad[:5], st[bad[:5]], st_o[bad[:5]], nd[bad[:5]], nd_o[bad[:5]])
            lin = np.nonzero(st == codec.STATUS_LIN)[0]
            for i in lin:
                a0, a1 = int(b.hdr[i]["ev_off"]), int(b.hdr[i]["ev_off"]) + int(b.hdr[i]["n_ev"])
                assert np.array_equal(w[a0:a1], w_o[a0:a1]), i
    finally:
        ctx.set_param("heavy_mode", 2)
        ctx.set_stage0_budget(32)
