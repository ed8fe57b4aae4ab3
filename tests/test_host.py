"""CPU tests of the host side: the C ABI library loads and exports every
symbol include/*.h declares (no compute calls), the marshaller, the
generator, and the host mirrors of `trace` / `wellformed`
(src/Linearisability.hs:73-135)."""

import ctypes
import os
import random
import re

import numpy as np
import pytest

import histgen
import linearise_lists as LL
import oracle_c
from kats import KAT2_TRACE, KATS
from qsmd import codec, device, gen, models
from qsmd.linearisability import NotSequential, replay_witness, trace, wellformed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(qsmd_\w+)\s*\(", txt)))


def test_abi_exports_every_declared_symbol():
    lib = ctypes.CDLL(device.LIB_PATH)
    names = _declared("qsmd.h")
    assert "qsmd_check_batch" in names and "qsmd_check_batch_device" in names
    # qsmd_gen.h's device entry point lives in libqsmd.so too
    names += [n for n in _declared("qsmd_gen.h") if n.endswith("_device")]
    for n in names:
        assert hasattr(lib, n), n
    assert set(device.EXPORTS) == set(names)
    assert device.load_library().qsmd_abi_version() == 3


def test_fast_host_entry_forwards_to_the_c_abi():
    """The binding's CPython fast path (csrc/pyfast.c) is built and is only a
    forwarder: on a NULL context it returns the C ABI's own QSMD_ERR_ARG, like
    the ctypes call; buffers that are not include/qsmd.h records are refused
    before any call."""
    from qsmd import _pyfast
    lib = device.load_library()
    fn = ctypes.cast(lib.qsmd_check_batch, ctypes.c_void_p).value
    hdr, ev, _ = gen.generate_config("ticket_2x10", 0, 4)
    st, nd, tot = np.empty(4, np.uint8), np.empty(4, np.uint64), device.Totals()
    rc_c = lib.qsmd_check_batch(None, models.MODEL_TICKET, hdr.ctypes.data, 4, ev.ctypes.data, len(ev), None, 1, 0,
                                st.ctypes.data, nd.ctypes.data, None, ctypes.byref(tot))
    rc_f = _pyfast.check_batch(fn, 0, models.MODEL_TICKET, hdr, ev, 0, 1, 0, st, nd, None, tot)
    assert rc_c == rc_f == -1
    with pytest.raises(ValueError):
        _pyfast.check_batch(fn, 0, 1, hdr, ev.view(np.uint8)[:12], 0, 1, 0, st, nd, None, tot)
    with pytest.raises(ValueError):
        _pyfast.check_batch(fn, 0, 1, hdr, ev, 0, 1, 0, st[:2], nd, None, tot)
    with pytest.raises(TypeError):
        _pyfast.check_batch(fn, 0, 1, hdr, ev, 0, 1, 0, st, nd, None, b"read-only")


def test_gen_abi_exports():
    lib = ctypes.CDLL(gen.LIB_PATH)
    for n in _declared("qsmd_gen.h"):
        if not n.endswith("_device"):                # host generator library
            assert hasattr(lib, n), n


def test_struct_layouts():
    assert codec.HDR_DTYPE.itemsize == 16 and codec.EV_DTYPE.itemsize == 8
    assert ctypes.sizeof(device.Totals) == 64
    assert ctypes.sizeof(models.BankModel) == 72 and ctypes.sizeof(models.TicketModel) == 16
    assert ctypes.sizeof(gen.GenParams) == 48


def test_no_device_is_loud():
    # No GPU in this container: opening a context must fail, never fall back.
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(device.DeviceError):
        device.Context(0)


def test_codec_round_trip():
    rng = random.Random(2)
    for model in ("ticket", "bank"):
        sub = [histgen.random_history(rng, model, rng.randint(0, 20), rng.randint(1, 5))
               for _ in range(200)]
        b = codec.encode(models.BY_NAME[model], sub)
        for i, h in enumerate(sub):
            if i in b.encode_errors:
                continue
            assert codec.decode_history(b, i) == h


def test_codec_pid_mapping_is_verdict_invariant():
    # Eq pid only: renaming pids cannot change the verdict (src/Linearisability.hs:30-45)
    model, hist, status, nodes = KATS["KAT3_distinct_pids"]
    ren = [({"c1": "pid://x:9", "c2": "pid://y:3"}[p], e) for p, e in hist]
    assert LL.check(model, ren)[:2] == (status, nodes)
    b1 = codec.encode(models.TICKET, [hist])
    b2 = codec.encode(models.TICKET, [ren])
    assert np.array_equal(b1.events, b2.events)


def test_codec_encode_errors():
    bad = [
        [("p", ("L", "Jump"))],                                      # unknown constructor
        [("p", ("R", ("Number", 2**31)))],                           # outside int32
        [("p", ("L", "Reset"))] * 129,                               # > 128 events
    ]
    b = codec.encode(models.TICKET, bad)
    assert set(b.encode_errors) == {0, 1, 2}
    assert (b.hdr["model_id"] == codec.BAD_MODEL).all()
    accts = [(f"a{i}", ("L", ("OpenAccount", f"a{i}"))) for i in range(9)]
    b = codec.encode(models.BANK, [accts])
    assert 0 in b.encode_errors                                      # > 8 accounts
    st, nd, _ = oracle_c.check_batch(models.MODEL_BANK, b.hdr, b.events)
    assert st[0] == codec.STATUS_ENCODE_ERROR and nd[0] == 0


def test_generator_deterministic_and_shardable():
    p = gen.params(**gen.CONFIGS["bank_4x16"])
    h1, e1, _ = gen.generate(p, 0, 3000, threads=4)
    h2, e2, _ = gen.generate(p, 0, 3000, threads=1)
    assert np.array_equal(e1, e2) and np.array_equal(h1, h2)
    # rank r of N generates [r*n, (r+1)*n) of the same global stream
    _, e3, _ = gen.generate(p, 1000, 2000, threads=2)
    assert np.array_equal(e3, e1[1000 * 32:])


@pytest.mark.parametrize("name", sorted(gen.CONFIGS))
def test_generator_configs_are_wellformed_and_as_specified(name):
    n = 400 if name != "ticket_8x64" else 50
    hdr, ev, bug = gen.generate_config(name, 0, n)
    cfg = gen.CONFIGS[name]
    model = models.BY_ID[cfg["model_id"]]
    assert (hdr["n_ev"] == 2 * cfg["n_ops"]).all()
    b = codec.Batch(model, hdr, ev, [{i: i for i in range(8)}] * n, [{i: i for i in range(8)}] * n)
    for i in range(0, n, 7):
        hist = codec.decode_history(b, i)
        pids = sorted({p for p, _ in hist})
        # per-client pids are well-formed; the shared pid of the reference's
        # parallel TicketDispenser property (Q1) is not (and is not checked there)
        if cfg["pid_mode"] == gen.PID_PER_CLIENT:
            assert wellformed(pids, hist) is None
    st, nd, _ = oracle_c.check_batch(cfg["model_id"], hdr, ev, threads=4, max_nodes=10**6)
    if cfg.get("p_bug", 0) == 0 and cfg.get("pid_mode", 0) == gen.PID_PER_CLIENT:
        assert (st == codec.STATUS_LIN).all()           # linearisable by construction
    if name == "ticket_2x10":
        assert (st == codec.STATUS_NONLIN).any()        # Q1: shared pid + reordering fails
    if name == "bank_4x16_bugs":
        assert 0.3 < bug.mean() < 0.7
        assert (st[bug == 0] == codec.STATUS_LIN).all()
        assert (st[bug == 1] == codec.STATUS_NONLIN).any()


def test_trace_matches_reference_example():
    _, hist, _, _ = KATS["KAT2_reference_example"]
    T = models.TICKET
    assert trace(T.transition, T.init_model, hist) == KAT2_TRACE
    pid = "pid://127.0.0.1:10501:0:8"
    assert trace(T.transition, None, [(pid, e) for _, e in hist]) == KAT2_TRACE


def test_wellformed_cases():
    L, R = codec.Left, codec.Right
    ok = [("a", L("Reset")), ("b", L("Reset")), ("a", R("Ok")), ("b", R("Ok"))]
    assert wellformed(["a", "b"], ok) is None
    assert wellformed(["a"], [("a", R("Ok"))]) == NotSequential("FirstEventIsntInvocation", ("a", "Ok"))
    assert wellformed(["a"], [("a", L("Reset")), ("a", L("Reset"))]).kind == "InvocationFollowedByInvocation"
    assert wellformed(["a"], [("a", L("Reset")), ("a", R("Ok")), ("a", R("Ok"))]).kind == "LoneResponse"
    assert wellformed(["a"], [("a", L("Reset")), ("a", R("Ok")), ("a", R("Ok")), ("a", R("Ok"))]).kind == \
        "ResponseFollowedByResponse"
    assert wellformed(["a"], [("a", L("Reset")), ("a", R("Ok")), ("a", R("Ok")), ("a", L("Reset"))]).kind == \
        "ResponseFollowedByInvocation"
    assert wellformed(["a"], [("a", L("Reset"))]) is None              # pending invocation


def test_replay_witness_accepts_oracle_witnesses_and_rejects_others():
    rng = random.Random(8)
    checked = 0
    for _ in range(3000):
        model = rng.choice(["ticket", "bank"])
        hist = histgen.wellformed_history(rng, model, rng.randint(1, 5), rng.randint(1, 3))
        m = models.BY_NAME[model]
        b = codec.encode(m, [hist])
        st, nd, w = oracle_c.check_batch(m.model_id, b.hdr, b.events, witness=True)
        if st[0] != codec.STATUS_LIN:
            continue
        wit = [int(x) for x in w[: len(hist)]]
        wit = wit[: wit.index(0xFF)] if 0xFF in wit else wit
        assert replay_witness(m, hist, wit)
        if len(wit) >= 1:
            assert not replay_witness(m, hist, wit[:-1]) or len(wit) == 0
        checked += 1
    assert checked > 50


def _ll_closures(model):
    if model == "ticket":
        return LL.ticket_transition, LL.ticket_postcondition, None
    return LL.bank_next, LL.bank_post, {}


def test_haskell_replay_accepts_exactly_the_reference_paths():
    """The Haskell drop-in re-checks every device True with `replay`
    (hs/Linearisability/Device.hs); its Python mirror (tests/hs_replay.py)
    accepts exactly the successful root-to-leaf paths of the reference's
    tree, and rejects truncated witnesses and invocations chosen after a
    pending response (outside takeInvocations, src/Linearisability.hs:25-28)."""
    from hs_replay import hs_replay, successful_paths
    rng = random.Random(31)
    n_paths = n_trunc = n_outside = 0

    def lin_ticket(n_ops, n_pid):
        # each operation takes effect at its response: always linearisable,
        # often in several orders
        pids = [f"p{i}" for i in range(n_pid)]
        h, pend, n, left = [("p0", ("L", "Reset")), ("p0", ("R", "Ok"))], {}, 0, n_ops
        while left or pend:
            p = rng.choice(pids)
            if p not in pend and left:
                pend[p] = rng.choice(["TakeTicket", "TakeTicket", "Reset"])
                h.append((p, ("L", pend[p])))
                left -= 1
            elif p in pend:
                inv = pend.pop(p)
                n = n + 1 if inv == "TakeTicket" else 0
                h.append((p, ("R", ("Number", n) if inv == "TakeTicket" else "Ok")))
        return h

    for it in range(400):
        model = rng.choice(["ticket", "bank"])
        if it % 2:
            model, hist = "ticket", lin_ticket(rng.randint(1, 5), rng.randint(1, 3))
        else:
            hist = histgen.wellformed_history(rng, model, rng.randint(1, 5), rng.randint(1, 3))
        tr, post, m0 = _ll_closures(model)

        def rep(ws, hist=hist, tr=tr, post=post, m0=m0):
            try:
                return hs_replay(tr, post, m0, hist, ws)
            except LL.ModelError:
                return False
        paths = successful_paths(tr, post, m0, hist)
        good = {tuple(p) for p in paths}
        for p in paths:
            assert rep(p), (hist, p)
            n_paths += 1
            for k in range(len(p)):                        # every truncation
                if tuple(p[:k]) not in good:
                    assert not rep(p[:k]), (hist, p[:k])
                    n_trunc += 1
        # random index sequences: accepted iff a successful path
        inv_idx = [i for i, (_, ev) in enumerate(hist) if ev[0] == "L"]
        for _ in range(20):
            ws = [rng.choice(inv_idx) for _ in range(rng.randint(1, len(inv_idx)))] if inv_idx else []
            assert rep(ws) == (tuple(ws) in good or (not ws and not hist)), (hist, ws)
        # an invocation after the first remaining response is never a root
        first_r = next((i for i, (_, ev) in enumerate(hist) if ev[0] == "R"), None)
        late = [i for i in inv_idx if first_r is not None and i > first_r]
        for j in late:
            assert not rep([j]), (hist, j)
            n_outside += 1
        # the Python host replay agrees with the Haskell one on the paths
        m = models.BY_NAME[model]
        for p in paths[:3]:
            assert replay_witness(m, hist, p)
    assert n_paths > 100 and n_trunc > 50 and n_outside > 50, (n_paths, n_trunc, n_outside)
    # KAT-7 by hand: `Open b` (event 2) lies after a's pending response
    # (event 1), so it cannot come first; `Open a` alone is not a leaf
    _, h7, _, _ = KATS["KAT7_bank_concurrent"]
    assert not hs_replay(LL.bank_next, LL.bank_post, {}, h7, [2])          # Open b before a's response
    assert not hs_replay(LL.bank_next, LL.bank_post, {}, h7, [0])          # truncated: Open a only
    src = open(os.path.join(ROOT, "hs", "Linearisability", "Device.hs")).read()
    assert "lookup j (prefix rest)" in src and "go _ rest [] = null (roots rest)" in src
    assert "replay _ _ _ hist [] = null hist" in src


def test_combine_tasks_host():
    """qsmd_combine_tasks (host code of the C ABI): the reference count is
    the nodes above the cut up to the deciding task + every earlier subtree."""
    fr = device.Frontier(status=codec.STATUS_NONLIN, depth=2, top_nodes=10, n_tasks=3)
    tasks = np.zeros(3, dtype=device.TASK_DTYPE)
    tasks["top_before"] = [3, 5, 8]
    nodes = np.array([4, 2, 7], dtype=np.uint64)
    # second subtree holds a linearisation
    assert device.combine_tasks(fr, tasks, np.array([0, 1, 0], np.uint8), nodes) == (1, 5 + 4 + 2, 1)
    # none does: exhausted above the cut
    assert device.combine_tasks(fr, tasks, np.array([0, 0, 0], np.uint8), nodes) == (0, 10 + 13, -1)
    # Map.! in the first subtree
    assert device.combine_tasks(fr, tasks, np.array([2, 1, 0], np.uint8), nodes) == (2, 3 + 4, 0)
    # node limit: the second subtree would cross it
    assert device.combine_tasks(fr, tasks, np.array([0, 1, 0], np.uint8), nodes, max_nodes=10) == (4, 10, -1)
    assert device.combine_tasks(fr, tasks, np.array([0, 1, 0], np.uint8), nodes, max_nodes=11) == (1, 11, 1)
    # decided above the cut after the tasks (True at top node 9)
    fr2 = device.Frontier(status=codec.STATUS_LIN, depth=2, top_nodes=9, n_tasks=3)
    assert device.combine_tasks(fr2, tasks, np.array([0, 0, 0], np.uint8), nodes) == (1, 9 + 13, -1)
    # a skipped task before any decision: skipped (batch early exit)
    assert device.combine_tasks(fr, tasks, np.array([0, 5, 0], np.uint8), nodes)[0] == 5


def test_oracle_memo_verdicts():
    """The oracle's QSMD_FLAG_MEMO restatement keeps every verdict and never
    counts more nodes; on the adversarial TicketDispenser history it turns
    923201 nodes into a few dozen."""
    for name in ("bank_4x16_bugs", "ticket_2x10", "bank_6x24"):
        hdr, ev, _ = gen.generate_config(name, 0, 2000)
        mid = gen.CONFIGS[name]["model_id"]
        s1, n1, w1 = oracle_c.check_batch(mid, hdr, ev, threads=4, witness=True)
        s2, n2, w2 = oracle_c.check_batch(mid, hdr, ev, threads=4, witness=True, memo=True)
        assert np.array_equal(s1, s2) and (n2 <= n1).all()
        assert np.array_equal(w1, w2)
    h, e, _ = gen.adversarial_ticket(4, 17, bug=True)
    assert oracle_c.check_batch(1, h, e)[1][0] == 923201
    st, nd, _ = oracle_c.check_batch(1, h, e, memo=True)
    assert st[0] == codec.STATUS_NONLIN and nd[0] < 100
    for bug in (True, False):
        h, e, _ = gen.adversarial_ticket(8, 64, bug=bug)
        st, _, _ = oracle_c.check_batch(1, h, e, memo=True)
        assert st[0] == (codec.STATUS_NONLIN if bug else codec.STATUS_LIN)


def _c_params(header, name):
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", header)).read(), flags=re.S)
    m = re.search(r"\b" + name + r"\s*\(([^)]*)\)", txt)
    params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
    return len(params)


def test_haskell_binding_matches_the_c_abi():
    """hs/Linearisability/Device.hs is source only (no GHC here): check that
    every `foreign import` names an exported symbol with the C prototype's
    arity, and that the model instances use include/qsmd.h's codes."""
    src = open(os.path.join(ROOT, "hs", "Linearisability", "Device.hs")).read()
    imports = re.findall(r'foreign import ccall safe "(\w+)"\s*\n\s*(\w+)\s*::(.*?)\n(?=\S|\s*\n)', src, re.S)
    assert {c for c, _, _ in imports} >= {"qsmd_open", "qsmd_check_batch", "qsmd_last_error"}
    declared = _declared("qsmd.h")
    for cname, _, sig in imports:
        assert cname in declared, cname
        sig = re.sub(r"--[^\n]*", "", sig)
        assert sig.count("->") == _c_params("qsmd.h", cname), cname
    hdr = open(os.path.join(ROOT, "include", "qsmd.h")).read()
    code = lambda n: int(re.search(r"#define " + n + r"\s+(\d+)u", hdr).group(1))  # noqa: E731
    inst = open(os.path.join(ROOT, "hs", "DeviceInstances.hs")).read()
    for hs_name, c_name in (("OpenAccount", "OPEN_ACCOUNT"), ("Deposit", "DEPOSIT"), ("Withdraw", "WITHDRAW"),
                            ("CheckBalance", "CHECK_BALANCE"), ("Transfer", "TRANSFER")):
        assert re.search(r"Bank\." + hs_name + r"\b[^\n]*Invocation " + str(code("QSMD_BANK_" + c_name)), inst), hs_name
    for hs_name, c_name in (("AccountCreated", "ACCOUNT_CREATED"), ("DepositMade", "DEPOSIT_MADE"),
                            ("WithdrawalMade", "WITHDRAWAL_MADE"), ("TransferMade", "TRANSFER_MADE"),
                            ("AccountAlreadyExists", "ACCOUNT_ALREADY_EXISTS"),
                            ("AccountDoesntExist", "ACCOUNT_DOESNT_EXIST"),
                            ("InsufficientFunds", "INSUFFICIENT_FUNDS"), ("Balance", "BALANCE")):
        assert re.search(r"Bank\." + hs_name + r"\b[^\n]*-> \(" + str(code("QSMD_BANK_" + c_name)), inst), hs_name
    assert re.search(r"TD\.TakeTicket\s*= Just \(Invocation " + str(code("QSMD_TICKET_TAKE_TICKET")), inst)
    assert re.search(r"TD\.Reset\s*= Just \(Invocation " + str(code("QSMD_TICKET_RESET")), inst)
    assert re.search(r"TD\.Number i\) = Just \(" + str(code("QSMD_TICKET_NUMBER")), inst)
    assert re.search(r"TD\.Ok\s*= Just \(" + str(code("QSMD_TICKET_OK")), inst)
    assert "qsmdModelBank   = " + str(code("QSMD_MODEL_BANK")) in src
    assert "qsmdModelTicket = " + str(code("QSMD_MODEL_TICKET")) in src
