"""Pin the oracle before trusting it (CPU only).

1. Both oracles reproduce the known answers of SURVEY.md §8c -- KAT-2 is the
   reference's own example (test/TicketDispenser.hs:326-347).
2. The C counter-state restatement (oracle/ref_cpu.c) agrees with the literal
   list transliteration (oracle/linearise_lists.py) on verdict AND node count
   for arbitrary histories (ill-formed, shared pids, pending invocations,
   stray responses, Bank Map.! errors), via hypothesis.
3. Both agree with the committed golden vectors (tests/golden/, produced by
   tests/golden/make_golden.py from the literal transliteration).
"""

import json
import os
import random

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import histgen
import linearise_lists as LL
import oracle_c
from kats import KATS
from qsmd import codec, models

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "histories.json")


def c_oracle(model, hist, model0=None, max_nodes=0):
    m = models.BY_NAME[model]
    b = codec.encode(m, [hist], model0)
    packed = m.pack_model0(model0, m.new_account_map(model0))
    st_, nd, w = oracle_c.check_batch(m.model_id, b.hdr, b.events, packed, max_nodes, witness=True)
    return codec.STATUS_NAMES[int(st_[0])], int(nd[0]), w


@pytest.mark.parametrize("name", sorted(KATS))
def test_kats_literal(name):
    model, hist, status, nodes = KATS[name]
    got = LL.check(model, hist)
    assert (got[0], got[1]) == (status, nodes)


@pytest.mark.parametrize("name", sorted(KATS))
def test_kats_c_oracle(name):
    model, hist, status, nodes = KATS[name]
    got = c_oracle(model, hist)
    assert (got[0], got[1]) == (status, nodes)


def test_kat2_path_is_reference_counterexample():
    # The reference prints exactly this history as non-linearisable; the search
    # tries Reset (ok), then the two identical (TakeTicket, Number 2) children.
    model, hist, _, _ = KATS["KAT2_reference_example"]
    status, nodes, path = LL.check(model, hist)
    assert status == "nonlin" and nodes == 3 and path == []


def _hist_strategy():
    @st.composite
    def strat(draw):
        model = draw(st.sampled_from(["ticket", "bank"]))
        seed = draw(st.integers(0, 2**32 - 1))
        rng = random.Random(seed)
        if draw(st.booleans()):
            h = histgen.random_history(rng, model, draw(st.integers(0, 12)), draw(st.integers(1, 4)))
        else:
            h = histgen.wellformed_history(rng, model, draw(st.integers(0, 7)), draw(st.integers(1, 4)))
        return model, h
    return strat()


@settings(max_examples=1500, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_hist_strategy())
def test_c_oracle_equals_literal(mh):
    model, hist = mh
    lit = LL.check(model, hist, max_nodes=20000)
    got = c_oracle(model, hist, max_nodes=20000)
    assert (got[0], got[1]) == (lit[0], lit[1])


def test_c_oracle_witness_is_literal_path():
    rng = random.Random(11)
    n = 0
    for _ in range(6000):
        model = rng.choice(["ticket", "bank"])
        hist = histgen.wellformed_history(rng, model, rng.randint(1, 5), rng.randint(1, 3))
        status, nodes, path = LL.check(model, hist)
        if status != "lin" or not hist:
            continue
        _, _, w = c_oracle(model, hist)
        seq = []
        for x in w:
            if x == 0xFF:
                break
            seq.append(int(x))
        # the literal path is [(pid, inv, resp)]; the witness names the
        # invocation events; same length and same invocations in order
        assert len(seq) == len(path)
        assert [hist[j][1][1] for j in seq] == [op[1] for op in path]
        assert [hist[j][0] for j in seq] == [op[0] for op in path]
        n += 1
    assert n > 50


def test_model0_c_oracle_equals_literal():
    rng = random.Random(3)
    for _ in range(600):
        model = rng.choice(["ticket", "bank"])
        hist = histgen.wellformed_history(rng, model, rng.randint(1, 6), 3)
        model0 = rng.choice([None, 0, 3]) if model == "ticket" else \
            {"p0": rng.randint(0, 20), "p1": rng.randint(0, 20)}
        lit = LL.check(model, hist, model0=model0)
        got = c_oracle(model, hist, model0=model0)
        assert (got[0], got[1]) == (lit[0], lit[1])


def test_golden_vectors():
    with open(GOLDEN) as f:
        golden = json.load(f)
    assert len(golden["cases"]) >= 500
    for case in golden["cases"]:
        hist = [(p, (k, _untuple(x))) for p, k, x in case["history"]]
        model0 = case.get("model0")
        got = c_oracle(case["model"], hist, model0=model0, max_nodes=case["max_nodes"])
        assert (got[0], got[1]) == (case["status"], case["nodes"]), case["id"]


def _untuple(x):
    return tuple(_untuple(y) for y in x) if isinstance(x, list) else x


def test_wellformed_ref_matches_host_mirror():
    """oracle/wellformed_ref.py (checker of the device kernel) and the host
    mirror qsmd.wellformed agree (src/Linearisability.hs:97-135)."""
    import random

    import histgen
    import wellformed_ref
    from qsmd.linearisability import wellformed
    rng = random.Random(5)
    for _ in range(3000):
        h = (histgen.random_history(rng, "bank", rng.randint(0, 20), rng.randint(1, 4)) if rng.random() < 0.5
             else histgen.wellformed_history(rng, "ticket", rng.randint(0, 8), rng.randint(1, 4)))
        pids = rng.sample(["p0", "p1", "p2", "p3"], rng.randint(1, 4))
        err = wellformed(pids, h)
        assert wellformed_ref.wellformed(pids, h) == (None if err is None else (err.kind, tuple(err.args)))


def _memo_count(transition, postcondition, model0, es):
    """Exact reference node count with a state memo (the argument of
    DESIGN.md §4.1): linearise_lists' own forest and models, a failed
    subtree's count reused for a repeated (remaining history, model)."""
    import linearise_lists as LL
    memo = {}

    def sub(model, es2):
        k = (tuple(es2), model if not isinstance(model, dict) else tuple(sorted(model.items())))
        if k in memo:
            return False, memo[k]
        cnt, first = 0, True
        for node in LL.interleavings(es2):
            first = False
            ok, c = step(model, node)
            cnt += c
            if ok:
                return True, cnt
        if first:
            return True, 0
        memo[k] = cnt
        return False, cnt

    def step(model, node):
        _pid, inv, resp, es2 = node
        if not postcondition(model, inv, resp):
            return False, 1
        ok, c = sub(transition(transition(model, ("L", inv)), ("R", resp)), es2)
        return ok, 1 + c

    total = 0
    for node in LL.interleavings(es):
        ok, c = step(model0, node)
        total += c
        if ok:
            return "lin", total
    return "nonlin", total


def test_memo_count_equals_plain_count_and_pins_large_adversarial_counts():
    """The memoised count equals the plain transliteration's on the 4x17
    adversarial history (923201 nodes), and pins the exact counts the GPU's
    exact memo reports beyond any plain search: 6x30 -> 88071120488677,
    8x40 -> 36212384984955121261601 (> 2^64: a budget on the GPU)."""
    import sys
    sys.setrecursionlimit(100000)
    import linearise_lists as LL
    from qsmd import codec, gen, models

    def hist(nc, no):
        h, e, _ = gen.adversarial_ticket(nc, no, bug=True)

        class B:
            pass
        b = B()
        b.hdr, b.events, b.model = h, e, models.TICKET
        b.pid_maps, b.account_maps = {0: {0: 0}}, {0: {}}
        return codec.decode_history(b, 0)

    h = hist(4, 17)
    assert _memo_count(LL.ticket_transition, LL.ticket_postcondition, None, h) == ("nonlin", 923201)
    assert LL.linearisable(LL.ticket_transition, LL.ticket_postcondition, None, h)[:2] == ("nonlin", 923201)
    assert _memo_count(LL.ticket_transition, LL.ticket_postcondition, None, hist(6, 30)) == ("nonlin", 88071120488677)
    assert _memo_count(LL.ticket_transition, LL.ticket_postcondition, None, hist(8, 40)) == \
        ("nonlin", 36212384984955121261601)
