"""Literal list-semantics transliteration of the reference checker.

TEST INFRASTRUCTURE ONLY. Nothing in the product path may import this file;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg use the oracle, and only as the checker.

This module restates ``src/Linearisability.hs:25-69`` of
advancedtelematic/quickcheck-state-machine-distributed *literally*: histories
are Python lists that are copied the way the Haskell cons lists are rebuilt
(``filter1``, ``findResponse``), the forest of interleavings is produced
lazily (generators), and ``step`` / ``any'`` short-circuit left to right exactly
as ``any``/``&&`` do in the Haskell source.  A node counter is incremented on
every ``step`` evaluation (``src/Linearisability.hs:63``); that is the
definition of "explored nodes" used throughout the build.

It also restates the two models the reference's properties check:

* Bank   -- ``test/Bank.hs:92-131`` (``next'``, ``invariant``, ``post``)
* TicketDispenser -- ``test/TicketDispenser.hs:81-102``

with Haskell ``Data.Map`` / ``Maybe`` semantics, including the ``Map.!``
failure (``test/Bank.hs:128``) which is raised here as :class:`ModelError`.

Representation (mirrors the Haskell values):

* history  : ``[(pid, ('L', inv)) | (pid, ('R', resp))]``  (``History`` at :18)
* Ticket   : inv ``'TakeTicket' | 'Reset'``; resp ``('Number', i) | 'Ok'``;
             model ``None`` (Nothing) or ``int`` (Just n)
* Bank     : inv ``('OpenAccount', a) | ('Deposit', a, m) | ('Withdraw', a, m)
             | ('CheckBalance', a) | ('Transfer', a, m, b)``; resp one of the
             nullary names or ``('Balance', v)``; model a ``dict`` account->int
             treated as immutable (Data.Map).

Parity anchor: the reference cannot be run anywhere in this pipeline (no GHC,
SURVEY.md §8c).  This transliteration is pinned by the reference's only
known answer (``test/TicketDispenser.hs:326-347``, KAT-2) and the hand-derived
KATs of SURVEY.md §8c; see ``tests/test_oracle.py``.
"""

from __future__ import annotations

import sys


class ModelError(Exception):
    """A model function diverged (Haskell exception), e.g. ``Map.!`` on a
    missing key -- ``test/Bank.hs:128``."""


class BudgetExceeded(Exception):
    pass


# ---------------------------------------------------------------------------
# src/Linearisability.hs:25-50
# ---------------------------------------------------------------------------

def take_invocations(hist):
    """``takeInvocations`` (src/Linearisability.hs:25-28)."""
    out = []
    for pid, ev in hist:
        if ev[0] == "L":
            out.append((pid, ev[1]))
        else:
            break
    return out


def find_response(pid, hist):
    """``findResponse`` (src/Linearisability.hs:30-34): first ``Right`` whose
    pid equals ``pid``; returns ``[(resp, hist_without_it)]`` or ``[]``."""
    for i, (p, ev) in enumerate(hist):
        if ev[0] == "R" and p == pid:
            return [(ev[1], hist[:i] + hist[i + 1:])]
    return []


def filter1(pred, xs):
    """``filter1`` (src/Linearisability.hs:47-50): keep elements while ``pred``
    holds, drop the first one for which it fails, keep the rest."""
    for i, x in enumerate(xs):
        if not pred(x):
            return xs[:i] + xs[i + 1:]
    return list(xs)


def interleavings(es):
    """``interleavings`` (src/Linearisability.hs:36-42), lazily: yields
    ``(pid, inv, resp, es')``; the subforest is ``interleavings(es')``."""
    if not es:
        return
    for pid, inv in take_invocations(es):
        def not_match_invocation(e, pid=pid):           # :44-45
            return not (e[0] == pid and e[1][0] == "L")
        es1 = filter1(not_match_invocation, es)
        for resp, es2 in find_response(pid, es1):
            yield (pid, inv, resp, es2)


# ---------------------------------------------------------------------------
# src/Linearisability.hs:52-69
# ---------------------------------------------------------------------------

class _Counter:
    __slots__ = ("nodes", "max_nodes", "path")

    def __init__(self, max_nodes=0):
        self.nodes = 0
        self.max_nodes = max_nodes
        self.path = []


def _step(transition, postcondition, model, node, ctr):
    """``step`` (src/Linearisability.hs:63-65)."""
    if ctr.max_nodes and ctr.nodes >= ctr.max_nodes:
        raise BudgetExceeded()
    ctr.nodes += 1
    _pid, inv, resp, es2 = node
    if not postcondition(model, inv, resp):
        return False
    model2 = transition(transition(model, ("L", inv)), ("R", resp))
    ctr.path.append((_pid, inv, resp))
    roses = interleavings(es2)
    # any' _ [] = True ; any' p xs = any p xs      (:67-69)
    first = next(roses, None)
    if first is None:
        return True
    if _step(transition, postcondition, model2, first, ctr):
        return True
    for child in roses:
        if _step(transition, postcondition, model2, child, ctr):
            return True
    ctr.path.pop()
    return False


def linearisable(transition, postcondition, model0, es, max_nodes=0):
    """``linearisable`` (src/Linearisability.hs:52-61).

    Returns ``(status, nodes, path)`` where status is one of
    ``'lin' | 'nonlin' | 'error' | 'budget'`` and ``path`` is the list of
    operations ``(pid, inv, resp)`` of the successful linearisation.
    """
    ctr = _Counter(max_nodes)
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 10000))
    try:
        if not es:                                     # :59
            return "lin", 0, []
        for node in interleavings(es):                 # :61 plain `any`
            if _step(transition, postcondition, model0, node, ctr):
                return "lin", ctr.nodes, list(ctr.path)
        return "nonlin", ctr.nodes, []
    except ModelError:
        return "error", ctr.nodes, []
    except BudgetExceeded:
        return "budget", ctr.nodes, []
    finally:
        sys.setrecursionlimit(old)


# ---------------------------------------------------------------------------
# TicketDispenser model, test/TicketDispenser.hs:81-102
# ---------------------------------------------------------------------------

def ticket_transition(m, ev):
    """``transition`` (test/TicketDispenser.hs:81-85); model ``Maybe Int``."""
    kind, x = ev
    if kind == "R":
        return m
    if x == "TakeTicket":
        return None if m is None else m + 1
    if x == "Reset":
        return 0
    raise ValueError(x)


def ticket_postcondition(m, inv, resp):
    """``postcondition`` (test/TicketDispenser.hs:99-102)."""
    if inv == "TakeTicket" and isinstance(resp, tuple) and resp[0] == "Number":
        return m is not None and resp[1] == m + 1
    if inv == "Reset" and resp == "Ok":
        return True
    return False


TICKET_INIT = None          # initModel = Nothing  (test/TicketDispenser.hs:73-74)


# ---------------------------------------------------------------------------
# Bank model, test/Bank.hs:92-131
# ---------------------------------------------------------------------------

def bank_next(model, ev):
    """``next'`` (test/Bank.hs:92-101), Data.Map.insertWith semantics."""
    kind, x = ev
    if kind == "R":
        return model
    op = x[0]
    if op == "OpenAccount":
        a = x[1]
        if a not in model:
            m2 = dict(model)
            m2[a] = 0
            return m2
        return model
    if op == "Deposit":                     # insertWith (+) acc money
        a, money = x[1], x[2]
        m2 = dict(model)
        m2[a] = model[a] + money if a in model else money
        return m2
    if op == "Withdraw":                    # insertWith (\new old -> old - new)
        a, money = x[1], x[2]
        m2 = dict(model)
        m2[a] = model[a] - money if a in model else money
        return m2
    if op == "CheckBalance":
        return model
    if op == "Transfer":
        a, money, b = x[1], x[2], x[3]
        return bank_next(bank_next(model, ("L", ("Withdraw", a, money))),
                         ("L", ("Deposit", b, money)))
    raise ValueError(x)


def bank_invariant(model):
    """``invariant`` (test/Bank.hs:103-104)."""
    return all(v >= 0 for v in model.values())


def _maybe_ge(model, a, money):
    # M.lookup acc model >= Just money ; Nothing < Just _
    return a in model and model[a] >= money


def bank_post(model, req, resp):
    """``post`` (test/Bank.hs:118-131)."""
    if not bank_invariant(model):
        return False
    op = req[0]
    if op == "OpenAccount":
        a = req[1]
        return resp == ("AccountAlreadyExists" if a in model else "AccountCreated")
    if op == "Deposit":
        return resp == "DepositMade"
    if op == "Withdraw":
        return resp == ("WithdrawalMade" if _maybe_ge(model, req[1], req[2])
                        else "InsufficientFunds")
    if op == "CheckBalance":
        # resp == Balance (model M.! acc): the derived Eq only forces the
        # field when resp is itself a Balance.
        if isinstance(resp, tuple) and resp[0] == "Balance":
            a = req[1]
            if a not in model:
                raise ModelError("Map.!: given key is not an element in the map")
            return resp[1] == model[a]
        return False
    if op == "Transfer":
        return resp == ("TransferMade" if _maybe_ge(model, req[1], req[2])
                        else "InsufficientFunds")
    raise ValueError(req)


BANK_INIT = {}              # initModel' = M.empty  (test/Bank.hs:86-87)


MODELS = {
    "ticket": (ticket_transition, ticket_postcondition, TICKET_INIT),
    "bank": (bank_next, bank_post, BANK_INIT),
}


def check(model_name, history, model0=None, max_nodes=0):
    """Convenience: run :func:`linearisable` with a named model."""
    tr, post, init = MODELS[model_name]
    return linearisable(tr, post, init if model0 is None else model0,
                        list(history), max_nodes)
