"""Random Python-level histories for tests (any shape: well-formed or not,
shared pids, pending invocations, stray responses, Bank model errors)."""

import random

TICKET_INV = ["TakeTicket", "Reset"]


def ticket_event(rng, vmax=6):
    if rng.random() < 0.5:
        return ("L", rng.choice(TICKET_INV))
    return ("R", "Ok" if rng.random() < 0.25 else ("Number", rng.randint(0, vmax)))


def bank_event(rng, accounts, vmax=12):
    if rng.random() < 0.5:
        op = rng.choice(["OpenAccount", "Deposit", "Withdraw", "CheckBalance", "Transfer"])
        a = rng.choice(accounts)
        if op in ("OpenAccount", "CheckBalance"):
            return ("L", (op, a))
        m = rng.randint(1, vmax)
        if op in ("Deposit", "Withdraw"):
            return ("L", (op, a, m))
        return ("L", (op, a, m, rng.choice(accounts)))
    r = rng.random()
    if r < 0.35:
        return ("R", ("Balance", rng.randint(-3, vmax)))
    return ("R", rng.choice(["AccountCreated", "DepositMade", "WithdrawalMade", "TransferMade",
                             "AccountAlreadyExists", "AccountDoesntExist", "InsufficientFunds"]))


def random_history(rng, model, n_ev, n_pid):
    pids = [f"p{i}" for i in range(n_pid)]
    accounts = pids[:6]
    h = []
    for _ in range(n_ev):
        p = rng.choice(pids)
        h.append((p, ticket_event(rng) if model == "ticket" else bank_event(rng, accounts)))
    return h


def wellformed_history(rng, model, n_ops, n_pid, p_pending=0.1):
    """Per-pid alternating inv/resp with random interleaving; responses are
    random (so verdicts are mixed)."""
    pids = [f"p{i}" for i in range(n_pid)]
    pending = {p: None for p in pids}
    h = []
    ops_left = n_ops
    while ops_left > 0 or any(v is not None for v in pending.values()):
        p = rng.choice(pids)
        if pending[p] is None:
            if ops_left == 0:
                continue
            ev = ticket_event(rng) if model == "ticket" else bank_event(rng, pids[:6])
            while ev[0] != "L":
                ev = ticket_event(rng) if model == "ticket" else bank_event(rng, pids[:6])
            h.append((p, ev))
            pending[p] = ev
            ops_left -= 1
        else:
            if rng.random() < p_pending and ops_left == 0:
                pending[p] = None          # leave it pending
                continue
            ev = ticket_event(rng) if model == "ticket" else bank_event(rng, pids[:6])
            while ev[0] != "R":
                ev = ticket_event(rng) if model == "ticket" else bank_event(rng, pids[:6])
            h.append((p, ev))
            pending[p] = None
    return h
