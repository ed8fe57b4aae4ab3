"""Host-side mirror of the reference module ``Linearisability``
(src/Linearisability.hs:1-7 exports ``History``, ``linearisable``, ``trace``,
``wellformed``), with the search itself on the GPU.

* :func:`linearisable` keeps the reference signature
  ``linearisable transition postcondition model0 history -> Bool``
  (src/Linearisability.hs:52-58).  ``transition``/``postcondition`` must be
  the closures of a :class:`~qsmd.models.DeviceModel` (the reference's
  Bank / TicketDispenser models); any other closure raises -- there is no CPU
  search to fall back to.  Model exceptions propagate as in Haskell
  (:class:`~qsmd.models.ModelError` for ``Map.!``, test/Bank.hs:128).
* :func:`linearisable_batch` is the throughput entry point.
* :func:`trace` (src/Linearisability.hs:73-93) and :func:`wellformed`
  (src/Linearisability.hs:97-135) are host utilities; :func:`replay_witness`
  re-checks a GPU witness against the host model.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import codec, device
from .models import BY_ID, BY_NAME, DeviceModel, EncodeError, ModelError

__all__ = ["linearisable", "linearisable_batch", "trace", "wellformed", "replay_witness",
           "CheckResult", "NotSequential", "BudgetExceeded", "wellformed_batch"]


class BudgetExceeded(RuntimeError):
    """max_nodes was reached before the search decided (not a reference outcome)."""


def _device_model(transition, postcondition) -> DeviceModel:
    for m in BY_ID.values():
        if transition is m.transition and postcondition is m.postcondition:
            return m
    raise NotImplementedError(
        "no device functor for these model closures: the GPU checker supports the "
        "reference's Bank (test/Bank.hs) and TicketDispenser (test/TicketDispenser.hs) models")


def _as_model(model) -> DeviceModel:
    if isinstance(model, DeviceModel):
        return model
    if isinstance(model, str):
        return BY_NAME[model]
    return BY_ID[int(model)]


@dataclass
class CheckResult:
    batch: codec.Batch
    status: np.ndarray
    nodes: np.ndarray
    witness: np.ndarray | None
    totals: dict = field(default_factory=dict)

    def verdict(self, i):
        return codec.STATUS_NAMES[int(self.status[i])]

    def witness_of(self, i):
        """Invocation-event indices of the linearisation of history i."""
        if self.witness is None or self.status[i] != codec.STATUS_LIN:
            return None
        h = self.batch.hdr[i]
        w = self.witness[h["ev_off"]: h["ev_off"] + h["n_ev"]]
        out = []
        for x in w:
            if x == codec.WITNESS_END:
                break
            out.append(int(x))
        return out


def linearisable_batch(model, histories, model0=None, *, max_nodes=0, witness=False,
                       flags=device.QSMD_FLAG_EXHAUSTIVE, ctx=None) -> CheckResult:
    """Check many histories in one device call."""
    m = _as_model(model)
    batch = codec.encode(m, histories, model0)
    accounts0 = m.new_account_map(model0)
    packed = m.pack_model0(model0, accounts0)
    ctx = ctx or device.default_context()
    status, nodes, wit, totals = ctx.check_arrays(m.model_id, batch.hdr, batch.events, packed,
                                                  flags, max_nodes, witness)
    return CheckResult(batch, status, nodes, wit, totals)


def linearisable(transition, postcondition, model0, history, *, max_nodes=0, ctx=None) -> bool:
    """``linearisable`` (src/Linearisability.hs:52-69) on the GPU."""
    m = _device_model(transition, postcondition)
    res = linearisable_batch(m, [history], model0, max_nodes=max_nodes, ctx=ctx)
    st = int(res.status[0])
    if st == codec.STATUS_LIN:
        return True
    if st == codec.STATUS_NONLIN:
        return False
    if st == codec.STATUS_MODEL_ERROR:
        raise ModelError("Map.!: given key is not an element in the map")
    if st == codec.STATUS_ENCODE_ERROR:
        raise EncodeError(res.batch.encode_errors.get(0, "history cannot be encoded"))
    raise BudgetExceeded(f"search stopped after {int(res.nodes[0])} nodes")


# ---------------------------------------------------------------------------
# trace (src/Linearisability.hs:73-93)
# ---------------------------------------------------------------------------

def pretty_print_pid(pid) -> str:
    """``prettyPrintProcessId = reverse . takeWhile (/= ':') . reverse . show``."""
    s = str(pid)
    return s.rsplit(":", 1)[-1]


def trace(transition, model0, history, model: DeviceModel | None = None) -> str:
    """Pretty-print a history with the model state before each event, applied
    in *history* order (src/Linearisability.hs:76-93)."""
    m = model
    if m is None:
        for cand in BY_ID.values():
            if transition is cand.transition:
                m = cand
        if m is None:
            raise NotImplementedError("trace needs a DeviceModel to show values")
    out = []
    cur = model0
    for pid, ev in history:
        kind, x = ev
        if kind == "L":
            out.append(f"{m.show_model(cur)}\n  ==> {m.show_inv(x)}  [{pretty_print_pid(pid)}]\n")
        else:
            out.append(f"{m.show_model(cur)}\n  <== {m.show_resp(x)}  [{pretty_print_pid(pid)}]\n")
        cur = transition(cur, ev)
    return "".join(out)


# ---------------------------------------------------------------------------
# wellformed (src/Linearisability.hs:97-135)
# ---------------------------------------------------------------------------

@dataclass(frozen=True)
class NotSequential:
    """``NotSequential`` constructors (src/Linearisability.hs:97-104)."""
    kind: str
    args: tuple


def _is_sequential(history):
    """``isSequential`` (src/Linearisability.hs:109-128)."""
    if history and history[0][1][0] == "R":
        pid, (_, resp) = history[0]
        return NotSequential("FirstEventIsntInvocation", (pid, resp))
    i = 0
    n = len(history)
    while True:
        rest = n - i
        if rest == 0:
            return None
        p0, (k0, x0) = history[i]
        if rest == 1:
            return NotSequential("LoneResponse", (p0, x0)) if k0 == "R" else None
        p1, (k1, x1) = history[i + 1]
        if k0 == "L" and k1 == "R":
            if p0 == p1:
                i += 2
                continue
            return NotSequential("InvocationFollowedByNonMatchingResponse", (p0, x0, p1, x1))
        if k0 == "L" and k1 == "L":
            return NotSequential("InvocationFollowedByInvocation", (p0, x0, p1, x1))
        if k0 == "R" and k1 == "R":
            return NotSequential("ResponseFollowedByResponse", (p0, x0, p1, x1))
        return NotSequential("ResponseFollowedByInvocation", (p0, x0, p1, x1))


def wellformed_batch(pids, histories, ctx=None):
    """Batched ``wellformed pids history`` on the GPU (csrc/wellformed.hip,
    src/Linearisability.hs:130-135, call site test/Bank.hs:281-283): for each
    history None (``Right ()``) or the first :class:`NotSequential`, checking
    each pid's subhistory in ``pids`` order.  Same results as
    :func:`wellformed` one history at a time."""
    from . import codec, device
    hdr, events, pid_index = codec.encode_shape(histories)
    ranks = [pid_index[p] for p in pids if p in pid_index]
    own = ctx is None
    if own:
        ctx = device.Context(0)
    try:
        res = ctx.wellformed_arrays(hdr, events, ranks)
    finally:
        if own:
            ctx.close()
    out = []
    for h, r in zip(histories, res):
        code = int(r["code"])
        if code == 0:
            out.append(None)
            continue
        if code == codec.WF_ENCODE_ERROR:
            raise ValueError("history not encodable")
        e0, e1 = h[int(r["ev0"])], h[int(r["ev1"])]
        kind = codec.WF_KINDS[code]
        if kind in ("FirstEventIsntInvocation", "LoneResponse"):
            out.append(NotSequential(kind, (e0[0], e0[1][1])))
        else:
            out.append(NotSequential(kind, (e0[0], e0[1][1], e1[0], e1[1][1])))
    return out


def wellformed(pids, history):
    """Returns None (``Right ()``) or the first :class:`NotSequential`
    (``Left err``), checking each pid's subhistory in ``pids`` order."""
    for pid in pids:
        err = _is_sequential([e for e in history if e[0] == pid])
        if err is not None:
            return err
    return None


# ---------------------------------------------------------------------------
# witness replay (host re-check of a GPU linearisation)
# ---------------------------------------------------------------------------

def replay_witness(model, history, witness, model0=None) -> bool:
    """Re-run the operations named by ``witness`` (invocation event indices,
    one per level) with the host model: each step pairs the chosen
    invocation with the first remaining response of its pid and removes the
    first remaining invocation and response of that pid (Lemma L1).  True iff
    every postcondition holds and the final state has no further child."""
    m = _as_model(model)
    if not witness:                     # only `linearisable _ _ _ [] = True` (:59)
        return len(history) == 0
    cur = m.init_model if model0 is None else model0
    removed = set()
    for j in witness:
        pid, (kind, inv) = history[j]
        if kind != "L" or j in removed:
            return False
        # first remaining response of this pid must come after every remaining
        # invocation we could pick (takeInvocations prefix)
        first_resp = next((i for i, (p, (k, _)) in enumerate(history)
                           if i not in removed and k == "R"), len(history))
        if j > first_resp:
            return False
        r = next((i for i, (p, (k, _)) in enumerate(history)
                  if i not in removed and k == "R" and p == pid), None)
        if r is None:
            return False
        resp = history[r][1][1]
        if not m.postcondition(cur, inv, resp):
            return False
        cur = m.transition(m.transition(cur, ("L", inv)), ("R", resp))
        i0 = next(i for i, (p, (k, _)) in enumerate(history)
                  if i not in removed and k == "L" and p == pid)
        removed.add(i0)
        removed.add(r)
    # leaf: no remaining invocation before the first remaining response has a response
    first_resp = next((i for i, (p, (k, _)) in enumerate(history)
                       if i not in removed and k == "R"), len(history))
    for i, (p, (k, _)) in enumerate(history[:first_resp]):
        if i in removed or k != "L":
            continue
        if any(ii not in removed and kk == "R" and pp == p
               for ii, (pp, (kk, _)) in enumerate(history)):
            return False
    return True
