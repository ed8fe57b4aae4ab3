"""Marshalling of ``History pid inv resp`` values into the SoA batch layout.

``History pid inv resp = [(pid, Either inv resp)]`` (src/Linearisability.hs:18)
becomes one 16-byte header plus 8 bytes per event (include/qsmd.h).  Pids are
only compared for equality by the reference (``Eq pid``, :30-45), so each
history maps its pids to dense ids 0..n_pid-1 in order of first use; the
verdict cannot depend on the choice.  Bank accounts are mapped likewise
(models.Bank.new_account_map).  A history that cannot be encoded is emitted
with ``model_id = 0xFF`` and no events, which every checker reports as
QSMD_STATUS_ENCODE_ERROR.
"""

from __future__ import annotations

import numpy as np

from .models import EncodeError

HDR_DTYPE = np.dtype([("ev_off", "<u4"), ("n_ev", "<u2"), ("n_pid", "u1"),
                      ("model_id", "u1"), ("tag", "<u4"), ("reserved", "<u4")])
EV_DTYPE = np.dtype([("kp", "u1"), ("code", "u1"), ("a", "u1"), ("b", "u1"),
                     ("val", "<i4")])
WF_DTYPE = np.dtype([("code", "u1"), ("pid", "u1"), ("ev0", "<u2"), ("ev1", "<u2"), ("reserved", "<u2")])
assert HDR_DTYPE.itemsize == 16 and EV_DTYPE.itemsize == 8 and WF_DTYPE.itemsize == 8

# qsmd_wf.code -> NotSequential constructor (src/Linearisability.hs:97-104)
WF_KINDS = {1: "FirstEventIsntInvocation", 2: "InvocationFollowedByInvocation",
            3: "InvocationFollowedByNonMatchingResponse", 4: "ResponseFollowedByResponse",
            5: "ResponseFollowedByInvocation", 6: "LoneResponse"}
WF_ENCODE_ERROR = 0xFE


def encode_shape(histories):
    """Only the shape of a batch (pid and kind of every event, payloads
    dropped) with ONE dense pid map for the whole batch, in first-use order,
    as `wellformed` needs: the same `pids` list applies to every history.
    Returns (hdr, events, pid_index dict)."""
    pid_index = {}
    hdr = np.zeros(len(histories), dtype=HDR_DTYPE)
    kps = []
    off = 0
    for i, h in enumerate(histories):
        for pid, (kind, _) in h:
            q = pid_index.setdefault(pid, len(pid_index))
            if q >= 128:
                raise ValueError("more than 128 distinct pids in the batch")
            kps.append(q | (0x80 if kind == "R" else 0))
        hdr[i]["ev_off"] = off
        hdr[i]["n_ev"] = len(h)
        off += len(h)
    hdr["n_pid"] = max(len(pid_index), 1)
    events = np.zeros(off, dtype=EV_DTYPE)
    events["kp"] = np.array(kps, dtype=np.uint8) if kps else 0
    return hdr, events, pid_index

MAX_EVENTS = 128
MAX_PIDS = 128
EV_RESP = 0x80
BAD_MODEL = 0xFF

STATUS_NONLIN = 0
STATUS_LIN = 1
STATUS_MODEL_ERROR = 2
STATUS_ENCODE_ERROR = 3
STATUS_BUDGET = 4
STATUS_SKIPPED = 5
STATUS_NAMES = {0: "nonlin", 1: "lin", 2: "error", 3: "encode", 4: "budget", 5: "skipped"}

WITNESS_END = 0xFF


def Left(x):           # noqa: N802  (Haskell constructor names)
    return ("L", x)


def Right(x):          # noqa: N802
    return ("R", x)


class Batch:
    """An encoded batch: ``hdr`` (n_hist,) HDR_DTYPE, ``events`` (n_events,)
    EV_DTYPE, plus per-history pid / account maps for decoding."""

    def __init__(self, model, hdr, events, pid_maps, account_maps, model0=None,
                 encode_errors=None):
        self.model = model
        self.hdr = hdr
        self.events = events
        self.pid_maps = pid_maps
        self.account_maps = account_maps
        self.model0 = model0
        self.encode_errors = encode_errors or {}

    def __len__(self):
        return len(self.hdr)


def _encode_one(model, history, model0):
    pids = {}
    accounts = model.new_account_map(model0)
    evs = []
    if len(history) > MAX_EVENTS:
        raise EncodeError(f"{len(history)} events > {MAX_EVENTS}")
    for pid, ev in history:
        if pid not in pids:
            if len(pids) >= MAX_PIDS:
                raise EncodeError("more than 128 pids")
            pids[pid] = len(pids)
        p = pids[pid]
        kind, x = ev
        if kind == "L":
            code, a, b, val = model.encode_inv(x, accounts)
            evs.append((p, code, a, b, val))
        elif kind == "R":
            code, val = model.encode_resp(x)
            evs.append((EV_RESP | p, code, 0, 0, val))
        else:
            raise EncodeError(f"not an Either: {ev!r}")
    return evs, pids, accounts


def encode(model, histories, model0=None):
    """Encode a list of histories for ``model`` (a models.DeviceModel)."""
    hdr = np.zeros(len(histories), dtype=HDR_DTYPE)
    chunks, pid_maps, account_maps, errors = [], [], [], {}
    off = 0
    for i, h in enumerate(histories):
        try:
            evs, pids, accounts = _encode_one(model, h, model0)
        except EncodeError as exc:
            errors[i] = str(exc)
            hdr[i] = (off, 0, 0, BAD_MODEL, i, 0)
            pid_maps.append({})
            account_maps.append({})
            continue
        hdr[i] = (off, len(evs), len(pids), model.model_id, i, 0)
        chunks.extend(evs)
        pid_maps.append(pids)
        account_maps.append(accounts)
        off += len(evs)
    events = np.array(chunks, dtype=EV_DTYPE) if chunks else np.zeros(0, dtype=EV_DTYPE)
    return Batch(model, hdr, events, pid_maps, account_maps, model0, errors)


def decode_history(batch, i):
    """Rebuild history ``i`` (with dense pids replaced by the originals)."""
    h = batch.hdr[i]
    inv_pid = {v: k for k, v in batch.pid_maps[i].items()}
    out = []
    model = batch.model
    for e in batch.events[h["ev_off"]: h["ev_off"] + h["n_ev"]]:
        pid = inv_pid[int(e["kp"]) & 0x7F]
        if int(e["kp"]) & EV_RESP:
            out.append((pid, ("R", model.decode_resp(int(e["code"]), int(e["val"])))))
        else:
            out.append((pid, ("L", model.decode_inv(int(e["code"]), int(e["a"]), int(e["b"]),
                                                    int(e["val"]), batch.account_maps[i]))))
    return out
