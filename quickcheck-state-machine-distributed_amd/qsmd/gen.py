"""Synthetic history generator (include/qsmd_gen.h -> lib/libqsmd_gen.so).

Restates the reference's history producer (deterministic scheduler,
src/Scheduler.hs:105-186; generators test/Bank.hs:133-146,
test/TicketDispenser.hs:108-112).  Deterministic per (seed, history index),
so rank r of N can generate its own shard of one global stream.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import codec
from .models import MODEL_BANK, MODEL_TICKET

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                        "libqsmd_gen.so")

LIN_AT_INVOKE = 0
LIN_IN_WINDOW = 1
PID_PER_CLIENT = 0
PID_SHARED = 1


class GenParams(ctypes.Structure):
    _fields_ = [("model_id", ctypes.c_uint32), ("n_clients", ctypes.c_uint32),
                ("n_ops", ctypes.c_uint32), ("prefix_ops", ctypes.c_uint32),
                ("lin_policy", ctypes.c_uint32), ("pid_mode", ctypes.c_uint32),
                ("overlap", ctypes.c_uint32), ("money_max", ctypes.c_uint32),
                ("p_bug", ctypes.c_double), ("seed", ctypes.c_uint64)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (make -C the package directory)")
        L = ctypes.CDLL(LIB_PATH)
        L.qsmd_gen_batch.restype = ctypes.c_int
        L.qsmd_gen_batch.argtypes = [ctypes.POINTER(GenParams), ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


# The BASELINE.json configurations.
CONFIGS = {
    # (1) TicketDispenser parallel property, 2 clients x ~10 ops, one shared pid (Q1)
    "ticket_2x10": dict(model_id=MODEL_TICKET, n_clients=2, n_ops=10, prefix_ops=4,
                        lin_policy=LIN_AT_INVOKE, pid_mode=PID_SHARED, seed=15),
    # (2) Bank 4 clients x 16 ops, linearisable
    "bank_4x16": dict(model_id=MODEL_BANK, n_clients=4, n_ops=16, prefix_ops=4,
                      lin_policy=LIN_IN_WINDOW, pid_mode=PID_PER_CLIENT, seed=0x5EED),
    # (3) Bank mixed histories with injected race bugs
    "bank_4x16_bugs": dict(model_id=MODEL_BANK, n_clients=4, n_ops=16, prefix_ops=4,
                           lin_policy=LIN_IN_WINDOW, pid_mode=PID_PER_CLIENT, p_bug=0.5, seed=0xB06),
    # (4) adversarial TicketDispenser 8 clients x 64 ops, heavy overlap
    "ticket_8x64": dict(model_id=MODEL_TICKET, n_clients=8, n_ops=64, prefix_ops=1,
                        lin_policy=LIN_IN_WINDOW, pid_mode=PID_PER_CLIENT, overlap=8, seed=0x8C64),
    # (5) Bank 6 clients x 24 ops, overlap <= 4, exhaustive node-count parity
    "bank_6x24": dict(model_id=MODEL_BANK, n_clients=6, n_ops=24, prefix_ops=6,
                      lin_policy=LIN_IN_WINDOW, pid_mode=PID_PER_CLIENT, overlap=4, seed=0x6C24),
}


def params(**kw):
    p = GenParams()
    p.money_max = 100
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def generate(p, first, n_hist, threads=8, ev_base=0):
    """Return (hdr, events, bug) numpy arrays for histories [first, first+n_hist)."""
    lib = _load()
    per = 2 * p.n_ops
    hdr = np.zeros(n_hist, dtype=codec.HDR_DTYPE)
    events = np.zeros(n_hist * per, dtype=codec.EV_DTYPE)
    bug = np.zeros(n_hist, dtype=np.uint8)
    rc = lib.qsmd_gen_batch(ctypes.byref(p), first, n_hist, ev_base, hdr.ctypes.data,
                            events.ctypes.data, bug.ctypes.data, threads)
    if rc != 0:
        raise ValueError(f"qsmd_gen_batch rejected the parameters ({rc})")
    return hdr, events, bug


def adversarial_ticket(n_clients=8, n_ops=64, bug=True):
    """BASELINE config 4: one TicketDispenser history, n_clients x n_ops with
    the heaviest overlap, every event on the test process's pid (Q1,
    test/TicketDispenser.hs:302-309).  After a sequential Reset, TakeTickets
    are invoked n_clients at a time and answered in order.  Every pending
    TakeTicket is a candidate child with the same successor state, so the
    reference search tree has (n_clients!)^(n_ops / n_clients) paths; with
    `bug` the last Number is off by one, the history is non-linearisable and
    the exhaustive search must visit all of them -- only state memoisation
    (QSMD_FLAG_MEMO) makes it tractable.  Returns (hdr[1], events, bug[1])."""
    ev = [(0x00, 1, 0, 0, 0), (0x80, 1, 0, 0, 0)]          # L Reset, R Ok
    n, left = 0, n_ops - 1
    while left > 0:
        w = min(n_clients, left)
        ev += [(0x00, 0, 0, 0, 0)] * w                     # L TakeTicket
        ev += [(0x80, 0, 0, 0, n + 1 + i) for i in range(w)]   # R Number
        n += w
        left -= w
    if bug:
        k, c, a, b, v = ev[-1]
        ev[-1] = (k, c, a, b, v + 1)
    events = np.array(ev, dtype=codec.EV_DTYPE)
    hdr = np.zeros(1, dtype=codec.HDR_DTYPE)
    hdr[0] = (0, len(ev), 1, MODEL_TICKET, 0, 0)
    return hdr, events, np.array([1 if bug else 0], dtype=np.uint8)


def plant_failure(hdr, events, i):
    """A copy of `events` in which history i fails: its last response becomes
    `Balance 2^20` (Bank), a value no interleaving explains -- the injected
    race bug of the early-exit leg's planted stream (bench.py --plant, tests
    test_distributed.py).  The history keeps its shape."""
    ev = events.copy()
    o, n = int(hdr[i]["ev_off"]), int(hdr[i]["n_ev"])
    resp = [k for k in range(o, o + n) if ev["kp"][k] & 0x80]
    k = resp[-1]
    ev["code"][k] = 7                                   # Balance
    ev["val"][k] = 1 << 20
    return ev


def generate_config(name, first, n_hist, threads=8, **override):
    kw = dict(CONFIGS[name])
    kw.update(override)
    return generate(params(**kw), first, n_hist, threads)
