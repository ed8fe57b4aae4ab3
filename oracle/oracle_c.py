"""ctypes loader for the C oracle (oracle/ref_cpu.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libqsmd_oracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_check_batch.restype = ctypes.c_int
        L.oracle_check_batch.argtypes = [
            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int]
        L.oracle_check_batch_flags.restype = ctypes.c_int
        L.oracle_check_batch_flags.argtypes = L.oracle_check_batch.argtypes + [ctypes.c_uint32]
        _lib = L
    return _lib


def check_batch(model_id, hdr, events, model0=None, max_nodes=0, threads=1, witness=False, memo=False):
    """Run the oracle.  hdr/events are numpy arrays in the include/qsmd.h
    layout; model0 is None or a ctypes struct.  memo=True prunes known-failing
    states (verdicts exact, node counts not the reference's).  Returns
    (status, nodes, witness_or_None)."""
    n = len(hdr)
    hdr = np.ascontiguousarray(hdr)
    events = np.ascontiguousarray(events)
    status = np.zeros(n, dtype=np.uint8)
    nodes = np.zeros(n, dtype=np.uint64)
    wit = np.full(max(len(events), 1), 0xFF, dtype=np.uint8) if witness else None
    m0 = ctypes.cast(ctypes.pointer(model0), ctypes.c_void_p) if model0 is not None else None
    lib().oracle_check_batch_flags(
        model_id, hdr.ctypes.data, n, events.ctypes.data if len(events) else None,
        m0, max_nodes, status.ctypes.data, nodes.ctypes.data,
        wit.ctypes.data if wit is not None else None, threads, 2 if memo else 0)
    return status, nodes, wit
