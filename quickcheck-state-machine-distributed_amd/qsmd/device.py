"""ctypes binding of the C ABI (include/qsmd.h) -> lib/libqsmd.so.

This is the product path: there is no CPU fallback.  If the HIP library is
missing or no GPU is visible, every entry point raises.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import codec

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("QSMD_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libqsmd.so")   # (A/B builds: tools/ab.py)

QSMD_FLAG_EXHAUSTIVE = 1
QSMD_FLAG_MEMO = 2
QSMD_FLAG_WITNESS = 4
QSMD_FLAG_EARLY_EXIT_BATCH = 8


class DeviceError(RuntimeError):
    pass


QSMD_SPLIT_MAX_DEPTH = 16
TASK_WITNESS_BYTES = 64

# qsmd_task / qsmd_frontier (include/qsmd.h, split search)
TASK_DTYPE = np.dtype([("hist", "<u4"), ("depth", "<u2"), ("reserved", "<u2"),
                       ("top_before", "<u8"), ("path", "u1", (QSMD_SPLIT_MAX_DEPTH,))])
assert TASK_DTYPE.itemsize == 32


class Frontier(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("depth", ctypes.c_uint32),
                ("top_nodes", ctypes.c_uint64), ("n_tasks", ctypes.c_uint64)]


class Totals(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "checked", "linearisable", "nonlinearisable", "model_errors", "encode_errors",
        "budget", "skipped", "nodes")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_lib = None

_P = ctypes.c_void_p
_U32, _U64, _I = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int

EXPORTS = {
    "qsmd_abi_version": (_U32, []),
    "qsmd_open": (_I, [ctypes.POINTER(_P), _I]),
    "qsmd_close": (None, [_P]),
    "qsmd_last_error": (ctypes.c_char_p, [_P]),
    "qsmd_set_time_limit_ms": (_I, [_P, _U64]),
    "qsmd_set_stage0_grid": (_I, [_P, _U64]),
    "qsmd_set_stage0_budget": (_I, [_P, _U64]),
    "qsmd_probe_read": (_I, [_P, _P]),
    "qsmd_timed_out": (_I, [_P, _P]),
    "qsmd_wellformed_batch": (_I, [_P, _P, _U64, _P, _U64, _P, _U32, _P]),
    "qsmd_wellformed_batch_device": (_I, [_P, _P, _U64, _P, _U64, _P, _U32, _P, _P]),
    "qsmd_gen_batch_device": (_I, [_P, _P, _U64, _U64, _U32, _P, _P, _P, _P]),   # include/qsmd_gen.h
    "qsmd_check_batch": (_I, [_P, _U32, _P, _U64, _P, _U64, _P, _U32, _U64, _P, _P, _P, _P]),
    "qsmd_check_batch_device": (_I, [_P, _U32, _P, _U64, _P, _U64, _P, _U32, _U64, _P, _P, _P, _P, _P]),
    "qsmd_last_kernel_ms": (_I, [_P, ctypes.POINTER(ctypes.c_float)]),
    "qsmd_timing_reset": (_I, [_P]),
    "qsmd_timing_read": (_I, [_P, _P, _P, _U64, ctypes.POINTER(_U64)]),
    "qsmd_timing_read_stages": (_I, [_P, _P, _P, _P, _U64, ctypes.POINTER(_U64)]),
    "qsmd_get_param": (_I, [_P, ctypes.c_char_p, ctypes.POINTER(_U64)]),
    "qsmd_set_split_budget": (_I, [_P, _U64]),
    "qsmd_set_param": (_I, [_P, ctypes.c_char_p, _U64]),
    "qsmd_set_memo_capacity": (_I, [_P, _U64]),
    "qsmd_split_frontier": (_I, [_P, _U32, _P, _P, _U64, _P, _U32, _U64, _U32, _P, _U64, _P, _P]),
    "qsmd_check_tasks": (_I, [_P, _U32, _P, _P, _U64, _P, _U32, _U64, _P, _U64, _P, _P, _P]),
    "qsmd_combine_tasks": (_I, [_P, _P, _P, _P, _U64, _U64, _P, _P, _P]),
}


def combine_tasks(frontier, tasks, status, nodes, max_nodes=0):
    """Fold task results in DFS order (qsmd_combine_tasks: host code of the
    library, no device).  Returns (status, nodes, winner index or -1)."""
    lib = load_library()
    tasks = np.ascontiguousarray(tasks, dtype=TASK_DTYPE)
    status = np.ascontiguousarray(status, dtype=np.uint8)
    nodes = np.ascontiguousarray(nodes, dtype=np.uint64)
    st, nd, win = ctypes.c_uint8(), ctypes.c_uint64(), ctypes.c_int64()
    n = len(tasks)
    if len(status) != n or len(nodes) != n:
        raise ValueError("one status and one node count per task")
    rc = lib.qsmd_combine_tasks(ctypes.byref(frontier), _ptr(tasks) if n else None,
                                _ptr(status) if n else None, _ptr(nodes) if n else None, n,
                                int(max_nodes), ctypes.byref(st), ctypes.byref(nd), ctypes.byref(win))
    if rc != 0:
        raise DeviceError(f"qsmd_combine_tasks failed ({rc})")
    return int(st.value), int(nd.value), int(win.value)


def load_library(path=LIB_PATH):
    """Load lib/libqsmd.so and declare every exported symbol."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DeviceError(f"{path} not built: run `make -C {PKG_DIR}` (no CPU fallback exists)")
    # One HIP runtime per process: PyTorch-ROCm bundles its own
    # libamdhip64.so (SONAME libamdhip64.so.7).  Importing torch first makes
    # libqsmd.so bind to that same runtime, so torch device memory, streams
    # and torch.distributed (RCCL) interoperate with our kernels; without
    # torch the library uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(arr):
    return None if arr is None else ctypes.c_void_p(arr.ctypes.data)


# The host entry's CPython fast path (csrc/pyfast.c: the buffers through the
# buffer protocol, one C call of qsmd_check_batch); without it, ctypes.
try:
    from . import _pyfast
except ImportError:
    _pyfast = None


class Context:
    """One context per GPU (one process per GPU)."""

    def __init__(self, device=0, time_limit_ms=None):
        lib = load_library()
        h = ctypes.c_void_p()
        rc = lib.qsmd_open(ctypes.byref(h), int(device))
        if rc != 0:
            raise DeviceError(f"qsmd_open(device={device}) failed with {rc}: no usable HIP device")
        self._h = h
        self._lib = lib
        self._check_fn = ctypes.cast(lib.qsmd_check_batch, ctypes.c_void_p).value
        if time_limit_ms is not None:
            lib.qsmd_set_time_limit_ms(h, int(time_limit_ms))

    def close(self):
        if self._h:
            self._lib.qsmd_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self._lib.qsmd_last_error(self._h)
            raise DeviceError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def check_arrays(self, model_id, hdr, events, model0=None, flags=QSMD_FLAG_EXHAUSTIVE,
                     max_nodes=0, witness=False):
        """Host-memory batch (numpy arrays in the include/qsmd.h layout).
        Returns (status u8[n], nodes u64[n], witness u8[n_events] or None, totals dict)."""
        hdr = np.ascontiguousarray(hdr, dtype=codec.HDR_DTYPE)
        events = np.ascontiguousarray(events, dtype=codec.EV_DTYPE)
        n = len(hdr)
        status = np.empty(n, dtype=np.uint8)
        nodes = np.empty(n, dtype=np.uint64)
        wit = np.full(len(events), 0xFF, dtype=np.uint8) if witness else None
        if witness:
            flags |= QSMD_FLAG_WITNESS
        tot = Totals()
        if _pyfast is not None:
            rc = _pyfast.check_batch(self._check_fn, (self._h.value or 0) if self._h else 0, int(model_id), hdr,
                                     events, ctypes.addressof(model0) if model0 is not None else 0, int(flags),
                                     int(max_nodes), status, nodes, wit, tot)
        else:
            m0 = ctypes.cast(ctypes.pointer(model0), ctypes.c_void_p) if model0 is not None else None
            rc = self._lib.qsmd_check_batch(
                self._h, model_id, _ptr(hdr) if n else None, n,
                _ptr(events) if len(events) else None, len(events), m0, flags, max_nodes,
                _ptr(status) if n else None, _ptr(nodes) if n else None,
                _ptr(wit) if (wit is not None and len(events)) else None, ctypes.byref(tot))
        self._check(rc, "qsmd_check_batch")
        return status, nodes, wit, tot.as_dict()

    def check_device(self, model_id, hdr_ptr, n_hist, events_ptr, n_events, status_ptr,
                     nodes_ptr=None, witness_ptr=None, totals_ptr=None, model0=None,
                     flags=QSMD_FLAG_EXHAUSTIVE, max_nodes=0, stream=None):
        """Device-resident batch: raw device pointers (ints), async on stream."""
        m0 = ctypes.cast(ctypes.pointer(model0), ctypes.c_void_p) if model0 is not None else None
        rc = self._lib.qsmd_check_batch_device(
            self._h, model_id, hdr_ptr, n_hist, events_ptr, n_events, m0, flags, max_nodes,
            status_ptr, nodes_ptr, witness_ptr, totals_ptr, stream)
        self._check(rc, "qsmd_check_batch_device")

    def last_kernel_ms(self):
        ms = ctypes.c_float()
        self._check(self._lib.qsmd_last_kernel_ms(self._h, ctypes.byref(ms)), "qsmd_last_kernel_ms")
        return float(ms.value)

    def set_time_limit_ms(self, ms):
        """qsmd_set_time_limit_ms: the safety net's wall time per search launch
        (0 disables)."""
        self._check(self._lib.qsmd_set_time_limit_ms(self._h, int(ms)), "qsmd_set_time_limit_ms")

    def set_stage0_grid(self, max_blocks):
        self._check(self._lib.qsmd_set_stage0_grid(self._h, int(max_blocks)), "qsmd_set_stage0_grid")

    def set_param(self, name, value):
        self._check(self._lib.qsmd_set_param(self._h, name.encode(), int(value)), f"qsmd_set_param({name})")

    def set_split_budget(self, nodes):
        self._check(self._lib.qsmd_set_split_budget(self._h, int(nodes)), "qsmd_set_split_budget")

    def set_memo_capacity(self, entries):
        self._check(self._lib.qsmd_set_memo_capacity(self._h, int(entries)), "qsmd_set_memo_capacity")

    @staticmethod
    def _one(hdr, events):
        hdr = np.ascontiguousarray(hdr, dtype=codec.HDR_DTYPE)
        events = np.ascontiguousarray(events, dtype=codec.EV_DTYPE)
        if len(hdr) != 1:
            raise ValueError("the split search takes exactly one history")
        return hdr, events

    def split_frontier(self, model_id, hdr, events, model0=None, flags=QSMD_FLAG_EXHAUSTIVE,
                       max_nodes=0, min_tasks=64, max_tasks=4096, witness=False):
        """Cut the search of one history (qsmd_split_frontier).
        Returns (Frontier, tasks TASK_DTYPE[n], witness u8[n_ev] or None)."""
        hdr, events = self._one(hdr, events)
        tasks = np.zeros(max(int(max_tasks), 1), dtype=TASK_DTYPE)
        fr = Frontier()
        n_ev = int(hdr[0]["n_ev"])
        wit = np.full(max(n_ev, 1), 0xFF, dtype=np.uint8) if witness else None
        m0 = ctypes.cast(ctypes.pointer(model0), ctypes.c_void_p) if model0 is not None else None
        rc = self._lib.qsmd_split_frontier(
            self._h, model_id, _ptr(hdr), _ptr(events) if len(events) else None, len(events), m0, flags,
            int(max_nodes), int(min_tasks), _ptr(tasks), int(max_tasks), ctypes.byref(fr),
            _ptr(wit) if wit is not None else None)
        self._check(rc, "qsmd_split_frontier")
        return fr, tasks[: fr.n_tasks].copy(), (wit[:n_ev] if wit is not None else None)

    def check_tasks(self, model_id, hdr, events, tasks, model0=None, flags=QSMD_FLAG_EXHAUSTIVE,
                    max_nodes=0, witness=False):
        """Search task subtrees of one history (qsmd_check_tasks).
        Returns (status u8[n], nodes u64[n], witness u8[n, 64] or None)."""
        hdr, events = self._one(hdr, events)
        tasks = np.ascontiguousarray(tasks, dtype=TASK_DTYPE)
        n = len(tasks)
        status = np.empty(n, dtype=np.uint8)
        nodes = np.empty(n, dtype=np.uint64)
        wit = np.full((n, TASK_WITNESS_BYTES), 0xFF, dtype=np.uint8) if witness else None
        m0 = ctypes.cast(ctypes.pointer(model0), ctypes.c_void_p) if model0 is not None else None
        rc = self._lib.qsmd_check_tasks(
            self._h, model_id, _ptr(hdr), _ptr(events) if len(events) else None, len(events), m0, flags,
            int(max_nodes), _ptr(tasks) if n else None, n, _ptr(status) if n else None,
            _ptr(nodes) if n else None, _ptr(wit) if (wit is not None and n) else None)
        self._check(rc, "qsmd_check_tasks")
        return status, nodes, wit

    def set_stage0_budget(self, nodes):
        self._check(self._lib.qsmd_set_stage0_budget(self._h, int(nodes)), "qsmd_set_stage0_budget")

    def wellformed_arrays(self, hdr, events, pids=None):
        """Batched `wellformed` (include/qsmd.h qsmd_wellformed_batch) on host
        arrays; pids = dense pid indices in `pids` order, None = all.
        Returns a codec.WF_DTYPE array."""
        hdr = np.ascontiguousarray(hdr, dtype=codec.HDR_DTYPE)
        events = np.ascontiguousarray(events, dtype=codec.EV_DTYPE)
        out = np.zeros(len(hdr), dtype=codec.WF_DTYPE)
        pl = None
        if pids is not None:
            pl = np.ascontiguousarray(pids, dtype=np.uint8)
        rc = self._lib.qsmd_wellformed_batch(
            self._h, _ptr(hdr) if len(hdr) else None, len(hdr), _ptr(events) if len(events) else None,
            len(events), _ptr(pl) if pl is not None and len(pl) else None,
            0 if pl is None else len(pl), _ptr(out) if len(hdr) else None)
        self._check(rc, "qsmd_wellformed_batch")
        return out

    def wellformed_device(self, hdr_ptr, n_hist, events_ptr, n_events, out_ptr, pids=None, stream=None):
        """Device-resident batched `wellformed` (async on stream)."""
        pl = None if pids is None else np.ascontiguousarray(pids, dtype=np.uint8)
        rc = self._lib.qsmd_wellformed_batch_device(
            self._h, hdr_ptr, n_hist, events_ptr, n_events, _ptr(pl) if pl is not None and len(pl) else None,
            0 if pl is None else len(pl), out_ptr, stream)
        self._check(rc, "qsmd_wellformed_batch_device")

    def gen_device(self, params, first, n_hist, hdr_ptr, events_ptr, bug_ptr=None, ev_base=0, stream=None):
        """On-device synthetic generation (include/qsmd_gen.h
        qsmd_gen_batch_device): the qsmd.gen stream [first, first + n_hist),
        byte-identical to the host generator, into device buffers (async)."""
        rc = self._lib.qsmd_gen_batch_device(self._h, ctypes.byref(params), first, n_hist, ev_base, hdr_ptr,
                                             events_ptr, bug_ptr, stream)
        self._check(rc, "qsmd_gen_batch_device")

    def probe(self):
        """Routing of the most recent check call (qsmd_probe_read): histories
        stage 0 passed to stage 0w, heavy histories of stages 0 and 0w,
        giants."""
        out = (ctypes.c_uint32 * 4)()
        self._check(self._lib.qsmd_probe_read(self._h, out), "qsmd_probe_read")
        return dict(zip(("deferred", "heavy32", "heavy64", "giants"), (int(x) for x in out)))

    def timed_out(self):
        """True when the time limit fired in the most recent check call (its
        QSMD_STATUS_BUDGET results then include unfinished searches, not only
        max_nodes ones)."""
        out = ctypes.c_int(0)
        self._check(self._lib.qsmd_timed_out(self._h, ctypes.byref(out)), "qsmd_timed_out")
        return bool(out.value)

    def timing_reset(self):
        self._check(self._lib.qsmd_timing_reset(self._h), "qsmd_timing_reset")

    def timing_read(self, max_calls=1024):
        """(stage0_ms, call_ms) arrays for the calls since timing_reset()."""
        s0, _, call = self.timing_read_stages(max_calls)
        return s0, call

    def timing_read_stages(self, max_calls=1024):
        """(stage0_ms, heavy_ms, call_ms) arrays for the calls since
        timing_reset(); heavy_ms = the lane-mode heavy-stage kernel (-1 in
        wave mode)."""
        s0 = np.zeros(max_calls, dtype=np.float32)
        hv = np.zeros(max_calls, dtype=np.float32)
        call = np.zeros(max_calls, dtype=np.float32)
        n = ctypes.c_uint64()
        self._check(self._lib.qsmd_timing_read_stages(self._h, _ptr(s0), _ptr(hv), _ptr(call), max_calls,
                                                      ctypes.byref(n)), "qsmd_timing_read_stages")
        return s0[: n.value], hv[: n.value], call[: n.value]

    def get_param(self, name):
        """qsmd_get_param: a knob's value, or "stage0_budget_last"."""
        out = ctypes.c_uint64()
        self._check(self._lib.qsmd_get_param(self._h, name.encode(), ctypes.byref(out)), f"qsmd_get_param({name})")
        return int(out.value)


_default = None


def default_context():
    global _default
    if _default is None:
        _default = Context(0)
    return _default
