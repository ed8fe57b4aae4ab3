"""Latency of one lane's search when its wavefront is alone: the histories of
config 2 that need > 64 nodes, checked as their own batch (diagnostic)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("quickcheck-state-machine-distributed_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import oracle_c
from qsmd import device, gen
hdr, ev, _ = gen.generate_config("bank_4x16", 0, 1_000_000, threads=16)
st, nd, _ = oracle_c.check_batch(2, hdr, ev, threads=16)
sel = np.nonzero(nd > 64)[0]
n = len(sel)
h2 = hdr[sel].copy()
ev2 = np.concatenate([ev[int(hdr[i]["ev_off"]): int(hdr[i]["ev_off"]) + int(hdr[i]["n_ev"])] for i in sel])
h2["ev_off"] = np.arange(n, dtype=np.uint32) * 32
ctx = device.Context(0)
ctx.set_stage0_budget(0)
out = {"n": int(n), "max_nodes": int(nd[sel].max()), "mean_nodes": float(nd[sel].mean())}
for variant in ({"stage0_kernel": 0}, {"stage0_kernel": 1, "share_nodes": 8}, {"stage0_kernel": 0, "stage0_budget": 8, "heavy_stage": 0},
                {"stage0_kernel": 0, "stage0_budget": 8, "heavy_stage": 1, "spread_budget": 16}):
    for k, v in variant.items():
        ctx.set_param(k, v)
    ctx.timing_reset()
    for _ in range(5):
        s2, n2, _, _ = ctx.check_arrays(2, h2, ev2)
    s0, call = ctx.timing_read()
    assert np.array_equal(n2, nd[sel]) and np.array_equal(s2, st[sel])
    out[json.dumps(variant)] = {"stage0_ms": float(np.median(s0)), "call_ms": float(np.median(call))}
    ctx.set_param("stage0_kernel", 0)
    ctx.set_stage0_budget(0)
print(json.dumps(out, indent=1))
