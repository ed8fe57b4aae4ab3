"""Debug one history through group_search sharing: dump the victim's state,
the emitted range tasks and the deciders' keys (diagnostic tool)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("quickcheck-state-machine-distributed_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch
import oracle_c
from qsmd import device, gen, models
ctx = device.Context(0)
hdr, ev, _ = gen.generate_config("bank_4x16", 0, 50000)
for i in (530, 22712):
    h1 = hdr[i:i+1].copy()
    o = int(h1[0]["ev_off"]); n = int(h1[0]["n_ev"])
    e1 = ev[o:o+n].copy(); h1[0]["ev_off"] = 0
    print("history", i, "events:")
    for k, x in enumerate(e1):
        print("  ", k, "R" if x["kp"] & 0x80 else "L", "pid", x["kp"] & 0x7F, "code", x["code"], "a", x["a"], "b", x["b"], "val", x["val"])
    st_o, nd_o, w_o = oracle_c.check_batch(2, h1, e1, witness=True)
    dbg = torch.zeros(256 * 4, dtype=torch.int64, device="cuda")
    ctx.set_param("stage0_kernel", 1); ctx.set_param("group_debug_ptr", dbg.data_ptr())
    st, nd, w, _ = ctx.check_arrays(2, h1, e1, witness=True)
    ctx.set_param("group_debug_ptr", 0); ctx.set_param("stage0_kernel", 0)
    d = dbg[:256].cpu().numpy().astype(np.uint64)
    print("dev", st[0], nd[0], list(w[:17]), "oracle", st_o[0], nd_o[0], list(w_o[:17]))
    print("victim nodes", d[0], "depth", d[1] & 0xFF, "found", (d[1] >> 8) & 0xFF, "k", (d[1] >> 16) & 0xFFFF,
          "cand", hex(int(d[1] >> 32)), "rem", hex(int(d[2] & 0xFFFFFFFF)), "paired", d[2] >> 32)
    stk = b"".join(int(x).to_bytes(4, "little") for x in d[3:7])
    print("stack", [b & 31 for b in stk[:int(d[1] & 0xFF)]])
    k = int((d[1] >> 16) & 0xFFFF)
    for e in range(min(k, 20)):
        hi, lo, cm, rm = d[8 + e*4: 12 + e*4]
        digs = [(int(hi) >> (56 - 7*q)) & 127 for q in range(9)] + [(int(lo) >> (56 - 7*q)) & 127 for q in range(7)]
        print("  entry", e, "cand", hex(int(cm) & 0xFFFFFFFF), "depth", (int(cm) >> 32) & 0xFF, "found", (int(cm) >> 40) & 1,
              "rem", hex(int(rm)), "digits", digs)
    nd_ = int(d[200])
    for q in range(nd_):
        hi, lo = int(d[201+2*q]), int(d[202+2*q])
        print("  decider", [(hi >> (56 - 7*t)) & 127 for t in range(9)] + [(lo >> (56 - 7*t)) & 127 for t in range(7)])
