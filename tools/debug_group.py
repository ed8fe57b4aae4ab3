"""Debug: group_search vs oracle on generated histories; prints mismatches
with witnesses (diagnostic tool)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("quickcheck-state-machine-distributed_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import oracle_c
from qsmd import device, gen, models
name = sys.argv[1] if len(sys.argv) > 1 else "bank_4x16"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
ctx = device.Context(0)
hdr, ev, _ = gen.generate_config(name, 0, n)
mid = gen.CONFIGS[name]["model_id"]
st_o, nd_o, w_o = oracle_c.check_batch(mid, hdr, ev, threads=8, witness=True)
for variant in ({"stage0_kernel": 1}, {"stage0_kernel": 1, "share_nodes": 1000},
                {"stage0_kernel": 1, "group_budget": 1000}, {"stage0_kernel": 1, "share_idle": 60}):
    for k, v in variant.items():
        ctx.set_param(k, v)
    st, nd, w, tot = ctx.check_arrays(mid, hdr, ev, witness=True)
    bad = np.nonzero((st != st_o) | (nd != nd_o))[0]
    print(variant, "mismatches", len(bad), flush=True)
    for i in bad[:4]:
        a, b = int(hdr[i]["ev_off"]), int(hdr[i]["ev_off"]) + int(hdr[i]["n_ev"])
        print("  h", i, "st", st[i], st_o[i], "nodes", nd[i], nd_o[i])
        print("   wit dev", list(w[a:b][:17]), "\n   wit ora", list(w_o[a:b][:17]))
    for k in variant:
        ctx.set_param(k, {"stage0_kernel": 0, "share_nodes": 32, "group_budget": 16, "share_idle": 16}[k])
