"""Fixed per-call cost: device time of a call on a tiny batch (64 histories
of config 2), default parameters vs the rare stages switched off."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402

n = 64
hdr, ev, _ = gen.generate_config("bank_4x16", 0, n)
dev = torch.device("cuda", 0)
d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
d_st = torch.empty(n, dtype=torch.uint8, device=dev)
d_nd = torch.empty(n, dtype=torch.int64, device=dev)
ctx = device.Context(0)
stream = torch.cuda.current_stream(dev).cuda_stream
for name, kv in (("default", {}), ("no_split", {"split_budget": 0}), ("no_0w", {"stage0w": 0}),
                 ("no_memo", {"memo_stage": 0}), ("none", {"split_budget": 0, "stage0w": 0, "memo_stage": 0})):
    for k, v in kv.items():
        ctx.set_param(k, v)
    ctx.timing_reset()
    for _ in range(200):
        ctx.check_device(1, d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st.data_ptr(), d_nd.data_ptr(),
                         None, None, stream=stream)
    torch.cuda.synchronize()
    s0, call = ctx.timing_read()
    print(json.dumps({"variant": name, "stage0_us": round(1e3 * float(np.median(s0)), 2),
                      "call_us": round(1e3 * float(np.median(call)), 2)}), flush=True)
    for k in kv:
        ctx.set_param(k, {"split_budget": 1024, "stage0w": 1, "memo_stage": 1}[k])
