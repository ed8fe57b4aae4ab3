"""Device time of the first calls and the steady state per config (default
parameters, fresh context per config): the adaptive cascade's first call has
no probe yet.  Prints one JSON line per config."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402

for name, n in (("bank_4x16", 1_000_000), ("ticket_2x10", 1_000_000), ("bank_4x16_bugs", 1_000_000),
                ("bank_6x24", 100_000)):
    cfg = gen.CONFIGS[name]
    hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
    dev = torch.device("cuda", 0)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    ctx = device.Context(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    times = []
    for i in range(8):
        ctx.timing_reset()
        ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st.data_ptr(),
                         d_nd.data_ptr(), None, None, stream=stream)
        torch.cuda.synchronize()
        times.append(round(float(np.median(ctx.timing_read()[1])), 4))
    print(json.dumps({"config": name, "n": n, "call_ms": times, "nodes": int(d_nd.sum().item())}), flush=True)
    ctx.close()
