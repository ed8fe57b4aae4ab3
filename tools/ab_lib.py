"""A/B two builds of libqsmd.so on one config, interleaved in two processes'
worth of contexts is not possible (one HIP library per process), so this runs
ONE library (path argument) and prints the steady-state call time; run it
once per build inside the same GPU job.
    python tools/ab_lib.py <lib.so> <config> [n]"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402

lib, name = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
device.LIB_PATH = lib
cfg = gen.CONFIGS[name]
hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
dev = torch.device("cuda", 0)
d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
d_st = torch.empty(n, dtype=torch.uint8, device=dev)
d_nd = torch.empty(n, dtype=torch.int64, device=dev)
ctx = device.Context(0)
stream = torch.cuda.current_stream(dev).cuda_stream
for _ in range(5):
    ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st.data_ptr(),
                     d_nd.data_ptr(), None, None, stream=stream)
torch.cuda.synchronize()
ctx.timing_reset()
for _ in range(30):
    ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st.data_ptr(),
                     d_nd.data_ptr(), None, None, stream=stream)
torch.cuda.synchronize()
s0, call = ctx.timing_read()
print(json.dumps({"lib": os.path.basename(lib), "config": name, "stage0_ms": round(float(np.median(s0)), 4),
                  "call_ms": round(float(np.median(call)), 4), "nodes": int(d_nd.sum().item())}))
