"""Throughput of the batched `wellformed` kernel on BASELINE config 2 (1M
4x16 Bank histories resident in HBM): HIP-event time per launch and the
achieved HBM rate on its bytes (16 B header + 8 B per event in, 8 B out)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))
import numpy as np
import torch
from qsmd import device, gen
n = 1_000_000
hdr, ev, _ = gen.generate_config("bank_4x16", 0, n, threads=16)
dev = torch.device("cuda:0")
d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
d_out = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
ctx = device.Context(0)
s = torch.cuda.current_stream()
for _ in range(3):
    ctx.wellformed_device(d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_out.data_ptr(), stream=s.cuda_stream)
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
t0.record(s)
for _ in range(reps):
    ctx.wellformed_device(d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_out.data_ptr(), stream=s.cuda_stream)
t1.record(s)
torch.cuda.synchronize()
ms = t0.elapsed_time(t1) / reps
byts = n * 16 + len(ev) * 8 + n * 8
print(json.dumps({"kernel": "wellformed_kernel", "histories": n, "ms_per_launch": ms,
                  "histories_per_s": n / ms * 1e3, "bytes_per_launch": byts,
                  "achieved_GBs": byts / ms / 1e6, "peak_GBs": 8000.0, "frac": byts / ms / 1e6 / 8000.0}))
