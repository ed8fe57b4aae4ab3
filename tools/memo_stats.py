"""Memo-stage counters on a config (default config 3): iterations, memo hits
and inserts of the memo stage in the cascade's steady state."""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="bank_4x16_bugs")
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--set", default="", help="k=v,... parameters")
args = ap.parse_args()
cfg = gen.CONFIGS[args.config]
hdr, ev, _ = gen.generate_config(args.config, 0, args.n, threads=16)
dev = torch.device("cuda", 0)
d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
d_st = torch.empty(args.n, dtype=torch.uint8, device=dev)
d_nd = torch.empty(args.n, dtype=torch.int64, device=dev)
ctx = device.Context(0)
for item in filter(None, args.set.split(",")):
    k, v = item.split("=")
    ctx.set_param(k, int(v))
stream = torch.cuda.current_stream(dev).cuda_stream


def call():
    ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev), d_st.data_ptr(),
                     d_nd.data_ptr(), None, None, stream=stream)


for _ in range(4):
    call()
torch.cuda.synchronize()
buf = torch.zeros(4, dtype=torch.int64, device=dev)
ctx.set_param("memo_stats_ptr", buf.data_ptr())
ctx.timing_reset()
call()
torch.cuda.synchronize()
ctx.set_param("memo_stats_ptr", 0)
s0, cl = ctx.timing_read()
it, hits, ins, mx = (int(x) for x in buf.cpu().numpy()[:4])
nd = d_nd.cpu().numpy()
print(json.dumps({"config": args.config, "set": args.set, "iterations": it, "hits": hits, "inserts": ins, "max_iters": mx,
                  "stage0_ms": round(float(s0[-1]), 4), "call_ms": round(float(cl[-1]), 4),
                  "nodes": int(nd.sum()), "over_64": int((nd > 64).sum())}))
