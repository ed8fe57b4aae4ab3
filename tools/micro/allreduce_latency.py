"""One rank: the wall time of the bench's end-of-window exchange pieces.
  rccl: one all-reduce of the 8 int64 totals on a stream of its own, launched
        while the GPU is idle, then synchronised;
  d2h:  the 64-B device-to-host copy of the totals (synchronous);
  gloo: one all-reduce of the 64-B host tensor over a gloo group.
    python tools/micro/allreduce_latency.py [rccl|gloo]"""
import os
import sys
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("TORCH_NCCL_ENABLE_MONITORING", "0")
os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
mode = sys.argv[1] if len(sys.argv) > 1 else "rccl"
dist.init_process_group("nccl" if mode == "rccl" else "gloo", rank=0, world_size=1)
dev = torch.device("cuda:0")
t = torch.zeros(8, dtype=torch.int64, device=dev)
s = torch.cuda.Stream(dev)


def med(f, n=50):
    for _ in range(5):
        f()
    xs = []
    for _ in range(n):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        f()
        xs.append((time.perf_counter() - t0) * 1e6)
    xs.sort()
    return round(xs[n // 2], 1)


def rccl():
    with torch.cuda.stream(s):
        dist.all_reduce(t)
    torch.cuda.synchronize(dev)


h = torch.zeros(8, dtype=torch.int64)
out = {"d2h_us": med(lambda: t.cpu())}
if mode == "rccl":
    out["rccl_allreduce_us"] = med(rccl)
else:
    g = dist.new_group(backend="gloo")
    out["gloo_allreduce_us"] = med(lambda: dist.all_reduce(h, group=g))
    out["gloo_default_group_us"] = med(lambda: dist.all_reduce(h))
print(out)
dist.destroy_process_group()
