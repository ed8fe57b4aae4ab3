"""Where the early-exit leg's step goes (bench.py --early-exit): host time
of each piece of qsmd.dist._early_rounds, unsynchronised (the Python/launch
cost) and synchronised after each piece (its device time on top)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "quickcheck-state-machine-distributed_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402
from qsmd import dist as qdist  # noqa: E402

dev = torch.device("cuda:0")
n = 1_250_000
hdr, ev, _ = gen.generate(gen.params(**gen.CONFIGS["bank_4x16_bugs"]), 0, n, threads=16)
d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
mid = gen.CONFIGS["bank_4x16_bugs"]["model_id"]
ctx = device.Context(0)
flags = device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_EARLY_EXIT_BATCH
s = torch.cuda.Stream(dev)


def pieces(sync):
    T = {}
    t = time.perf_counter

    def mark(k, t0):
        if sync:
            torch.cuda.synchronize(dev)
        T[k] = T.get(k, 0.0) + (t() - t0) * 1e6
        return t()

    t0 = t()
    st_ = torch.cuda.Stream(dev)
    t0 = mark("stream", t0)
    with torch.cuda.stream(s):
        status = torch.full((n,), 5, dtype=torch.uint8, device=dev)
        nodes = torch.zeros(n, dtype=torch.int64, device=dev)
        tot = torch.zeros((4, 8), dtype=torch.int64, device=dev)
        local = torch.full((1,), n, dtype=torch.int64, device=dev)
        searched = torch.zeros((), dtype=torch.int64, device=dev)
        t0 = mark("alloc", t0)
        ctx.check_device(mid, d_hdr.data_ptr(), 4096, d_ev.data_ptr(), len(ev), status.data_ptr(), nodes.data_ptr(),
                         None, tot[0].data_ptr(), flags=flags, stream=s.cuda_stream)
        t0 = mark("check_device", t0)
        tk = tot[0]
        ff = (4096 - 1) - tk[6]
        local = torch.where((tk[2] + tk[3]) > 0, torch.minimum(local, ff), local)
        searched += 4096 - tk[6]
        t0 = mark("torch_ops", t0)
        best = int(local.item())
        local.fill_(best)
        t0 = mark("item", t0)
        status[best + 1:] = 5
        nodes[best + 1:] = 0
        t0 = mark("mark", t0)
        tt = torch.zeros(8, dtype=torch.int64, device=dev)
        bc = torch.bincount(status.to(torch.int64), minlength=6)
        tt[1], tt[2], tt[3], tt[4], tt[5], tt[6] = bc[1], bc[0], bc[2], bc[3], bc[4], bc[5]
        tt[0] = bc[0] + bc[1] + bc[2]
        tt[7] = nodes.sum()
        t0 = mark("totals", t0)
        int(searched.item())
        t0 = mark("searched_item", t0)
    torch.cuda.synchronize(dev)
    return T


for sync in (False, True):
    for _ in range(5):
        pieces(sync)
    acc = {}
    for _ in range(50):
        for k, v in pieces(sync).items():
            acc[k] = acc.get(k, 0.0) + v / 50
    print("sync" if sync else "async", {k: round(v, 1) for k, v in acc.items()}, "sum %.1f" % sum(acc.values()))

t0 = time.perf_counter()
for _ in range(50):
    qdist.check_shard_early_exit_device(ctx, mid, d_hdr, d_ev, len(ev), n, 0, 1, first_chunk=4096)
torch.cuda.synchronize(dev)
print("whole call us %.1f" % ((time.perf_counter() - t0) / 50 * 1e6))
