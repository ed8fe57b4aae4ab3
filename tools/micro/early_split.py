"""Where the early-exit leg's step goes (bench.py --early-exit, one rank):
the whole qsmd.dist.check_shard_early_exit_device call against its floor,
the first round's qsmd_check_batch_device call alone (launch + wait), and
a bare torch D2H read for scale."""
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
status = torch.empty(n, dtype=torch.uint8, device=dev)
nodes = torch.empty(n, dtype=torch.int64, device=dev)
tot = torch.empty(8, dtype=torch.int64, device=dev)


def per_call(f, reps=100):
    for _ in range(10):
        f()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps * 1e6


for fc in (None, 4096, 1024):
    us = per_call(lambda: qdist.check_shard_early_exit_device(ctx, mid, d_hdr, d_ev, len(ev), n, 0, 1, first_chunk=fc))
    print(f"whole call, first_chunk {fc}: {us:.1f} us")
for m in (4096, 262144):
    def one():
        ctx.check_device(mid, d_hdr.data_ptr(), m, d_ev.data_ptr(), len(ev), status.data_ptr(), nodes.data_ptr(),
                         None, tot.data_ptr(), flags=flags)
        torch.cuda.synchronize(dev)
    print(f"qsmd_check_batch_device over {m} + wait: {per_call(one):.1f} us")
print(f"torch 64-byte D2H read: {per_call(lambda: tot.cpu()):.1f} us")
