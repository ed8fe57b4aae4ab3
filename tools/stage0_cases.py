"""Stage-0 kernel timing cases (diagnostic, run under rocprofv3 --kernel-trace):
one device-resident batch, each case's knobs + max_nodes, `reps` calls each,
synchronised, in the order given.  Case syntax: NAME:k=v,k=v[,max=N]

    python tools/stage0_cases.py bank_4x16 1000000 5 base:stage0_budget=40 t16:stage0_budget=16 u16:max=16
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quickcheck-state-machine-distributed_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    name, n, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    hdr, ev, _ = gen.generate_config(name, 0, n)
    mid = gen.CONFIGS[name]["model_id"]
    dev = torch.device("cuda:0")
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8).copy()).to(dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    nd = torch.empty(n, dtype=torch.int64, device=dev)
    ctx = device.Context(0)
    for case in sys.argv[4:]:
        label, _, spec = case.partition(":")
        max_nodes = 0
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            if k == "max":
                max_nodes = int(v)
            else:
                ctx.set_param(k, int(v))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.check_device(mid, d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), st.data_ptr(), nd.data_ptr(),
                             max_nodes=max_nodes, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"{label}: {dt * 1e3:.3f} ms/call, nodes {int(nd.sum())}, budget-status {int((st == 4).sum())}",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
