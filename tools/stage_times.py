"""Per-stage device timing of one check call on a generated configuration
(QSMD_SYNC_STAGES=1 prints each launch's time and the routing counters).

    QSMD_SYNC_STAGES=1 python tools/stage_times.py bank_4x16 1000000 [param=value ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    name, n = sys.argv[1], int(sys.argv[2])
    ctx = device.Context(0)
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        ctx.set_param(k, int(v))
    hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
    dev = torch.device("cuda:0")
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ctx.timing_reset()   # (timing events on)
    for i in range(4):
        t = time.perf_counter()
        ctx.check_device(gen.CONFIGS[name]["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                         d_st.data_ptr(), d_nd.data_ptr(), stream=s)
        torch.cuda.synchronize()
        print(f"call {i}: {1e3 * (time.perf_counter() - t):.3f} ms wall, {ctx.last_kernel_ms():.3f} ms device, "
              f"{ctx.probe()}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
