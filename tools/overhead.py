"""Fixed per-call cost of the cascade (verdict r01 item 5): device time of a
call (first event before stage 0 -> event after the giant stage) and host
wall time per synchronous call, on tiny batches of config 2 with the default
parameters.  One call is 4 launches (stage 0, stage 0w, the heavy stage,
the giant stage); with nothing to do, the last three return at once.

    python tools/overhead.py [--calls 300] [--param NAME=VALUE ...]
Prints one JSON line per batch size.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--param", action="append", default=[], metavar="NAME=VALUE", help="qsmd_set_param")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = device.Context(0)
    for kv in args.param:
        k, v = kv.split("=")
        ctx.set_param(k, int(v))
    stream = torch.cuda.current_stream(dev).cuda_stream
    mid = gen.CONFIGS["bank_4x16"]["model_id"]
    for n in (1, 64, 4096):
        hdr, ev, _ = gen.generate_config("bank_4x16", 0, n)
        d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).to(dev)
        d_ev = torch.from_numpy(ev.view(np.uint8).copy()).to(dev)
        d_st = torch.empty(n, dtype=torch.uint8, device=dev)
        d_nd = torch.empty(n, dtype=torch.int64, device=dev)

        def call():
            ctx.check_device(mid, d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st.data_ptr(), d_nd.data_ptr(),
                             stream=stream)

        for _ in range(20):
            call()
        torch.cuda.synchronize()
        ctx.timing_reset()
        for _ in range(args.calls):
            call()
        torch.cuda.synchronize()
        s0, dev_ms = ctx.timing_read()
        walls = []
        for _ in range(args.calls):
            t = time.perf_counter()
            call()
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t)
        ok = bool((d_st.cpu().numpy() == 1).all())
        print(json.dumps({"n_hist": n, "launches_per_call": 4,
                          "device_us_median": round(1e3 * float(np.median(dev_ms)), 2),
                          "stage0_us_median": round(1e3 * float(np.median(s0)), 2),
                          "sync_wall_us_median": round(1e6 * float(np.median(walls)), 2),
                          "all_linearisable": ok}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
