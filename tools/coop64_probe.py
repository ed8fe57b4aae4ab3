"""coop64 on the heaviest 48-event histories: time and cooperative-stage
counters per variant (stage0w_budget, coop_budget).
    python tools/coop64_probe.py [--top 32]"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="bank_6x24")
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--top", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    cfg = gen.CONFIGS[args.config]
    hdr, ev, _ = gen.generate_config(args.config, 0, args.n, threads=16)
    ctx = device.Context(0)
    st, nd, _, _ = ctx.check_arrays(cfg["model_id"], hdr, ev)
    top = np.argsort(nd)[::-1][:args.top]
    sub = hdr[np.sort(top)].copy()
    print(json.dumps({"top_nodes": [int(x) for x in nd[top][:8]], "sum": int(nd[top].sum())}), flush=True)
    dev = torch.device("cuda", 0)
    d_hdr = torch.from_numpy(sub.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    n = len(sub)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ref = None
    for wb in (0, 16, 64, 256):
        for cb in (4, 16, 64):
            if wb == 0 and cb != 16:
                continue
            ctx.set_param("stage0w_budget", wb)
            ctx.set_param("coop_budget", cb)
            ctx.timing_reset()
            for _ in range(args.reps):
                ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                                 d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
            torch.cuda.synchronize()
            _, call = ctx.timing_read()
            got = (d_st.cpu().numpy().copy(), d_nd.cpu().numpy().copy())
            ref = ref or got
            par = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
            buf = torch.zeros(512 * 8, dtype=torch.int64, device=dev)
            ctx.set_param("spread_stamps_ptr", buf.data_ptr())
            ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                             d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
            torch.cuda.synchronize()
            ctx.set_param("spread_stamps_ptr", 0)
            q = buf.view(512, 8).cpu().numpy()
            hist = int(q[:, 0].sum())
            cs = {"histories": hist, "iters_hist_max": int(q[:, 6].max()), "iters_mean": float(q[:, 1].sum() / max(hist, 1)),
                  "splits": int(q[:, 2].sum()), "nosplit": int(q[:, 3].sum()), "compactions": int(q[:, 4].sum()),
                  "tasks": int(q[:, 5].sum()), "nodes": int(q[:, 7].sum())}
            print(json.dumps({"stage0w_budget": wb, "coop_budget": cb, "call_ms": round(float(np.median(call)), 4),
                              "parity": par, "coop": cs}), flush=True)
    ctx.set_param("stage0w_budget", 0)
    ctx.set_param("coop_budget", 16)


if __name__ == "__main__":
    main()
