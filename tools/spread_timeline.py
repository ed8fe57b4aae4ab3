"""Spread-stage task timeline (diagnostic build path: spread_stamps_ptr):
per task s_memrealtime (100 MHz) at slot assignment, start, search start,
end.  Prints the distribution of wait / setup / search times and the span.
    python tools/spread_timeline.py --config bank_4x16 --stage0 64 --budget 128"""

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
    ap.add_argument("--config", default="bank_4x16")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--stage0", type=int, default=64)
    ap.add_argument("--budget", type=int, default=128)
    ap.add_argument("--grid", type=int, default=2048)
    args = ap.parse_args()
    cfg = gen.CONFIGS[args.config]
    hdr, ev, _ = gen.generate_config(args.config, 0, args.n, threads=16)
    dev = torch.device("cuda", 0)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(args.n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(args.n, dtype=torch.int64, device=dev)
    ctx = device.Context(0)
    cap = 1 << 22
    stamps = torch.zeros(cap * 4, dtype=torch.int64, device=dev)
    ctx.set_param("stage0_budget", args.stage0)
    ctx.set_param("spread_budget", args.budget)
    ctx.set_param("spread_grid", args.grid)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for it in range(2):
        if it == 1:
            stamps.zero_()
            ctx.set_param("spread_stamps_ptr", stamps.data_ptr())
        ctx.timing_reset()
        ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev),
                         d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
        torch.cuda.synchronize()
    ctx.set_param("spread_stamps_ptr", 0)
    s0, call = ctx.timing_read()
    st = ctx.spread_stats()
    n_tasks = st[1]
    t = stamps.view(cap, 4)[:n_tasks].cpu().numpy().astype(np.int64)
    t0 = t[:, 0].min()
    us = lambda x: (x / 100.0)
    ok = t[:, 2] > 0
    def pct(x):
        return [round(float(np.percentile(x, q)), 2) for q in (50, 90, 99, 100)] if len(x) else []
    out = {"call_ms": float(call[0]), "stage0_ms": float(s0[0]), "tasks": n_tasks, "searched": int(ok.sum()),
           "span_us": us(float(t[:, 3].max() - t0)),
           "wait_us_p50_90_99_max": pct(us(t[:, 1] - t[:, 0])),
           "setup_us": pct(us(t[ok, 2] - t[ok, 1])),
           "search_us": pct(us(t[ok, 3] - t[ok, 2])),
           "search_us_total": us(float((t[ok, 3] - t[ok, 2]).sum())),
           "reference_nodes": st[3],
           "start_offset_us": pct(us(t[:, 1] - t0)),
           "end_offset_us": pct(us(t[:, 3] - t0))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
