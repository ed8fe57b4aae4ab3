"""Spread-stage diagnostics: per variant (qsmd_set_param settings), the device
time of one call and the spread stage's task / explored-node counts.
    python tools/spread_diag.py --config bank_4x16 --variants 'stage0_budget=64;stage0_budget=64,spread_budget=32'"""

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

DEFAULTS = {"stage0_auto": 1, "spread_budget": 1024, "spread_grid": 1024, "refill_min": 8, "heavy_stage": 2,
            "coop_budget": 16, "coop_grid": 2048}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="bank_4x16")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", required=True)
    ap.add_argument("--coop-stats", action="store_true", help="diagnostic coop counters (one extra call)")
    args = ap.parse_args()
    cfg = gen.CONFIGS[args.config]
    hdr, ev, _ = gen.generate_config(args.config, 0, args.n, threads=16)
    dev = torch.device("cuda", 0)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(args.n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(args.n, dtype=torch.int64, device=dev)
    ctx = device.Context(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ref = None
    for v in args.variants.split(";"):
        kv = dict(DEFAULTS)
        for item in filter(None, v.split(",")):
            k, x = item.split("=")
            kv[k.strip()] = int(x)
        for k, x in kv.items():
            ctx.set_param(k, x)
        ctx.timing_reset()
        walls = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev),
                             d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t)
        s0, call = ctx.timing_read()
        stats = ctx.spread_stats()
        got = (d_st.cpu().numpy().copy(), d_nd.cpu().numpy().copy())
        if ref is None:
            ref = got
        par = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
        cstats = None
        if args.coop_stats:
            grid = kv.get("coop_grid", 2048)
            buf = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
            ctx.set_param("spread_stamps_ptr", buf.data_ptr())
            ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev),
                             d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
            torch.cuda.synchronize()
            ctx.set_param("spread_stamps_ptr", 0)
            q = buf.view(grid, 8).cpu().numpy()
            hist = int(q[:, 0].sum())
            cstats = {"histories": hist, "iters_mean": float(q[:, 1].sum() / max(hist, 1)),
                      "iters_wave_max": int(q[:, 1].max()), "iters_hist_max": int(q[:, 6].max()),
                      "splits": int(q[:, 2].sum()), "nosplit": int(q[:, 3].sum()), "compactions": int(q[:, 4].sum()),
                      "tasks": int(q[:, 5].sum()), "nodes": int(q[:, 7].sum())}
        print(json.dumps({"coop": cstats, "variant": v, "stage0_ms": round(float(np.median(s0)), 4),
                          "call_ms": round(float(np.median(call)), 4), "wall_ms": round(1e3 * min(walls), 3),
                          "spread": {"histories": stats[0], "tasks": stats[1], "explored": stats[2],
                                     "reference_nodes": stats[3]}, "parity_vs_first": par}), flush=True)


if __name__ == "__main__":
    main()
