"""Interleaved A/B timing of search-kernel tuning knobs in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Usage on the GPU box:
    python tools/sweep.py [--config bank_4x16] [--n 1000000] [--rounds 5]
Prints, per variant, the median / min stage-0 kernel time over all rounds."""

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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grids", default="65536")
    ap.add_argument("--budgets", default="64", help="stage-0 node budgets (0 = none)")
    ap.add_argument("--no-stamps", action="store_true")
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
    variants = [(int(g), int(b)) for g in args.grids.split(",") for b in args.budgets.split(",")]
    res = {v: ([], []) for v in variants}
    for _ in range(args.rounds):
        for g, b in variants:
            ctx.set_stage0_grid(g)
            ctx.set_stage0_budget(b)
            ctx.timing_reset()
            for _ in range(args.reps):
                ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev),
                                 d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
            s0, call = ctx.timing_read()
            res[(g, b)][0].extend(float(x) for x in s0)
            res[(g, b)][1].extend(float(x) for x in call)
    out = {f"grid{g}_budget{b}": {"stage0_median_ms": float(np.median(v[0])),
                                  "call_median_ms": float(np.median(v[1])),
                                  "call_min_ms": float(np.min(v[1]))} for (g, b), v in res.items()}
    if args.no_stamps:
        print(json.dumps({"config": args.config, "n": args.n, "variants": out}, indent=1))
        return
    # diagnostic build: per-phase s_memtime cycles per 64-history group
    g0 = min((args.n + 63) // 64, 65536)
    st = torch.zeros(g0 * 8, dtype=torch.int64, device=dev)
    ctx.set_stage0_grid(65536)
    ctx.set_stage0_budget(0)
    ctx.diag_stamps(st.data_ptr())
    ctx.timing_reset()
    ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev),
                     d_st.data_ptr(), d_nd.data_ptr(), None, None, stream=stream)
    s0, _ = ctx.timing_read()
    ctx.diag_stamps(None)
    raw = st.view(g0, 8).cpu().numpy()
    stamps = raw[:, :4].astype(np.float64)
    # residency: waves resident per SIMD over the kernel (realtime 100 MHz)
    t0, t1 = raw[:, 4], raw[:, 5]
    hw, xcc = raw[:, 6], raw[:, 7]
    simd = (xcc & 0xF) * 10**6 + ((hw >> 13) & 7) * 10**4 + ((hw >> 12) & 1) * 10**3 + \
        ((hw >> 8) & 0xF) * 10 + ((hw >> 4) & 3)
    span = float(t1.max() - t0.min())
    n_simd = len(np.unique(simd))
    resid = {"span_us": span / 100.0, "simds_seen": int(n_simd),
             "mean_waves_per_simd": float((t1 - t0).sum() / span / max(n_simd, 1)),
             "wave_life_us_p50_p90_max": [float(np.percentile(t1 - t0, q)) / 100.0 for q in (50, 90, 100)],
             "start_spread_us": float(np.percentile(t0 - t0.min(), 99)) / 100.0}
    groups = stamps[:, 3].sum()
    nd = d_nd.cpu().numpy()
    diag = {"stamped_kernel_ms": float(s0[0]),
            "cycles_per_group": {"stage": stamps[:, 0].sum() / groups, "search": stamps[:, 1].sum() / groups,
                                 "output": stamps[:, 2].sum() / groups},
            "search_cycles_p50_p90_max": [float(np.percentile(stamps[:, 1], q)) for q in (50, 90, 100)],
            "nodes_mean": float(nd.mean()), "nodes_group_max_mean": float(nd.reshape(-1, 64).max(1).mean())
            if args.n % 64 == 0 else None, "residency": resid}
    print(json.dumps({"config": args.config, "n": args.n, "variants": out, "diag": diag}, indent=1))


if __name__ == "__main__":
    main()
