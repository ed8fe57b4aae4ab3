"""Interleaved A/B timing of named tuning parameters (qsmd_set_param) in ONE
process, with a parity check of every variant against the first.
    python tools/sweep_params.py --config bank_4x16 \
        --variants 'stage0_persistent_grid=0;stage0_persistent_grid=2048,refill_min=8'
Prints JSON: per variant the median / min device time of the whole call."""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402

DEFAULTS = {"stage0_persistent_grid": 0, "refill_min": 8, "split_budget": 1024, "stage0_auto": 1,
            "stage0_grid": 65536}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="bank_4x16")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", required=True)
    ap.add_argument("--memo", action="store_true")
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
    flags = device.QSMD_FLAG_EXHAUSTIVE | (device.QSMD_FLAG_MEMO if args.memo else 0)
    variants = []
    for v in args.variants.split(";"):
        kv = dict(DEFAULTS)
        for item in filter(None, v.split(",")):
            k, x = item.split("=")
            kv[k.strip()] = int(x)
        variants.append((v, kv))
    res = {v: ([], []) for v, _ in variants}
    ref = None
    parity = {}
    for rnd in range(args.rounds):
        for name, kv in variants:
            for k, x in kv.items():
                ctx.set_param(k, x)
            ctx.timing_reset()
            for _ in range(args.reps):
                ctx.check_device(cfg["model_id"], d_hdr.data_ptr(), args.n, d_ev.data_ptr(), len(ev),
                                 d_st.data_ptr(), d_nd.data_ptr(), None, None, flags=flags, stream=stream)
            s0, call = ctx.timing_read()
            res[name][0].extend(float(x) for x in s0)
            res[name][1].extend(float(x) for x in call)
            if rnd == 0:
                torch.cuda.synchronize()
                got = (d_st.cpu().numpy().copy(), d_nd.cpu().numpy().copy())
                if ref is None:
                    ref = got
                parity[name] = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
    out = {name: {"stage0_median_ms": float(np.median(v[0])), "call_median_ms": float(np.median(v[1])),
                  "call_min_ms": float(np.min(v[1])), "parity_vs_first": parity[name]}
           for name, v in res.items()}
    print(json.dumps({"config": args.config, "n": args.n, "variants": out}, indent=1), flush=True)


if __name__ == "__main__":
    main()
