"""Where a lone stage 0 spends its time (diagnostic build QSMD_DIAG_STAGE0=2:
tools/build_variant.sh s0stamp "-DQSMD_DIAG_STAGE0=2").

Runs `calls` synchronous calls of config 2 (bench knobs: stage-0 budget 26)
and, for the last one, reads each stage-0 group's stamps: s_memtime at the
group's start / after staging / after the search, s_memrealtime at the start
and after the search, the wave's DFS iterations.  Prints per-group phase
cycles and a timeline (how many groups are staging / searching per 5 us).

    QSMD_LIB_PATH=ablib/s0stamp.so python tools/stage0_anatomy.py [n_hist] [budget]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qsmd import device, gen  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    budget = int(sys.argv[2]) if len(sys.argv) > 2 else 26
    name = "bank_4x16"
    dev = torch.device("cuda:0")
    hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    groups = (n + 63) // 64
    stamps = torch.zeros(groups * 8, dtype=torch.int64, device=dev)
    ctx = device.Context(0)
    ctx.set_stage0_budget(budget)
    ctx.set_param("heavy_mode", 1)
    ctx.set_param("memo_lds", 0)
    try:
        ctx.set_param("stage0_stamps_ptr", stamps.data_ptr())
    except Exception:                                   # (a build without the knob)
        pass
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        try:
            ctx.set_param(k, int(v))
        except Exception:                               # (a build without the knob)
            print(f"no knob {k}", file=sys.stderr)
    s = torch.cuda.current_stream().cuda_stream
    ctx.timing_reset()
    for _ in range(8):
        ctx.check_device(gen.CONFIGS[name]["model_id"], d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev),
                         d_st.data_ptr(), d_nd.data_ptr(), stream=s)
        torch.cuda.synchronize()
    s0, call = ctx.timing_read()
    st = stamps.cpu().numpy().reshape(groups, 8).astype(np.int64)
    ctx.close()
    raw = os.environ.get("QSMD_STAMPS_OUT")
    if raw:
        np.save(raw, st)
    mt0, mt1, mt2, rt0, rt2, it = (st[:, k] for k in range(6))
    ok = (mt0 > 0) & (rt0 > 0)
    if not ok.any():                                    # a build without stamps: the event times only
        print(json.dumps({"stage0_ms_events": [float(x) for x in s0], "call_ms": [float(x) for x in call]}))
        return
    mt0, mt1, mt2, rt0, rt2, it = mt0[ok], mt1[ok], mt2[ok], rt0[ok], rt2[ok], it[ok]
    stage = mt1 - mt0
    search = mt2 - mt1
    life_us = (rt2 - rt0) / 100.0                       # s_memrealtime: 100 MHz
    t_us = (rt0 - rt0.min()) / 100.0
    end_us = (rt2 - rt0.min()) / 100.0
    pct = lambda x: {q: float(np.percentile(x, q)) for q in (5, 50, 95, 99)}  # noqa: E731
    out = {
        "groups": int(ok.sum()), "stage0_ms_events": float(np.mean(s0[-4:])), "call_ms": float(np.mean(call[-4:])),
        "span_us_stamps": float(end_us.max()),
        "staging_cycles": {"mean": float(stage.mean()), **{f"p{k}": v for k, v in pct(stage).items()}},
        "search_cycles": {"mean": float(search.mean()), **{f"p{k}": v for k, v in pct(search).items()}},
        "search_frac_of_group": float(search.sum() / (stage.sum() + search.sum())),
        "group_life_us": {"mean": float(life_us.mean()), **{f"p{k}": v for k, v in pct(life_us).items()}},
        "dfs_iterations": {"mean": float(it.mean()), **{f"p{k}": v for k, v in pct(it).items()}},
        "cycles_per_iteration": float(search.sum() / max(1, it.sum())),
        "start_us": {f"p{k}": v for k, v in pct(t_us).items()},
    }
    # timeline: groups alive per 5 us bucket, and the share of them staging
    rt1 = rt0 + (mt1 - mt0) * 0.0                       # (staging end in realtime: scaled below)
    scale = (rt2 - rt0) / np.maximum(1, mt2 - mt0)      # realtime ticks per cycle, per group
    rt1 = rt0 + (mt1 - mt0) * scale
    base = rt0.min()
    tl = []
    for b in range(0, int(end_us.max()) + 5, 5):
        lo, hi = base + b * 100, base + (b + 5) * 100
        alive = int(((rt0 < hi) & (rt2 > lo)).sum())
        staging = int(((rt0 < hi) & (rt1 > lo)).sum())
        tl.append((b, alive, staging))
    out["timeline_5us"] = tl
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
