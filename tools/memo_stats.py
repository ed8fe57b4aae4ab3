"""Heavy-stage (lane mode) diagnostics on a generated configuration: per
group of 64 histories, the wall time from its start to its staging and to its
last history, the DFS iterations of its longest lane, memo hits and shader
cycles per iteration, and the wavefront's cycles per iteration in each phase
of the DFS step (memo_stats_ptr, memo.hip PhaseClock: each phase drained of
its memory operations before its end stamp, so the phases add up to more
than the undrained loop; one diagnostic call after warm-up).

    python tools/memo_stats.py bank_4x16 1000000 [param=value ...]
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
    name, n = sys.argv[1], int(sys.argv[2])
    ctx = device.Context(0)
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        ctx.set_param(k, int(v))
    dev = torch.device("cuda:0")
    hdr, ev, _ = gen.generate_config(name, 0, n, threads=16)
    mid = gen.CONFIGS[name]["model_id"]
    d_hdr = torch.from_numpy(hdr.view(np.uint8)).to(dev)
    d_ev = torch.from_numpy(ev.view(np.uint8)).to(dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    d_nd = torch.empty(n, dtype=torch.int64, device=dev)
    groups = (n + 63) // 64
    W = 16                                  # u64 per group (memo.hip kMemoStatsWords)
    stats = torch.zeros(groups * W, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def call():
        ctx.check_device(mid, d_hdr.data_ptr(), n, d_ev.data_ptr(), len(ev), d_st.data_ptr(), d_nd.data_ptr(),
                         stream=stream)

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_param("memo_stats_groups", groups)
    ctx.set_param("memo_stats_ptr", stats.data_ptr())
    call()
    torch.cuda.synchronize()
    ctx.set_param("memo_stats_ptr", 0)
    s0, dev_ms = ctx.timing_read()
    q = stats.view(groups, W).cpu().numpy().astype(np.int64)
    q = q[q[:, 6] > 0]
    if len(q) == 0:
        print(json.dumps({"groups": 0}))
        return
    t0 = q[:, 0].min()
    start = (q[:, 0] - t0) / 100.0          # s_memrealtime: 100 MHz -> us
    staged = (q[:, 1] - q[:, 0]) / 100.0
    span = (q[:, 2] - q[:, 0]) / 100.0
    end = (q[:, 2] - t0) / 100.0
    it = np.maximum(q[:, 3], 1)
    cyc_per_it = q[:, 7] / it
    worst = int(np.argmax(end))
    out = {
        "config": name, "histories": n, "groups": int(len(q)), "heavy_histories": int(q[:, 6].sum()),
        "call_device_us": round(1e3 * float(dev_ms[-1]), 1), "stage0_us": round(1e3 * float(s0[-1]), 1),
        "stage_span_us": round(float(end.max()), 1),
        "group_start_us_max": round(float(start.max()), 1),
        "staging_us_median": round(float(np.median(staged)), 2),
        "group_span_us": {"median": round(float(np.median(span)), 1), "max": round(float(span.max()), 1)},
        "max_iterations": {"median": int(np.median(q[:, 3])), "p90": int(np.percentile(q[:, 3], 90)),
                           "p99": int(np.percentile(q[:, 3], 99)), "max": int(q[:, 3].max())},
        "iterations_total": int(q[:, 4].sum()),
        "lane_utilisation": round(float(q[:, 4].sum()) / float((q[:, 3] * 64).sum()), 3),
        "iterations_per_history": {"mean": round(float(q[:, 4].sum()) / float(q[:, 6].sum()), 1)},
        "max_over_mean_per_group": {"median": round(float(np.median(q[:, 3] / np.maximum(q[:, 4] / np.maximum(q[:, 6], 1), 1))), 2)},
        "memo_hits_total": int(q[:, 5].sum()),
        "cycles_per_iteration": {"median": round(float(np.median(cyc_per_it)), 0),
                                 "of_longest_group": round(float(cyc_per_it[worst]), 0)},
        "longest_group": {"start_us": round(float(start[worst]), 1), "staging_us": round(float(staged[worst]), 2),
                          "span_us": round(float(span[worst]), 1), "max_iterations": int(q[worst, 3]),
                          "histories": int(q[worst, 6])},
    }
    wave_it = max(int(q[:, 15].sum()), 1)
    names = ("backtrack", "try_next", "memo_slot", "hbm_probe")
    out["phase_cycles_per_wave_iteration"] = {k: round(float(q[:, 8 + i].sum()) / wave_it, 0)
                                              for i, k in enumerate(names)}
    # LaneDFS::fold against the balances it folds, after every try (must be 0)
    out["fold_mismatch_wave_iterations"] = int(q[:, 12].sum())
    out["wave_iterations"] = wave_it
    out["fraction_of_wave_iterations"] = {"with_backtrack": round(float(q[:, 13].sum()) / wave_it, 3),
                                          "with_hbm_probe": round(float(q[:, 14].sum()) / wave_it, 3)}
    lw = worst
    wl = max(int(q[lw, 15]), 1)
    out["longest_group"]["phase_cycles_per_iteration"] = {k: round(float(q[lw, 8 + i]) / wl, 0)
                                                          for i, k in enumerate(names)}
    out["longest_group"]["with_hbm_probe"] = round(float(q[lw, 14]) / wl, 3)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
