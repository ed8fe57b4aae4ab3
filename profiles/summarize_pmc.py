"""Summarise a profiles/profile.sh run: per-dispatch durations (kernel trace)
and PMC counters of the two search kernels that bound a call -- stage 0
(compact_search<..., G32>) and the lane-mode heavy stage (memo_search) --
over the LAST `--last` dispatches of each: bench.py's roofline leg, the
synchronous calls it times after its timed region, so that the profile's
mean durations are the ones bench.py's `roofline.kernels.*.kernel_ms.mean`
divide by.  The whole-run rocprofv3 --stats table is kept beside it
(`kernels`; its means include the launches that ran beside other calls in
flight), and every kernel's stats over the roofline leg alone
(`roofline_leg_kernels`).

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
collected in separate passes, are in KiB, and on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read, so traffic = (2*FETCH_SIZE +
WRITE_SIZE) * 1024 per dispatch (the uncorrected value is reported too).
(The heavy stage's reads are per-lane gathers, not wide coalesced ones; its
block reports both.)

    python3 profiles/summarize_pmc.py <out_dir> [--last 30]
"""

import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict

DOMINANT = "compact_search"
GEOMETRY = "G32>"            # stage 0 (stage 0w is the G64 instance)
HEAVY = "memo_search"        # the heavy stage in lane mode


def rows(path_glob):
    out = []
    for p in sorted(glob.glob(path_glob, recursive=True)):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def is_dominant(name):
    return DOMINANT in name and GEOMETRY in name


def is_heavy(name):
    return HEAVY in name


def dispatch_key(r):
    d = r.get("Dispatch_Id") or r.get("Correlation_Id") or "0"
    return int(d)


def durations(out_dir, last, pick=is_dominant):
    """Durations (ns) of a kernel's dispatches, in dispatch order."""
    tr = [r for r in rows(os.path.join(out_dir, "trace", "**", "*kernel_trace.csv")) if pick(r["Kernel_Name"])]
    tr.sort(key=dispatch_key)
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
    return d, d[-last:] if last else d


def leg_kernels(out_dir, last):
    """Per-kernel stats over the roofline leg only: every dispatch from the
    first of the last `last` stage-0 dispatches on (synchronous calls, one
    at a time: each kernel's mean is its per-launch work time)."""
    tr = rows(os.path.join(out_dir, "trace", "**", "*kernel_trace.csv"))
    dom = sorted((r for r in tr if is_dominant(r["Kernel_Name"])), key=lambda r: int(r["Start_Timestamp"]))
    if not dom or not last:
        return {}
    t0 = int(dom[-last]["Start_Timestamp"])
    per = defaultdict(list)
    for r in tr:
        if int(r["Start_Timestamp"]) >= t0:
            per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: {"calls": len(v), "mean_ns": statistics.mean(v), "median_ns": statistics.median(v),
                "min_ns": min(v), "max_ns": max(v)} for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}


def counters(out_dir, name, last, pick=is_dominant):
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value
    for r in rows(os.path.join(out_dir, name, "**", "*counter_collection.csv")):
        if not pick(r.get("Kernel_Name", "")):
            continue
        per[dispatch_key(r)][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        return {}, 0
    keys = sorted(per)[-last:] if last else sorted(per)
    names = set(c for k in keys for c in per[k])
    return {c: sum(per[k].get(c, 0.0) for k in keys) / len(keys) for c in names}, len(keys)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir", nargs="?", default="gpurun_out/prof")
    ap.add_argument("--last", type=int, default=30, help="dispatches of the dominant kernel to summarise (0 = all)")
    args = ap.parse_args()
    out_dir = args.out_dir
    res = {"dominant_kernel": f"{DOMINANT}<..., {GEOMETRY[:-1]}> (stage 0)", "last_dispatches": args.last}
    stats = rows(os.path.join(out_dir, "trace", "**", "*kernel_stats.csv"))
    res["kernels"] = {r["Name"]: {"calls": int(r["Calls"]), "mean_ns": float(r["AverageNs"]),
                                  "pct": float(r["Percentage"])} for r in stats}
    res["roofline_leg_kernels"] = leg_kernels(out_dir, args.last)
    all_d, d = durations(out_dir, args.last)
    if d:
        res["dominant"] = {"dispatches": len(d), "mean_ns": statistics.mean(d), "median_ns": statistics.median(d),
                           "min_ns": min(d), "max_ns": max(d), "all_dispatches": len(all_d),
                           "all_mean_ns": statistics.mean(all_d)}
        res["dominant_mean_ns"] = statistics.mean(d)
    f, nf = counters(out_dir, "fetch", args.last)
    w, nw = counters(out_dir, "write", args.last)
    f, w = f.get("FETCH_SIZE"), w.get("WRITE_SIZE")
    res["FETCH_SIZE_kib"] = f
    res["WRITE_SIZE_kib"] = w
    res["pmc_dispatches"] = {"fetch": nf, "write": nw}
    if f is not None and w is not None:
        res["hbm_bytes_per_launch"] = (2.0 * f + w) * 1024.0
        res["hbm_bytes_per_launch_uncorrected"] = (f + w) * 1024.0
    sq, _ = counters(out_dir, "sq1", args.last)
    sq2, _ = counters(out_dir, "sq2", args.last)
    sq.update(sq2)
    res["sq"] = sq
    res["valu_insts_per_launch"] = sq.get("SQ_INSTS_VALU")
    res["lds_bank_conflict_cycles"] = sq.get("SQ_LDS_BANK_CONFLICT")
    res["lds_active_inst"] = sq.get("SQ_ACTIVE_INST_LDS")
    if sq.get("SQ_WAVE_CYCLES"):
        wc = sq["SQ_WAVE_CYCLES"]
        res["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0) / wc
        res["wait_inst_any_frac"] = sq.get("SQ_WAIT_INST_ANY", 0) / wc
        res["active_inst_frac"] = sq.get("SQ_ACTIVE_INST_ANY", 0) / wc
    # the heavy stage: the same per-dispatch figures for memo_search
    _, hd = durations(out_dir, args.last, is_heavy)
    hv = {}
    if hd:
        hv = {"kernel": "memo_search (heavy stage, lane mode)", "dispatches": len(hd),
              "mean_ns": statistics.mean(hd), "median_ns": statistics.median(hd), "min_ns": min(hd),
              "max_ns": max(hd)}
        hf, _ = counters(out_dir, "fetch", args.last, is_heavy)
        hw, _ = counters(out_dir, "write", args.last, is_heavy)
        hf, hw = hf.get("FETCH_SIZE"), hw.get("WRITE_SIZE")
        hv["FETCH_SIZE_kib"], hv["WRITE_SIZE_kib"] = hf, hw
        if hf is not None and hw is not None:
            hv["hbm_bytes_per_launch"] = (2.0 * hf + hw) * 1024.0
            hv["hbm_bytes_per_launch_uncorrected"] = (hf + hw) * 1024.0
        hsq, _ = counters(out_dir, "sq1", args.last, is_heavy)
        hsq2, _ = counters(out_dir, "sq2", args.last, is_heavy)
        hsq.update(hsq2)
        hv["sq"] = hsq
        hv["valu_insts_per_launch"] = hsq.get("SQ_INSTS_VALU")
    res["heavy"] = hv
    try:
        with open(os.path.join(out_dir, "trace.json")) as fjs:
            b = json.loads(fjs.read().strip().splitlines()[-1])
        res["config"] = b["config"]["workload"]
        res["n_hist"] = b["config"]["histories_per_gpu"]
        res["stage0_budget"] = b["roofline"].get("stage0_budget_used")
        res["fold"] = b["config"].get("fold")
        ks = b["roofline"]["kernels"]
        res["bench_kernels"] = ks
        if d:
            res["frac_from_profile"] = ks["stage0"]["alg_bytes_per_launch"] / (res["dominant_mean_ns"] * 1e-9) / 8e12
        if hd and ks.get("heavy"):
            hv["frac_from_profile"] = ks["heavy"]["alg_bytes_per_launch"] / (hv["mean_ns"] * 1e-9) / 8e12
    except Exception:
        pass
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
