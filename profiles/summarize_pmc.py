"""Summarise a profiles/profile.sh run: per-kernel mean duration (kernel
trace) and per-dispatch PMC counters of the dominant search kernel.

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
collected in separate passes, are in KiB, and on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read, so traffic = (2*FETCH_SIZE +
WRITE_SIZE) * 1024 per dispatch (the uncorrected value is reported too).
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict

DOMINANT = "compact_search"
GEOMETRY = "G32>"            # stage 0 (stage 0w is the G64 instance)


def rows(path_glob):
    out = []
    for p in glob.glob(path_glob, recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def counters(out_dir, name):
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value
    kname = {}
    for r in rows(os.path.join(out_dir, name, "**", "*counter_collection.csv")):
        k = r.get("Kernel_Name", "")
        if DOMINANT not in k or GEOMETRY not in k:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        kname[d] = k
    if not per:
        return {}
    names = set(c for v in per.values() for c in v)
    return {c: sum(v.get(c, 0.0) for v in per.values()) / len(per) for c in names}


def main(out_dir):
    res = {"dominant_kernel": DOMINANT}
    stats = rows(os.path.join(out_dir, "trace", "**", "*kernel_stats.csv"))
    res["kernels"] = {r["Name"]: {"calls": int(r["Calls"]), "mean_ns": float(r["AverageNs"]),
                                  "pct": float(r["Percentage"])} for r in stats}
    dur = [v["mean_ns"] for k, v in res["kernels"].items() if DOMINANT in k and GEOMETRY in k]
    res["dominant_mean_ns"] = dur[0] if dur else None
    f = counters(out_dir, "fetch").get("FETCH_SIZE")
    w = counters(out_dir, "write").get("WRITE_SIZE")
    res["FETCH_SIZE_kib"] = f
    res["WRITE_SIZE_kib"] = w
    if f is not None and w is not None:
        res["hbm_bytes_per_launch"] = (2.0 * f + w) * 1024.0
        res["hbm_bytes_per_launch_uncorrected"] = (f + w) * 1024.0
    sq = counters(out_dir, "sq1")
    sq.update(counters(out_dir, "sq2"))
    res["sq"] = sq
    res["valu_insts_per_launch"] = sq.get("SQ_INSTS_VALU")
    res["lds_bank_conflict_cycles"] = sq.get("SQ_LDS_BANK_CONFLICT")
    res["lds_active_inst"] = sq.get("SQ_ACTIVE_INST_LDS")
    if sq.get("SQ_WAVE_CYCLES"):
        wc = sq["SQ_WAVE_CYCLES"]
        res["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0) / wc
        res["wait_inst_any_frac"] = sq.get("SQ_WAIT_INST_ANY", 0) / wc
        res["active_inst_frac"] = sq.get("SQ_ACTIVE_INST_ANY", 0) / wc
    try:
        with open(os.path.join(out_dir, "trace.json")) as fjs:
            b = json.loads(fjs.read().strip().splitlines()[-1])
        res["config"] = b["config"]["workload"]
        res["n_hist"] = b["config"]["histories_per_gpu"]
    except Exception:
        pass
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
