"""Summarise a tools/gpu/profile_round.sh run: per-kernel stats, per-launch
PMC counters of the stage-0 kernel (compact_search<Bank, G32>), HBM traffic
per launch with the gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md, HBM).
    python tools/profile_summary.py <gpurun_out dir> <profiles/tag>"""

import collections
import csv
import glob
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
KEY = "compact_search<2u, false, qsmd::(anonymous namespace)::G32>"

stats = {}
for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
    shutil.copy(f, os.path.join(dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(f)):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "mean_ns": float(r["AverageNs"]),
                            "pct": float(r["Percentage"])}
counters = collections.defaultdict(list)
for d in ("fetch", "write", "sq", "lds"):
    for f in glob.glob(os.path.join(src, d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if KEY in r.get("Kernel_Name", ""):
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for disp in per.values():
            for k, v in disp.items():
                counters[k].append(v)
mean = {k: sum(v) / len(v) for k, v in counters.items() if v}
out = {"dominant_kernel": KEY, "kernels": stats, "stage0_pmc_mean_per_launch": mean,
       "launches": {k: len(v) for k, v in counters.items()}}
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    out["hbm_bytes_per_launch"] = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
if "SQ_INSTS_VALU" in mean and "SQ_WAVES" in mean:
    out["valu_per_wave"] = mean["SQ_INSTS_VALU"] / mean["SQ_WAVES"]
json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
bench = os.path.join(src, "bench_under_rocprof.json")
if os.path.exists(bench):
    shutil.copy(bench, os.path.join(dst, "bench_under_rocprof.json"))
if "hbm_bytes_per_launch" in out:
    json.dump({"source": f"{dst}/summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
               "config": "bank_4x16", "n_hist": 1000000, "kernel": KEY,
               "hbm_bytes_per_launch": out["hbm_bytes_per_launch"],
               "FETCH_SIZE_kib": mean["FETCH_SIZE"], "WRITE_SIZE_kib": mean["WRITE_SIZE"],
               "correction": "traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE reports half of "
                             "a wide coalesced read)"},
              open("profiles/pmc_traffic.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in out if k != "kernels"}, indent=1))
for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["pct"])[:8]:
    print(f"{v['pct']:6.2f}% {v['mean_ns'] / 1e3:9.2f} us x{v['calls']:3d}  {k[:90]}")
