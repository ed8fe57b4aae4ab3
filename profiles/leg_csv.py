"""profiles/<round>/kernel_stats.csv from a profile summary (profiles/profile.sh
-> summarize_pmc.py): every kernel over the bench's roofline leg only (the
last N synchronous calls), one row per kernel.
    python profiles/leg_csv.py gpurun_out/measure/prof/summary.json profiles/r03/kernel_stats.csv"""
import csv
import json
import sys


def main(src, dst, window="roofline leg: the last 30 synchronous calls of bench.py --steps 20 --warmup 5 "
                          "under rocprofv3 --kernel-trace"):
    with open(src) as f:
        leg = json.load(f)["roofline_leg_kernels"]
    with open(dst, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "MeanNs", "MedianNs", "MinNs", "MaxNs", "Window"])
        for name, k in sorted(leg.items(), key=lambda kv: -kv[1]["mean_ns"]):
            w.writerow([name, k["calls"], round(k["mean_ns"], 1), k["median_ns"], k["min_ns"], k["max_ns"], window])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
