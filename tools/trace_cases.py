"""Per-case median kernel durations from a rocprofv3 kernel trace of
tools/stage0_cases.py (diagnostic): the trace is cut into consecutive
blocks of `reps` calls per case (one call = the launches between two
giant_search launches).

    python tools/trace_cases.py TRACE_DIR REPS CASE...
"""
import collections
import csv
import glob
import statistics
import sys


def short(name):
    name = name.replace("qsmd::", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0][:48]


def main():
    d, reps, cases = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "qsmd::" in r["Kernel_Name"]]
    calls, cur = [], []
    for r in rows:
        if r["Kernel_Name"].startswith("void qsmd::gen_") or "generate" in r["Kernel_Name"]:
            continue
        cur.append(r)
        if "giant_search" in r["Kernel_Name"]:
            calls.append(cur)
            cur = []
    for i, case in enumerate(cases):
        blk = calls[i * reps:(i + 1) * reps]
        per = collections.defaultdict(list)
        span = []
        for c in blk:
            seen = collections.Counter()
            for r in c:
                k = short(r["Kernel_Name"])
                seen[k] += 1
                per[f"{k}#{seen[k]}"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            span.append((int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3)
        print(f"== {case}: call span {statistics.median(span):.1f} us")
        for k, v in per.items():
            print(f"   {k:52s} {statistics.median(v):9.1f} us")


if __name__ == "__main__":
    main()
