"""Per-call anatomy of BASELINE config 4's host-entry calls from a rocprofv3
kernel + HIP API trace (CSV) of tools/config4.py (tools/gpu/r06_config4.sh):
the last N qsmd_check_batch calls, each delimited by its closing
hipStreamSynchronize; for each, the host time before the first launch, the
launch calls, each kernel, the gaps between them, and the wait from the last
kernel's end to hipStreamSynchronize's return.  Medians in microseconds.

    python tools/trace_c4.py <rocprofv3 output dir> [N]
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def main(d, last=100):
    ker = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(d, "**", "*hip_api_trace.csv"))
    kby = {r["Correlation_Id"]: r for r in ker}
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the thread that issued the config-4 launches (wave_search over 128-bit masks)
    c4 = [r for r in ker if "wave_search" in r["Kernel_Name"]]
    if not c4:
        raise SystemExit("no wave_search kernel in the trace")
    launch_ids = {r["Correlation_Id"] for r in c4}
    tid = next(r["Thread_Id"] for r in api if r["Correlation_Id"] in launch_ids)
    mine = [r for r in api if r["Thread_Id"] == tid]
    # calls: the API records between two closing hipStreamSynchronize on that thread,
    # keeping those that launched a config-4 kernel
    calls, cur = [], []
    for r in mine:
        cur.append(r)
        if r["Function"] == "hipStreamSynchronize":
            if any(x["Correlation_Id"] in launch_ids for x in cur):
                calls.append(cur)
            cur = []
    calls = calls[-last:]
    per = defaultdict(list)
    fn_time = defaultdict(list)
    kernel_names = set()
    for c in calls:
        c = [r for r in c if r["Function"] != "hipStreamSynchronize" or r is c[-1]]
        first = int(c[0]["Start_Timestamp"])
        sync = c[-1]
        launches = [r for r in c if r["Correlation_Id"] in kby]
        ks = sorted((kby[r["Correlation_Id"]] for r in launches), key=lambda k: int(k["Start_Timestamp"]))
        if not ks:
            continue
        per["host_before_first_launch_us"].append((int(launches[0]["Start_Timestamp"]) - first) / 1e3)
        per["first_launch_call_to_kernel_start_us"].append(
            (int(ks[0]["Start_Timestamp"]) - int(launches[0]["Start_Timestamp"])) / 1e3)
        for i, k in enumerate(ks):
            name = k["Kernel_Name"].split("(")[0][:60]
            kernel_names.add(name)
            per[f"kernel{i}_us ({name})"].append((int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3)
            if i:
                per[f"gap_kernel{i - 1}_end_to_kernel{i}_start_us"].append(
                    (int(k["Start_Timestamp"]) - int(ks[i - 1]["End_Timestamp"])) / 1e3)
        per["last_kernel_end_to_sync_return_us"].append((int(sync["End_Timestamp"]) - int(ks[-1]["End_Timestamp"])) / 1e3)
        per["call_first_api_to_sync_return_us"].append((int(sync["End_Timestamp"]) - first) / 1e3)
        for r in c:
            fn_time[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"config-4 host-entry calls analysed: {len(calls)} (thread {tid})")
    for k, v in per.items():
        print(f"  {k:70s} median {statistics.median(v):8.2f}  min {min(v):8.2f}  max {max(v):8.2f}")
    print("  HIP API calls per call (median duration us, count per call):")
    for k, v in sorted(fn_time.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"    {k:40s} {statistics.median(v):8.2f}  x{len(v) / max(len(calls), 1):.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100)
