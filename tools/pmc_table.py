"""Per-kernel mean of every PMC counter over the dispatches of rocprofv3
--pmc runs (one or more output directories).

    python tools/pmc_table.py gpurun_out/pmc1 gpurun_out/pmc2 [--json out.json]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?(?:qsmd::)?([A-Za-z_0-9]+)", name)
    base = m.group(1) if m else name[:40]
    t = re.search(r"<([^>]*)>", name)
    return base + (f"<{t.group(1)[:40]}>" if t else "")


def main(argv):
    out_json = None
    if "--json" in argv:
        i = argv.index("--json")
        out_json = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    per = defaultdict(lambda: defaultdict(list))      # kernel -> counter -> [per-dispatch totals]
    for d in argv:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            acc = defaultdict(float)
            names = {}
            with open(p) as f:
                for r in csv.DictReader(f):
                    key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                    acc[key] += float(r["Counter_Value"])
                    names[key[0]] = short(r.get("Kernel_Name", "?"))
            for (disp, c), v in acc.items():
                per[names[disp]][c].append(v)
    table = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    for k, cs in sorted(table.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {v:16.1f}")
    if out_json:
        with open(out_json, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
