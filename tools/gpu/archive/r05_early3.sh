#!/bin/bash
# The early-exit step's kernels (rocprofv3 kernel trace of tools/micro/early_split.py).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/early3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/micro/early_split.py > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
tail -8 $O/prof.log
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); echo "$f"; [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
t=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python3 - "$t" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 40 dispatches: name, duration, gap to the previous end (us)
prev = None
for r in rows[-40:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{r["Kernel_Name"][:60]:60s} {(e - s) / 1e3:8.1f} us  gap {((s - prev) / 1e3 if prev else 0):8.1f}')
    prev = e
PY
