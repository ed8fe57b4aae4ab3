#!/bin/bash
# The early-exit step's pieces (tools/micro/early_split.py) and its kernel trace.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/early2
mkdir -p $O
timeout -k 10 200 python tools/micro/early_split.py > $O/split.txt 2>&1 || { tail $O/split.txt; exit 1; }
cat $O/split.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --early-exit --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cut -d, -f1-5 "$f" | head -20 || true
