#!/bin/bash
# Lane mode's tail: its counters and per-kernel durations at a few caps.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/tail2
mkdir -p $O
for cap in 0 24 48; do
  timeout -k 10 120 python tools/tail_stats.py bank_4x16 1000000 tail_cap=$cap > $O/ts_$cap.txt 2>&1 || { tail $O/ts_$cap.txt; exit 1; }
  echo "cap $cap"; tail -2 $O/ts_$cap.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cap in 0 24; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$cap -o run -- python bench.py --inflight 1 --steps 50 --warmup 5 --no-extra --no-cpu-baseline --param tail_cap=$cap > $O/prof_$cap.log 2>&1 || { tail $O/prof_$cap.log; exit 1; }
  f=$(ls $O/prof_$cap/*/run_kernel_stats.csv | head -1); echo "cap $cap"; cut -d, -f1-6 "$f" | head -8
done
