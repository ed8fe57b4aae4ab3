#!/bin/bash
# Round 6: A/B of two builds (tools/ab.py) at the driver's command (4 calls
# in flight, 20 steps) and one call at a time, after the heavy stage's
# per-group anatomy of build B (tools/memo_stats.py at the bench's knobs).
#   bash tools/gpu/r06_ab.sh ablib/A.so ablib/B.so [rounds] [memo_stats knobs...]
set -o pipefail
export PYTHONUNBUFFERED=1
A=$1; B=$2; R=${3:-3}; shift 3
O=gpurun_out/r06_ab
mkdir -p $O
K="stage0_budget=20 heavy_mode=1 memo_lds=0 $*"
QSMD_LIB_PATH=$PWD/$B timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/memo_stats.json 2> $O/memo_stats.err &&
cat $O/memo_stats.json &&
timeout -k 10 400 python tools/ab.py $A $B $R --steps 20 --warmup 5 --inflight 4 &&
timeout -k 10 300 python tools/ab.py $A $B $R --steps 50 --warmup 5 --inflight 1
