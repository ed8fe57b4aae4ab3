#!/bin/bash
# Round 4, final build: one call at a time (automatic budget, 16 on config 2)
# against lane mode's memo_after and its HBM table entries
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/i1after; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
  for kv in "memo_after=32" "memo_after=20" "memo_after=48" "memo_lane_entries=256" "memo_lane_entries=64"; do
    n=i1_${kv/=/_}_$r
    step $n python bench.py --inflight 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extra --param $kv
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
done
