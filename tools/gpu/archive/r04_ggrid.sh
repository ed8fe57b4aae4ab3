#!/bin/bash
# Round 4: one call at a time (automatic budget) against the giant stage's
# grid when no call has had a giant (its short path: totals, probe, restore)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/ggrid; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
  for g in 1 8 64; do
    n=i1_g${g}_$r
    step $n python bench.py --inflight 1 --steps 200 --warmup 10 --no-cpu-baseline --no-extra --param giant_grid=$g
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
done
