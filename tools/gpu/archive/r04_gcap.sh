#!/bin/bash
# Round 4, final build: lane mode's hand-off to the giant stage (after 64 x
# split_budget iterations) as a straggler cut -- split_budget 1 / 2 / 4 vs
# the default 1024, the driver's command and one call at a time
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/gcap; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
  for sb in 1024 1 2 4; do
    n=drv_sb${sb}_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param split_budget=$sb
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'alone', round(d['device_ms']['alone']['call_mean'],4))"
    n=i1_sb${sb}_$r
    step $n python bench.py --inflight 1 --steps 100 --warmup 20 --no-cpu-baseline --no-extra --param split_budget=$sb
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
