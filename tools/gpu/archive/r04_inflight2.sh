#!/bin/bash
# Round 4, final build (no timing events in the window): calls in flight x
# hardware queues, the driver's command and 200 steps
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/inflight2; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
  for cfg in "3 4" "4 8" "3 8"; do
    set -- $cfg
    n=drv_i$1_q$2_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --inflight $1 --hw-queues $2
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
for cfg in "3 4" "4 8"; do
  set -- $cfg
  n=d200_i$1_q$2
  step $n python bench.py --no-cpu-baseline --no-extra --inflight $1 --hw-queues $2
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
done
