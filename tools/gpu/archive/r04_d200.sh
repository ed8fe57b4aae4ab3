#!/bin/bash
# Round 4, final: 200-step runs (no CPU baseline, no extra configs) with 4
# and 3 calls in flight, alternating, 8 hardware queues
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/d200; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
  for i in 4 3; do
    n=d200_i${i}_$r
    step $n python bench.py --no-cpu-baseline --no-extra --inflight $i
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
    n=d20_i${i}_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --inflight $i
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
