#!/bin/bash
# Round 4: the driver's command against calls in flight and hardware queues
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/if; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for cfg in "3 0" "4 0" "4 8" "5 8" "6 8" "3 8"; do
  set -- $cfg
  hq=""; [ "$2" != 0 ] && hq="--hw-queues $2"
  n=drv_$1_$2_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --inflight $1 $hq --param memo_refill=0
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms/step', round(d['ms_per_step'],4))"
done
done
