#!/bin/bash
# Round 4, final build: 3 calls in flight on 4 hardware queues (the default)
# against 4 and 5 on 8, alternating, the driver's command; one rank over
# the RCCL path for 3 / 4 in flight
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/inflight3; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3 4; do
  for cfg in "3 4" "4 8" "5 8"; do
    set -- $cfg
    n=drv_i$1_q$2_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --inflight $1 --hw-queues $2
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
for i in 3 4; do
  n=dist_i$i
  step $n env QSMD_BENCH_DIST=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --inflight $i
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
done
