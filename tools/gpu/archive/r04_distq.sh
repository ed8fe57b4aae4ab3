#!/bin/bash
# Round 4, final build: one rank over the RCCL path, 3 calls in flight,
# against the hardware queue count (the environment's 4, 8, 12), alternating
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/distq; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
  for q in 4 8 12; do
    n=dist_q${q}_$r
    step $n env QSMD_BENCH_DIST=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --hw-queues $q
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
  n=none_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
done
