#!/bin/bash
# Round 4: the library's default stage-0 budget (32) against 16 / 20 on the other configurations (calls in flight)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/lb; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for c in bank_4x16_bugs ticket_2x10 bank_6x24; do
  for b in 16 20 32; do
    n=${c}_${b}_$r
    nh=1000000; [ $c = bank_6x24 ] && nh=100000
    step $n python bench.py --config $c --n-hist $nh --steps 10 --warmup 3 --no-cpu-baseline --no-extra --stage0-budget $b
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', '%.3e' % d['value'], 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
done
