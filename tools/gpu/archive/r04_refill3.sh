#!/bin/bash
# Round 4: lane refill on the other configurations (config 3: injected bugs; 1; 5)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/rf3; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for c in bank_4x16_bugs ticket_2x10 bank_6x24; do
  for rf in 0 1; do
    for hm in 1 2; do
      n=${c}_${rf}_${hm}_$r
      nh=1000000; [ $c = bank_6x24 ] && nh=100000
      step $n python bench.py --config $c --n-hist $nh --steps 10 --warmup 3 --no-cpu-baseline --no-extra --param memo_refill=$rf --param heavy_mode=$hm
      python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', '%.3e' % d['value'], 'call', round(d['device_ms']['alone']['call_mean'],4), d['config'].get('heavy_stage'))"
    done
  done
done
done
