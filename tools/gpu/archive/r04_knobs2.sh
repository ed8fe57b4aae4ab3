#!/bin/bash
# Round 4: the bench's in-flight knobs on the final build (no timing events
# in the window): stage-0 budget x lane-mode memo table entries
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/knobs2; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
for b in 17 18 20; do
for e in 128 256; do
  n=drv_${b}_${e}_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b --param memo_lane_entries=$e
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
done
done
done
for e in 128 256; do
  n=d200_$e
  step $n python bench.py --no-cpu-baseline --no-extra --param memo_lane_entries=$e
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  n=c3_$e
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --config bank_4x16_bugs --stage0-budget 32 --param memo_lane_entries=$e
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
done
