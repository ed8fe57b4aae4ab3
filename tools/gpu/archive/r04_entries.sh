#!/bin/bash
# Round 4: lane mode's HBM memo table size per lane (memo_lane_entries): the driver's command and one call at a time
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/me; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for e in ${ES:-8 16 32 128}; do
  n=drv_${e}_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param memo_lane_entries=$e
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  n=i1_${e}_$r
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget 16 --param memo_lane_entries=$e --param heavy_mode=1
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
