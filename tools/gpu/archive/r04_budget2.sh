#!/bin/bash
# Round 4 (sharded heavy list): the driver's command and one call at a time against the stage-0 budget
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/b2; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for b in ${DBUDGETS:-14 16 17 18 19 20}; do
  step drv_${b}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b
  python3 -c "import json; d=json.load(open('$O/drv_${b}_$r.out')); print('drv budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
for b in ${IBUDGETS:-16 18 20 24 32}; do
  step i1_${b}_$r python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget $b
  python3 -c "import json; d=json.load(open('$O/i1_${b}_$r.out')); print('i1 budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4), d['config'].get('heavy_stage'))"
done
done
