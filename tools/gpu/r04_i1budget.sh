#!/bin/bash
# Round 4: one call at a time (--inflight 1) against the stage-0 budget and heavy mode
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/i1b; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for b in ${BUDGETS:-16 20 24 28 32 40}; do
  for hm in ${HMODES:-0 1}; do
    step i1_${b}_${hm}_$r python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget $b --param heavy_mode=$hm
    python3 -c "import json; d=json.load(open('$O/i1_${b}_${hm}_$r.out')); print('i1 budget $b heavy_mode $hm', round(d['value']/1e9,3), round(d['ms_per_step'],4), 's0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
done
