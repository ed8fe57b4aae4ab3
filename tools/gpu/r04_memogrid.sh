#!/bin/bash
# Round 4: the driver's command against lane mode's workgroup cap (memo_grid) and the stage-0 budget
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/mg; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for g in ${GRIDS:-0 32 64 128 256}; do
  for b in ${DBUDGETS:-18 20}; do
    step drv_${g}_${b}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b --param memo_grid=$g
    python3 -c "import json; d=json.load(open('$O/drv_${g}_${b}_$r.out')); print('drv memo_grid $g budget $b', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
done
