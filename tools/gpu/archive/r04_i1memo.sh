#!/bin/bash
# Round 4: one call at a time in lane mode against the stage-0 budget, the
# memo's start (memo_after) and the LDS tables (memo_lds 1 = when the heavy
# groups fit the CUs)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/i1memo; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for b in ${BUDGETS:-18 24 28}; do
  for ma in ${AFTERS:-0 16 32}; do
    for ml in ${LDS:-0 1}; do
      n=i1_${b}_${ma}_${ml}
      step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget $b \
           --param heavy_mode=1 --param memo_after=$ma --param memo_lds=$ml
      python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
    done
  done
done
