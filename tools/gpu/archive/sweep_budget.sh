#!/bin/bash
# Stage-0 node budget sweep (config 2) with the heavy stage in wave mode:
# calls in flight (bench default) and one call at a time.
#   tools/gpu/archive/sweep_budget.sh "16 20 26" [steps]
set -o pipefail
mkdir -p gpurun_out/sweep
B=${1:-"16 18 20 22 24 26 32"}
STEPS=${2:-200}
for b in $B; do
  for inf in 3 1; do
    timeout -k 10 120 python bench.py --steps $STEPS --warmup 10 --no-cpu-baseline --no-extra --roof-calls 5 \
        --stage0-budget $b --inflight $inf > gpurun_out/sweep/b${b}_i${inf}.json 2> gpurun_out/sweep/b${b}_i${inf}.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "budget $b inflight $inf rc=$rc"; tail -5 gpurun_out/sweep/b${b}_i${inf}.err; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep/b${b}_i${inf}.json')); print('budget', $b, 'inflight', $inf, '%.3e' % d['value'], 'alone stage0 %.3f call %.3f' % (d['device_ms']['alone']['stage0_mean'], d['device_ms']['alone']['call_mean']))"
  done
done
