#!/bin/bash
# The bench's stage-0 budget at 4 calls in flight after the heavy stage got
# faster (written-slot map): 17 / 18 / 20 / 22, the driver's 20 steps, 3 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_budget2
mkdir -p $O
for r in 1 2 3; do
  for b in 17 18 20 22; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --stage0-budget $b > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('budget $b round $r %.3e' % d['value'], 'alone', {k: round(v*1e3,1) for k, v in d['device_ms']['alone'].items()})"
  done
done
