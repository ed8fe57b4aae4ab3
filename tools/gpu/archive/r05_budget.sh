#!/bin/bash
# Round 5: the stage-0 budget at 4 calls in flight over 5 distinct batches
# (the bench's defaults now), the driver's 20 steps, 3 alternating rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_budget
mkdir -p $O
for r in 1 2 3; do
  for b in 16 17 18 20 22; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --stage0-budget $b > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('budget $b round $r %.3e' % d['value'], 'alone', d['device_ms']['alone'])"
  done
done
