#!/bin/bash
# Round 6: one call at a time (config 2, the library's other defaults) at
# explicit stage-0 budgets 12 / 14 / 16 (the automatic one) / 18 / 20 / 24, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_one
mkdir -p $O
for r in 1 2; do
  for b in 12 14 16 18 20 24; do
    timeout -k 10 200 python bench.py --inflight 1 --steps 50 --warmup 5 --no-extra --no-cpu-baseline --stage0-budget $b > $O/b$b.$r.json 2> $O/b$b.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/b$b.$r.json'))
print('budget $b round $r', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
