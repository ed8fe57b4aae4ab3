#!/bin/bash
# Round 6: the driver's command at stage-0 budgets 17 / 18 / 20 / 22 / 24
# (the bench's 20 was chosen in round 5; the heavy stage is ~10 % shorter
# now), 3 interleaved rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_budget}
mkdir -p $O
for r in 1 2 3; do
  for b in 17 18 20 22 24; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --stage0-budget $b > $O/b$b.$r.json 2> $O/b$b.$r.err || { tail $O/b$b.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/b$b.$r.json'))
print('budget $b round $r', '%.3e' % d['value'], 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
