#!/bin/bash
# Round 6: config 3 (bench.py's extra-config shape, the tail and the ordered
# groups on) at stage-0 budgets 24 / 32 (the library's automatic) / 40 / 48.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_c3budget}
mkdir -p $O
for r in 1 2; do
  for b in 24 32 40 48; do
    timeout -k 10 200 python bench.py --config bank_4x16_bugs --steps 10 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget $b > $O/b$b.$r.json 2> $O/b$b.$r.err || { tail $O/b$b.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/b$b.$r.json'))
print('config3 budget $b round $r', '%.3e' % d['value'], 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
