#!/bin/bash
# Round 6: the extra configs 1 / 3 / 5 (bench.py's extra-config shape, 3 calls
# in flight) at stage-0 budgets 16 / 20 / 24 / 32 and the library's automatic
# budget (-1), to set the automatic budget for bug-laden batches.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_xbudget}
mkdir -p $O
for cfg in ticket_2x10:1000000 bank_4x16_bugs:1000000 bank_6x24:100000; do
  name=${cfg%%:*}; n=${cfg##*:}
  for b in -1 16 20 24 32; do
    timeout -k 10 200 python bench.py --config $name --n-hist $n --steps 10 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget $b > $O/$name.b$b.json 2> $O/$name.b$b.err || { tail $O/$name.b$b.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/$name.b$b.json'))
print('$name budget $b', '%.3e' % d['value'], 'used', d['roofline'].get('stage0_budget_used'), 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
