#!/bin/bash
# Round 6: config 3 (1M bug-laden, 3 calls in flight, the automatic stage-0
# budget) at lane mode's memo_after 4 / 16 / 32 (the default) / 64, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c3after
mkdir -p $O
for r in 1 2; do
  for m in 4 16 32 64; do
    timeout -k 10 200 python bench.py --config bank_4x16_bugs --steps 10 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget -1 --param memo_after=$m > $O/a$m.$r.json 2> $O/a$m.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/a$m.$r.json'))
print('memo_after $m round $r', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
