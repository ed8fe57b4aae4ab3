#!/bin/bash
# The bench's stage-0 budget 19 against 20 (4 calls in flight), after the
# heavy-stage and staging changes, 4 rounds of the driver's command.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_b19
mkdir -p $O
for r in 1 2 3 4; do
  for b in 19 20; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --stage0-budget $b > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('budget $b round $r %.3e' % d['value'])"
  done
done
