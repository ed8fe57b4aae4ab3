#!/bin/bash
# Round 5: one call at a time (the library's defaults: automatic stage-0
# budget, heavy mode by the last call) over one batch and over five.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_i1
mkdir -p $O
for k in 1 5; do
  for r in 1 2; do
    timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline --rotate $k --timing-events 1 > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('rotate $k %.3e' % d['value'], d['device_ms'], d['roofline']['stage0_budget_used'])"
  done
done
