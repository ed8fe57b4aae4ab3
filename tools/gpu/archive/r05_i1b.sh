#!/bin/bash
# Round 5: one call at a time with and without the per-call timing events.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_i1
mkdir -p $O
for r in 1 2; do
  for t in 0 1; do
    timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline --rotate 1 --timing-events $t > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('timing $t %.3e' % d['value'], d['device_ms']['alone'])"
  done
done
