#!/bin/bash
# The driver's 20-step command after 5 vs 40 warm-up steps (3 rounds each):
# does a short warm-up leave the timed region cold?
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/warm.log
: > $out
for r in 1 2 3; do
  for w in 5 40; do
    line=$(timeout -k 10 120 python -u bench.py --steps 20 --warmup $w --no-extra --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('warmup', sys.argv[2], round(d['value']/1e9,3), 'in_flight', d['device_ms']['in_flight'])" "$line" $w >> $out
  done
done
cat $out
