#!/bin/bash
# Lane mode's knobs after the written-slot map: memo table entries per lane
# (64 / 128 / 256) and the memo's join point (memo_after 16 / 32 / 48), the
# driver's command and one call at a time, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_knobs
mkdir -p $O
for r in 1 2; do
  for v in "memo_lane_entries=128" "memo_lane_entries=64" "memo_lane_entries=256" "memo_after=16" "memo_after=48"; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param $v > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    timeout -k 10 120 python bench.py --inflight 1 --no-extra --no-cpu-baseline --param $v > $O/i.json 2> $O/i.err || { tail $O/i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/r.json')); i=json.load(open('$O/i.json'))
print('$v $r %.3e' % d['value'], 'i1 %.3e' % i['value'], 'heavy alone', round(d['device_ms']['alone']['heavy_mean']*1e3,1), round(i['device_ms']['alone']['heavy_mean']*1e3,1))"
  done
done
