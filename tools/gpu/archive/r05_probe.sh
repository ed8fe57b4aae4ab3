#!/bin/bash
# Round 5: the heavy stage's memo probe in one round trip (both 16-B loads
# before any compare) -- its per-group anatomy (tools/memo_stats.py) at the
# bench's knobs, memo after 32 and 18 nodes, and the driver's command.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_probe
mkdir -p $O
K="stage0_budget=18 heavy_mode=1 memo_lds=0"
for v in "memo_after=32" "memo_after=18" "memo_after=0"; do
  timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K $v > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  echo "$v: $(cat $O/ms.json)"
done
for r in 1 2 3; do
  for a in 32 18; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param memo_after=$a > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('memo_after $a round $r %.3e' % d['value'], d['device_ms']['alone'])"
  done
done
