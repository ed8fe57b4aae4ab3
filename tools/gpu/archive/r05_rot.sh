#!/bin/bash
# Round 5: distinct resident batches (--rotate K) against one batch, and
# copies of one batch (the same hints, no reuse of the batch through the
# caches) -- 3 rounds each at the driver's 20 steps and at 100.  Then the
# early-exit leg and the heavy stage's cycles per iteration (memo_stats).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_rot
mkdir -p $O
B="--warmup 5 --no-extra --no-cpu-baseline"
for steps in 20 100; do
for r in 1 2 3; do
  for v in "1" "4" "2c" "4c"; do
    case $v in
      1) A="";; 4) A="--rotate 4";; 2c) A="--rotate 2 --rotate-copies";; 4c) A="--rotate 4 --rotate-copies";;
    esac
    timeout -k 10 150 python bench.py --steps $steps $B $A > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('steps $steps rotate $v round $r %.3e' % d['value'])"
  done
done
done
timeout -k 10 200 python bench.py --early-exit --steps 5 --warmup 2 > $O/ee.json 2> $O/ee.err || { tail -20 $O/ee.err; exit 1; }
cat $O/ee.json
K="stage0_budget=18 heavy_mode=1"
for v in "memo_lds=0" "memo_lds=0 memo_after=1000000000" "memo_lds=2" "memo_lds=2 memo_lds_entries=16" "memo_lds=0 memo_after=18"; do
  timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K $v > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  echo "$v: $(cat $O/ms.json)"
done
