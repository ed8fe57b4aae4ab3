#!/bin/bash
# The early-exit leg's first chunk (histories per rank in round 1): 64 /
# 256 / 1024 / 4096, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/fc
mkdir -p $O
for r in 1 2; do
  for fc in 64 256 1024 4096; do
    timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 --no-cpu-baseline --first-chunk $fc > $O/e_${fc}_$r.json 2> $O/e_${fc}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/e_${fc}_$r.json')); e=d['early_exit']; print($fc, $r, '%.3e' % d['value'], 'ms %.4f' % d['ms_per_step'], e['searched'], e['rounds'])"
  done
done
