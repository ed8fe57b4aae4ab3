#!/bin/bash
# After the table-headroom fix: K = 1 against K = 5 distinct batches and
# K = 5 copies of batch 0 (the same histories at other addresses: the same
# cross-call hints, no reuse of a batch through the caches), 3 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/rot3
mkdir -p $O
for r in 1 2 3; do
  for v in 1 5 5c; do
    case $v in 1) A="--rotate 1";; 5) A="--rotate 5";; 5c) A="--rotate 5 --rotate-copies";; esac
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline $A > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.3e' % d['value'], 'alone', round(d['device_ms']['alone']['stage0_mean'], 4))"
  done
done
