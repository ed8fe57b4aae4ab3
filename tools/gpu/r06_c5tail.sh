#!/bin/bash
# Round 6: config 5 (100k 6x24, 3 calls in flight, lane mode) with its long
# lane searches handed to the wave-mode tail launch (tail_min 0) after
# tail_cap 32 / 64 / 96 iterations, against no tail (the default: the list
# is under tail_min), 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c5tail
mkdir -p $O
for r in 1 2; do
  for c in 0 32 64 96; do
    P="--param tail_min=0 --param tail_cap=$c"; [ $c = 0 ] && P=""
    timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget -1 $P > $O/t$c.$r.json 2> $O/t$c.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/t$c.$r.json'))
print('tail_cap $c round $r', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
