#!/bin/bash
# Round 6: config 5 after the sharded deferred list -- lane mode at
# stage0w_budget 16 / 24 / 32 / 48, wave mode at 32 / 48 / 64 / 96 (3 calls in
# flight, 2 rounds).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c5sweep2
mkdir -p $O
run() {  # tag, bench args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -3 $O/$t.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/$t.json'))
print('$t', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
}
for r in 1 2; do
  for b in 16 24 32 48; do run lane_w$b.$r --param stage0w_budget=$b; done
  for b in 32 48 64 96; do run wave_w$b.$r --param stage0w_budget=$b --param heavy_mode=0; done
done
