#!/bin/bash
# Round 6: config 5 (Bank 6x24, 100k, 3 calls in flight) against the heavy
# stage's mode and the stage-0w budget: lane mode (the bench's) at
# stage0w_budget 32 / 64 / 128 / 256 and memo_after 16, wave mode at 32 / 64.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c5sweep
mkdir -p $O
run() {  # tag, bench args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -3 $O/$t.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/$t.json'))
print('$t', '%.3e' % d['value'], 'mism', d.get('mismatches_vs_oracle'), {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
}
for r in 1 2; do
  run lane_w32.$r --param stage0w_budget=32
  run lane_w64.$r --param stage0w_budget=64
  run lane_w128.$r --param stage0w_budget=128
  run lane_w256.$r --param stage0w_budget=256
  run lane_w32_after16.$r --param stage0w_budget=32 --param memo_after=16
  run wave_w32.$r --param stage0w_budget=32 --param heavy_mode=0 --param memo_lds=1
  run wave_w64.$r --param stage0w_budget=64 --param heavy_mode=0 --param memo_lds=1
done
