#!/bin/bash
# Round 6: stage 0's grid (knob stage0_grid: workgroups at most, grid-stride
# beyond) at 4096 / 8192 against the default (one workgroup per group of 64,
# 15625 for 1M) -- the driver's command, 3 rounds in rotation.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_grid
mkdir -p $O
for r in 1 2 3; do
  for g in 65536 8192 4096; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param stage0_grid=$g > $O/g$g.$r.json 2> $O/g$g.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/g$g.$r.json'))
print('grid $g round $r', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
