#!/bin/bash
# Round 6: stage 0's grid, second pass -- the driver's command at the default
# (65536: one workgroup per group) / 12288 / 8192 / 6144, 5 rounds in
# rotation, then the 200-step default at 65536 / 8192, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_grid2
mkdir -p $O
for r in 1 2 3 4 5; do
  for g in 65536 12288 8192 6144; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param stage0_grid=$g > $O/g$g.$r.json 2> $O/g$g.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/g$g.$r.json'))
print('grid $g round $r', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
for r in 1 2; do
  for g in 65536 8192; do
    timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --param stage0_grid=$g > $O/d$g.$r.json 2> $O/d$g.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/d$g.$r.json'))
print('200 steps grid $g round $r', '%.3e' % d['value'])
"
  done
done
