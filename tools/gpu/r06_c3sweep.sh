#!/bin/bash
# Round 6: config 3 (1.25M bank_4x16_bugs per GPU, 3 calls in flight) against
# the stage-0 budget (-1: the library's automatic one) and the lane-mode
# heavy stage's grid (memo_grid 0: at most 12 workgroups per CU, grid-stride;
# 8192: one workgroup per group of 64 heavy histories).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c3sweep
mkdir -p $O
for cfg in ${CFGS:-"-1:0" "-1:8192" "64:0" "64:8192" "128:8192" "48:8192"}; do
  B=${cfg%%:*}; G=${cfg##*:}
  timeout -k 10 200 python bench.py --config bank_4x16_bugs --n-hist 1250000 --steps 10 --warmup 3 --inflight 3 --stage0-budget $B --rotate 1 --no-extra --no-cpu-baseline --roof-calls 5 --param memo_grid=$G ${EXTRA:-} > $O/b${B}_g$G.json 2> $O/b${B}_g$G.err || { tail $O/b${B}_g$G.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/b${B}_g$G.json'))
print('budget $B grid $G', '%.3e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], d['device_ms']['alone'])"
done
