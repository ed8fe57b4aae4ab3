#!/bin/bash
# Round 6: lane mode with 16 / 32 / 64 histories per workgroup
# (memo_group_lanes) -- the parity tests, then the driver's command, one call
# at a time and config 5 (3 in flight), 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_gl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "group_lanes" > $O/tests.txt 2>&1 &&
tail -2 $O/tests.txt || exit 1
run() {  # tag, bench args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -3 $O/$t.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/$t.json'))
print('$t', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
}
for r in 1 2; do
  for g in 64 32 16; do
    run drv_g$g.$r --steps 20 --warmup 5 --param memo_group_lanes=$g
    run one_g$g.$r --steps 50 --warmup 5 --inflight 1 --param memo_group_lanes=$g
    run c5_g$g.$r --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --stage0-budget -1 --param memo_group_lanes=$g
  done
done
