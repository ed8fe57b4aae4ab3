#!/bin/bash
# Round 4: lane mode with the memo joining a search after N nodes -- the
# parity tests, then the driver's command against N.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/ma; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "memo_after or lane_mode or generated_configs" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for ma in ${MAS:-0 32 64 128 512 1000000}; do
  for b in ${DBUDGETS:-16 20}; do
    step drv_${ma}_${b}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b --param memo_after=$ma
    python3 -c "import json; d=json.load(open('$O/drv_${ma}_${b}_$r.out')); print('drv memo_after $ma budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
done
