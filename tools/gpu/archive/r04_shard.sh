#!/bin/bash
# Round 4: stage 0's heavy list in shards -- a parity subset, lone stage 0
# against the budget, the driver's command and one call at a time against
# the budget.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/shard; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "generated_configs or lane_mode or wave_mode or packed or budget or early_exit or device_resident or grids or knobs or lds" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for b in ${BUDGETS:-16 18 20 22 24 26}; do
  step lone_$b python tools/stage0_anatomy.py 1000000 $b
  python3 -c "import json; d=json.load(open('$O/lone_$b.out')); x=d['stage0_ms_events'][2:]; print('lone budget $b', round(sum(x)/len(x),4))"
done
for r in 1 2; do
for b in ${DBUDGETS:-18 20 22 24 26}; do
  step drv_${b}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b
  python3 -c "import json; d=json.load(open('$O/drv_${b}_$r.out')); print('drv budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
