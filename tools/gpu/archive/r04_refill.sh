#!/bin/bash
# Round 4: lane mode with lane refill -- parity, then the driver's command
# against the refill knobs and the stage-0 budget.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/rf; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "refill or lane_mode or memo_after or generated_configs or sharded or bench_knobs or budget or early or witness or model_error or handoff" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for cfg in "0 16 16 0" "1 16 16 0" "1 8 8 0" "1 32 32 0" "1 16 16 512"; do
  set -- $cfg
  for b in ${DBUDGETS:-16 18}; do
    n=drv_$1_$2_$3_$4_${b}_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b --param memo_refill=$1 --param refill_steps=$2 --param refill_min=$3 --param refill_grid=$4
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
done
