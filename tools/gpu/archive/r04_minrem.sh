#!/bin/bash
# Round 4: lane mode's memo only above min_rem remaining events -- parity, then the driver's command
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/mr; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "memo_after or lane_mode or generated_configs" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for mr in ${MRS:-0 4 8 12 16}; do
  n=drv_${mr}_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param memo_min_rem=$mr
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
for cfg in "memo_lds=2,memo_lds_entries=16" "memo_lds=2,memo_lds_entries=64"; do
  n=drv_lds_$(echo $cfg | tr ',=' '__')_$r
  args=""; for kv in $(echo $cfg | tr ',' ' '); do args="$args --param $kv"; done
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra $args
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
