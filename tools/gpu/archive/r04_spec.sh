#!/bin/bash
# Round 4: lane mode's memo probe resolved one step later -- parity, then the driver's command and one call at a time
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/sp; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "spec_probe or lane_mode or memo_after or generated_configs or bench_knobs or model_error or handoff or budget" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for sp in 0 1; do
  n=drv_${sp}_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param memo_spec=$sp
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  n=i1_${sp}_$r
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget 16 --param heavy_mode=1 --param memo_spec=$sp
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  n=c3_${sp}_$r
  step $n python bench.py --config bank_4x16_bugs --steps 10 --warmup 3 --no-cpu-baseline --no-extra --param memo_spec=$sp
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', '%.3e' % d['value'], 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
