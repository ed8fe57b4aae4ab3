#!/bin/bash
# Round 4: lane mode's per-level entry counts in HBM instead of LDS (10 KB
# of LDS per heavy-stage workgroup instead of 14) -- the lane-mode tests on
# the new build, then the driver's command and one call at a time, A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/entryhbm; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
T=600 step tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "memo_after or sharded_heavy or lane_mode or generated_configs or cascade"
tail -2 $O/tests.out
for r in 1 2 3; do
for v in base entryhbm; do
  n=drv_${v}_$r
  step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
for v in base entryhbm; do
  n=i1_${v}
  step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget 16 --param heavy_mode=1
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  n=c3_${v}
  step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --config bank_4x16_bugs --stage0-budget 32
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
