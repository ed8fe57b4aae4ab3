#!/bin/bash
# Round 4: the driver's command with the heavy stage removed (diagnostic
# build: budget-stopped histories reported BUDGET) -- the headroom a cheaper
# heavy stage could give.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/hr; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for v in prod noheavy; do
  L=ablib/$v.so; [ $v = prod ] && L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so
  for b in 16 20; do
    step drv_${v}_${b}_$r env QSMD_LIB_PATH=$L python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b
    python3 -c "import json; d=json.load(open('$O/drv_${v}_${b}_$r.out')); print('drv $v budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
done
