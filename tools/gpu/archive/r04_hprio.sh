#!/bin/bash
# Round 4: issue priority (s_setprio) for the lane-mode heavy stage's wavefronts
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/hp; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
for v in prio0 prio2 prio3; do
  n=drv_${v}_$r
  step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
