#!/bin/bash
# Round 4: the call's completion event (hipEventRecord, timing disabled) --
# a diagnostic build that records it only on a context's first call, A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/nodone; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
  for v in base2 nodone; do
    n=i1_${v}_$r
    step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --inflight 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extra
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
    n=drv_${v}_$r
    step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
