#!/bin/bash
# Round 4: stage 0 through the plain launch when untimed (hipLaunchKernel
# instead of hipExtLaunchKernel with null events), A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/plain; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2 3; do
  for v in base3 plain; do
    n=i1_${v}_$r
    step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --inflight 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extra
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
    n=d200_${v}_$r
    step $n env QSMD_LIB_PATH=ablib/$v.so python bench.py --no-cpu-baseline --no-extra
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
