#!/bin/bash
# Round 4, final: the round's measurements (tools/gpu/measure.sh) with 4
# calls in flight on a lone rank, then the stage-0 budget at that depth
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu/measure.sh > gpurun_out/final4_measure.log 2>&1 || { tail -30 gpurun_out/final4_measure.log; exit 1; }
grep -E "^bench_" gpurun_out/final4_measure.log
O=gpurun_out/final4; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
  for b in 16 18 20 22; do
    n=drv_b${b}_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
  done
done
