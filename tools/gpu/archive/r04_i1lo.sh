#!/bin/bash
# Round 4: one call at a time at a set stage-0 budget around the automatic
# budget's low value (16), lane mode; 14 with a larger heavy-stage grid cap
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/i1lo; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
  for b in 15 16 17; do
    n=i1_${b}_$r
    step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget $b --param heavy_mode=1
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
  for g in 4096 6144; do
    n=i1_14_g${g}_$r
    step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget 14 --param heavy_mode=1 --param memo_grid=$g
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
  n=i1_auto_$r
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
done
