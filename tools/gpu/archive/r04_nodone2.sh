#!/bin/bash
# Round 4: the completion event only for contexts used from two streams --
# the GPU suite, smoke, then one call at a time and the driver's command
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/nodone2; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
T=900 step suite python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
tail -2 $O/suite.out
step smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 $O/smoke.out
for r in 1 2 3; do
  n=i1_$r
  step $n python bench.py --inflight 1 --steps 200 --warmup 20 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  n=drv_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3))"
done
