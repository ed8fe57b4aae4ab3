#!/bin/bash
# Round 4: the GPU suite, then one call at a time with the timing events off
# (library default) at the library's knobs and in lane mode, and the
# driver's command
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/sync2; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
if [ -z "$NOSUITE" ]; then
T=900 step suite python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
tail -2 $O/suite.out
fi
for r in 1 2; do
  n=i1_lib_$r
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  for b in 16 18 20; do
    n=i1_lane${b}_$r
    step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget $b --param heavy_mode=1
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
  n=drv_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4), 'alone', round(d['device_ms']['alone']['call_mean'],4))"
done
