#!/bin/bash
# Round 4: the per-call timing events (two event records and the stage-0
# launch's start/stop events) inside the timed window, on and off
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/tev; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
T=600 step tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "timing or generated_configs"
tail -2 $O/tests.out
for r in 1 2 3; do
for te in 1 0; do
  n=drv_${te}_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --timing-events $te
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4), 'alone', round(d['device_ms']['alone']['call_mean'],4))"
done
done
for te in 1 0; do
  n=d200_${te}
  step $n python bench.py --no-cpu-baseline --no-extra --timing-events $te
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  n=i1_${te}
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --timing-events $te
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
done
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --roof-calls 1 --timing-events 0 > $O/trace.log 2>&1 && echo traced
