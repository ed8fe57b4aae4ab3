#!/bin/bash
# Round 4: the automatic stage-0 budget -- the GPU suite, one call at a time
# at the library's defaults (automatic) and at a set 32, the driver's
# command, the 200-step default with the extra configs
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/auto; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
T=900 step suite python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
tail -2 $O/suite.out
for r in 1 2; do
  n=i1_auto_$r
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
done
n=i1_32
step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget 32
python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
for c in bank_4x16_bugs ticket_2x10; do
  n=i1_auto_$c
  step $n python bench.py --inflight 1 --steps 40 --warmup 10 --no-cpu-baseline --no-extra --config $c
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  n=i1_32_$c
  step $n python bench.py --inflight 1 --steps 40 --warmup 10 --no-cpu-baseline --no-extra --config $c --stage0-budget 32
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
done
n=drv
step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4), 'alone', round(d['device_ms']['alone']['call_mean'],4))"
T=400 step d200 python bench.py --no-cpu-baseline
python3 -c "
import json; d=json.load(open('$O/d200.out')); print('d200', round(d['value']/1e9,3))
for k,v in d['extra']['configs'].items(): print(' ', k, v.get('histories_per_sec'), v.get('ms_per_history'), v.get('mismatches_vs_oracle'))"
