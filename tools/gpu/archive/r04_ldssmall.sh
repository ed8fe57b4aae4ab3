#!/bin/bash
# Round 4: lane mode's LDS memo tables with few entries per lane (several
# workgroups per CU) for one call at a time (automatic budget: 16 on config 2)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/ldssmall; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
T=600 step tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "lane_mode or automatic"
tail -2 $O/tests.out
for r in 1 2; do
  for e in 4 64; do
    n=i1_e${e}_$r
    step $n python bench.py --inflight 1 --steps 200 --warmup 10 --no-cpu-baseline --no-extra --param memo_lds_entries=$e
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
  for e in 4 8; do
    n=i1_force_e${e}_$r
    step $n python bench.py --inflight 1 --steps 200 --warmup 10 --no-cpu-baseline --no-extra --param memo_lds_entries=$e --param memo_lds=2
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
  done
done
for c in bank_4x16_bugs ticket_2x10; do
  n=i1_e4_$c
  step $n python bench.py --inflight 1 --steps 40 --warmup 10 --no-cpu-baseline --no-extra --config $c --param memo_lds_entries=4
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],4))"
done
