#!/bin/bash
# Round 4: lane mode in two passes (lane_pass_cap) -- the parity tests, then
# the driver's command and one call at a time against the first pass's cap
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/twopass; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
T=600 step tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "two_passes or memo_after or sharded_heavy or lane_mode"
tail -2 $O/tests.out
for r in 1 2; do
  for pc in ${CAPS:-0 4 8 12 16 24}; do
    n=drv_${pc}_$r
    step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param lane_pass_cap=$pc
    python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'alone', round(d['device_ms']['alone']['call_mean'],4), 'mism', d.get('mismatches_vs_oracle'))"
  done
done
for pc in ${CAPS:-0 4 8 12 16 24}; do
  n=i1_${pc}
  step $n python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --stage0-budget 16 \
       --param heavy_mode=1 --param lane_pass_cap=$pc
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
