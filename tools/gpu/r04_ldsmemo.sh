#!/bin/bash
# Round 4: lane mode's memo tables in LDS vs HBM at the driver's command (after resume / memo_after)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/lm; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for cfg in "0 64" "2 16" "2 32" "2 64" "1 64"; do
  set -- $cfg
  n=drv_$1_$2_$r
  step $n python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param memo_lds=$1 --param memo_lds_entries=$2
  python3 -c "import json; d=json.load(open('$O/$n.out')); print('$n', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4), d['config'].get('heavy_stage'))"
done
done
