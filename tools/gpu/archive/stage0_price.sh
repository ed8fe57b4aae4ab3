#!/bin/bash
# Round 4: the price of stage 0's parts on a lone call (config 2, bench knobs):
# the product build, the search run twice (its marginal cost), no search
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/price; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for v in prod search2 s0nosearch; do
  L=ablib/$v.so; [ $v = prod ] && L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so
  step lone_${v}_$r env QSMD_LIB_PATH=$L python tools/stage0_anatomy.py 1000000 26
  python3 -c "import json; d=json.load(open('$O/lone_${v}_$r.out')); x=d['stage0_ms_events'][2:]; print('$v', round(sum(x)/len(x),4), [round(y,4) for y in x])"
done
done
