#!/bin/bash
# Round 4: lone stage 0 against its node budget (stage0_anatomy: heavy list on, HBM memo)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/s0b; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for b in ${BUDGETS:-16 17 18 20 22 24 26 28 32}; do
  step lone_$b python tools/stage0_anatomy.py 1000000 $b
  python3 -c "import json; d=json.load(open('$O/lone_$b.out')); x=d['stage0_ms_events'][2:]; print('lone budget $b', round(sum(x)/len(x),4), {k: v for k, v in d.items() if k != 'stage0_ms_events'})"
done
