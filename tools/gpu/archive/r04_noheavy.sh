#!/bin/bash
# Round 4: lone stage 0 against its budget, product vs the build without the heavy-list append
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/nh; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for b in ${BUDGETS:-16 20 22 24 26}; do
  for v in prod noheavy; do
    L=ablib/$v.so; [ $v = prod ] && L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so
    step lone_${v}_$b env QSMD_LIB_PATH=$L python tools/stage0_anatomy.py 1000000 $b
    python3 -c "import json; d=json.load(open('$O/lone_${v}_$b.out')); x=d['stage0_ms_events'][2:]; print('lone $v budget $b', round(sum(x)/len(x),4))"
  done
done
