#!/bin/bash
# Round 5: the folded lane-mode tail.  The GPU suite on the new default
# (fold 1: no stage-0w launch after a call that deferred nothing), then the
# driver's command A/B: fold 0 (round 4's chain), fold 1, and the diagnostic
# fold 2 (no giant launch either; ablib/fold2.so), alternating.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_fold
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for steps in 20 100; do
for r in 1 2 3; do
  for v in 0 1 2; do
    if [ $v = 2 ]; then L="QSMD_LIB_PATH=$PWD/ablib/fold2.so"; else L=""; fi
    env $L timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-extra --no-cpu-baseline --param fold=$v > $O/b_${steps}_${v}_$r.json 2> $O/b_${steps}_${v}_$r.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/b_${steps}_${v}_$r.json')); print('steps $steps fold $v round $r %.3e' % d['value'], 'alone call %.4f' % d['device_ms']['alone']['call_mean'])"
  done
done
done
