#!/bin/bash
# A/B: lane mode's DFS loop with a wavefront-uniform iteration count (the
# hand-off cap and the 1024-iteration checks outside the inner loop; the
# library in lib/) against the loop before it, with the entry wait only
# (ablib/ewait.so).  The full GPU suite first.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_loop
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="stage0_budget=18 heavy_mode=1 memo_lds=0"
for v in new ewait; do
  E=""; [ $v != new ] && E="QSMD_LIB_PATH=$PWD/ablib/$v.so"
  env $E timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  echo "$v: $(cat $O/ms.json)"
done
for r in 1 2 3; do
  for v in new ewait; do
    E=""; [ $v != new ] && E="QSMD_LIB_PATH=$PWD/ablib/$v.so"
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('$v $r %.3e' % d['value'], d['device_ms']['alone'])"
    env $E timeout -k 10 120 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/i.json 2> $O/i.err || { tail $O/i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/i.json')); print('$v i1 $r %.3e' % d['value'])"
  done
done
