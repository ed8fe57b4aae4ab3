#!/bin/bash
# A/B: lane mode's probe skipped when the lane never wrote that slot for its
# history (the written-slot map, memo.hip) against the build without the
# map (ablib/nomap.so).  The lane-mode / memo parity tests first.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_map
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "lane or memo or resume or fold or giant or stress or full_size" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="stage0_budget=18 heavy_mode=1 memo_lds=0"
for v in new nomap; do
  E=""; [ $v != new ] && E="QSMD_LIB_PATH=$PWD/ablib/$v.so"
  env $E timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  echo "$v: $(cat $O/ms.json)"
done
for r in 1 2 3; do
  for v in new nomap; do
    E=""; [ $v != new ] && E="QSMD_LIB_PATH=$PWD/ablib/$v.so"
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('$v $r %.3e' % d['value'], d['device_ms']['alone'])"
    env $E timeout -k 10 120 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/i.json 2> $O/i.err || { tail $O/i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/i.json')); print('$v i1 $r %.3e' % d['value'])"
  done
done
