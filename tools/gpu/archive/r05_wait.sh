#!/bin/bash
# A/B: lane mode's DFS loop entered with no memory operation outstanding
# (memo.hip: the compiler's wait for the memo insert's stores leaves the
# loop) against the build without that wait (ablib/nowait.so).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_wait
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lane or memo or resume or fold" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="stage0_budget=18 heavy_mode=1 memo_lds=0"
for v in new nowait; do
  E=""; [ $v = nowait ] && E="QSMD_LIB_PATH=$PWD/ablib/nowait.so"
  env $E timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  echo "$v: $(cat $O/ms.json)"
done
for r in 1 2 3; do
  for v in new nowait; do
    E=""; [ $v = nowait ] && E="QSMD_LIB_PATH=$PWD/ablib/nowait.so"
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('$v $r %.3e' % d['value'], d['device_ms']['alone'])"
    env $E timeout -k 10 120 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/i.json 2> $O/i.err || { tail $O/i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/i.json')); print('$v i1 $r %.3e' % d['value'])"
  done
done
