#!/bin/bash
# A/B: lane mode's insert with the level's entry count read beside the key's
# balances (lib/) against the entry count read first (abtmp/prev.so).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_ent
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lane or memo or resume or fold or giant" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="stage0_budget=18 heavy_mode=1 memo_lds=0"
for v in new prev; do
  E=""; [ $v != new ] && E="QSMD_LIB_PATH=$PWD/abtmp/$v.so"
  env $E timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ms.json')); print('$v', d['cycles_per_iteration'], d['stage_span_us'])"
done
for r in 1 2 3; do
  for v in new prev; do
    E=""; [ $v != new ] && E="QSMD_LIB_PATH=$PWD/abtmp/$v.so"
    env $E timeout -k 10 120 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/i.json 2> $O/i.err || { tail $O/i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/i.json')); print('$v i1 $r %.3e' % d['value'], round(d['device_ms']['alone']['heavy_mean']*1e3,1))"
  done
done
