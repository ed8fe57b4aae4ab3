#!/bin/bash
# The early-exit step: the GPU early-exit parity tests, the call against its
# floor (tools/micro/early_split.py), the bench leg at both schedules.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/early2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/micro/early_split.py > $O/split.txt 2>&1 || { tail $O/split.txt; exit 1; }
cat $O/split.txt
for fc in 0 4096; do
  timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 --no-cpu-baseline --first-chunk $fc > $O/early_$fc.json 2> $O/early_$fc.err || exit 1
  python3 -c "import json; d=json.load(open('$O/early_$fc.json')); e=d['early_exit']; print($fc, '%.3e' % d['value'], 'ms %.4f' % d['ms_per_step'], e['searched'], e['rounds'], e['totals'])"
done
