#!/bin/bash
# Round-5 baseline: the heavy stage's per-group anatomy at the bench's knobs
# (tools/memo_stats.py) and the driver's bench command on the current tree.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_base
mkdir -p $O
K="stage0_budget=18 heavy_mode=1 memo_lds=0"
timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/memo_stats.json 2> $O/memo_stats.err &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err
rc=$?
cat $O/memo_stats.json
python3 -c "
import json; d=json.load(open('$O/bench20.json')); print('%.3e' % d['value'], d['device_ms'])"
exit $rc
