#!/bin/bash
# Round 6: stage 0 / 0w compiled with the max-ILP scheduler (Makefile
# FLAGS_compact) -- the GPU suite, then against the default build
# (ablib/base.so): the driver's command (3 rounds, tools/ab.py) and config 5
# (the G64 stage, 3 calls in flight, 2 rounds).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_sched2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.txt 2>&1 &&
tail -1 $O/tests.txt || { tail -30 $O/tests.txt; exit 1; }
timeout -k 10 600 python tools/ab.py ablib/base.so ablib/new.so 3 --steps 20 --warmup 5 --inflight 4 > $O/ab_driver.txt 2>&1 && tail -2 $O/ab_driver.txt || exit 1
for r in 1 2; do
  for v in base new; do
    QSMD_LIB_PATH=$PWD/ablib/$v.so timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget -1 > $O/c5_$v.$r.json 2> $O/c5_$v.$r.err || exit 1
    python3 -c "
import json; d = json.load(open('$O/c5_$v.$r.json'))
print('c5 $v $r', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
