#!/bin/bash
# Round 6: stage 0's deferred list sharded like its heavy list -- the GPU
# suite, then config 5 (100k 6x24, every history deferred to stage 0w; 3
# calls in flight, the bench's extra-config shape) and config 2 (the
# driver's command) against the previous build (ablib/fold.so).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_defer
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
tail -2 $O/tests.txt || { tail -30 $O/tests.txt; exit 1; }
for r in 1 2; do
  for v in old new; do
    L=$PWD/quickcheck-state-machine-distributed_amd/lib/libqsmd.so; [ $v = old ] && L=$PWD/ablib/fold.so
    QSMD_LIB_PATH=$L timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget -1 > $O/c5_$v.$r.json 2> $O/c5_$v.$r.err || exit 1
    QSMD_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/c2_$v.$r.json 2> $O/c2_$v.$r.err || exit 1
    python3 -c "
import json
for c in ('c5', 'c2'):
    d = json.load(open('$O/' + c + '_$v.$r.json'))
    print(c, '$v', '%.3e' % d['value'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
