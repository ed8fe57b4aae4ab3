#!/bin/bash
# Early-exit leg (BASELINE config 3): fixed 262144-history rounds against
# the geometric schedule (qsmd.dist.early_chunks), plus the GPU early-exit
# parity test.  Every GPU step has its own limit.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/early
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for fc in 0 4096 1024 16384; do
  timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 --no-cpu-baseline --first-chunk $fc > $O/early_$fc.json 2> $O/early_$fc.err || exit 1
  python3 -c "import json; d=json.load(open('$O/early_$fc.json')); e=d['early_exit']; print($fc, '%.3e' % d['value'], 'ms %.4f' % d['ms_per_step'], {k: e[k] for k in e if k not in ('histories','steps')})"
done
