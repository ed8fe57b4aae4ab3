#!/bin/bash
# One rank at the driver's 20 steps: no process group / RCCL counters after
# the window (the default) / inside it / gloo after it; then the GPU
# multi-process tests.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_cnt
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in none after rccl gloo; do
    E=""
    case $v in
      after) E="QSMD_BENCH_DIST=1";;
      rccl) E="QSMD_BENCH_DIST=1 QSMD_BENCH_COUNTERS=rccl";;
      gloo) E="QSMD_BENCH_DIST=1 QSMD_BENCH_COUNTERS=gloo";;
    esac
    env $E timeout -k 10 120 python bench.py $B > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'exchange_ms', d['config'].get('exchange_ms'), d['verdicts']['checked'])"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -4 $O/pytest.log
