#!/bin/bash
# The batch path's totals over gloo (no RCCL communicator) against none and
# against the RCCL totals, one rank at the driver's 20 steps; then the GPU
# multi-process tests (incl. bench.py under torchrun with 2 ranks on cuda:0).
set -o pipefail
export PYTHONUNBUFFERED=1 QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_gloo
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in none gloo rccl; do
    E=""
    case $v in
      gloo) E="QSMD_BENCH_DIST=1";;
      rccl) E="QSMD_BENCH_DIST=1 QSMD_BENCH_COUNTERS=rccl";;
    esac
    env $E timeout -k 10 120 python bench.py $B > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['verdicts']['checked'], d['config']['counters'])"
    grep enqueue_ms $O/$v.$r.err
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -6 $O/pytest.log
