#!/bin/bash
# One rank: where the window's host time goes with and without the RCCL
# path's one in-window all-reduce (bench.py QSMD_BENCH_HOSTTIME=1 prints the
# enqueue / drain / synchronize split of the timed window on stderr).
set -o pipefail
export PYTHONUNBUFFERED=1 QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_host
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in none dist noar; do
    case $v in
      none) E="";;
      dist) E="QSMD_BENCH_DIST=1";;
      noar) E="QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR=1";;
    esac
    env $E timeout -k 10 120 python bench.py $B > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'])"
    grep enqueue_ms $O/$v.$r.err
  done
done
