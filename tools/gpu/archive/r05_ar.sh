#!/bin/bash
# One rank: the RCCL path with and without the window's one all-reduce
# (QSMD_BENCH_NOAR_WINDOW=1: the communicator created in the warm-up, no
# collective in the window), and the latency of one all-reduce alone.
set -o pipefail
export PYTHONUNBUFFERED=1 QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_ar
mkdir -p $O
timeout -k 10 120 python tools/micro/allreduce_latency.py > $O/lat.txt 2> $O/lat.err || { tail $O/lat.err; exit 1; }
cat $O/lat.txt
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in none dist noarw; do
    E=""
    case $v in
      dist) E="QSMD_BENCH_DIST=1";;
      noarw) E="QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR_WINDOW=1";;
    esac
    env $E timeout -k 10 120 python bench.py $B > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'])"
    grep enqueue_ms $O/$v.$r.err
  done
done
