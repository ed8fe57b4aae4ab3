#!/bin/bash
# One rank: the RCCL path against none at 4 calls in flight, on the box's 4
# hardware queues and with 6 / 8 (the slot streams, the all-reduce's stream
# and RCCL's own share the queues otherwise).
set -o pipefail
export PYTHONUNBUFFERED=1 QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_q
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in none dist dq6 dq8 nq8; do
    E=""; A=""
    case $v in
      dist) E="QSMD_BENCH_DIST=1";;
      dq6) E="QSMD_BENCH_DIST=1"; A="--hw-queues 6";;
      dq8) E="QSMD_BENCH_DIST=1"; A="--hw-queues 8";;
      nq8) A="--hw-queues 8";;
    esac
    env $E timeout -k 10 120 python bench.py $B $A > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'])"
    grep enqueue_ms $O/$v.$r.err
  done
done
