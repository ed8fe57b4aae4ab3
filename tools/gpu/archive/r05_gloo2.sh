#!/bin/bash
# Same-box A/B, one rank, the driver's 20 steps: the previous bench (per-block
# counters, no process group) against this one (a row per step, one sum at
# the window's end) without a process group, with the gloo exchange and with
# the RCCL exchange.
set -o pipefail
export PYTHONUNBUFFERED=1 QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_gloo2
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in none gloo; do
    E=""; P=bench.py
    case $v in
      prev) P=bench_prev.py;;
      gloo) E="QSMD_BENCH_DIST=1";;
      rccl) E="QSMD_BENCH_DIST=1 QSMD_BENCH_COUNTERS=rccl";;
    esac
    env $E timeout -k 10 120 python $P $B > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'])"
    grep enqueue_ms $O/$v.$r.err || true
  done
done
