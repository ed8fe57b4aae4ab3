#!/bin/bash
# One rank, the previous bench (RCCL all-reduce of the counters at the
# window's end, on its own stream): none / RCCL / RCCL with
# NCCL_IGNORE_CPU_AFFINITY=1 (RCCL pins its threads, and during init the
# caller's, to the GPU's NUMA cores) / RCCL with the NCCL debug banner off.
set -o pipefail
export PYTHONUNBUFFERED=1 QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_aff
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
python3 -c "import os; print('affinity', sorted(os.sched_getaffinity(0))[:4], len(os.sched_getaffinity(0)))"
for r in 1 2 3; do
  for v in none dist aff; do
    E=""
    case $v in
      dist) E="QSMD_BENCH_DIST=1";;
      aff) E="QSMD_BENCH_DIST=1 NCCL_IGNORE_CPU_AFFINITY=1";;
    esac
    env $E timeout -k 10 120 python bench_prev.py $B > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); print('$v $r %.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'])"
    grep enqueue_ms $O/$v.$r.err || true
  done
done
