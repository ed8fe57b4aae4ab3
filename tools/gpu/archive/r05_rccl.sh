#!/bin/bash
# Round 5: one rank with and without the RCCL path at the
# driver's 20 steps -- 3 runs each of none / the RCCL path / the RCCL path
# without its all-reduce -- then a kernel + HIP API trace of one run each way
# (rocprofv3 --kernel-trace --hip-trace, the program directly after --).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_rccl
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
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --stats -d $O/trace_none -o run --output-format csv -- python3 bench.py $B > $O/trace_none.json 2> $O/trace_none.err || exit 1
QSMD_BENCH_DIST=1 timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --stats -d $O/trace_dist -o run --output-format csv -- python3 bench.py $B > $O/trace_dist.json 2> $O/trace_dist.err || exit 1
ls -R $O | head -40
