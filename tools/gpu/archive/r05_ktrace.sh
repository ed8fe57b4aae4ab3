#!/bin/bash
# One rank, the previous bench: a kernel trace (no API trace) of the
# driver's 20 steps without and with the RCCL path, for the window's GPU
# timeline.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp QSMD_BENCH_HOSTTIME=1
O=gpurun_out/r05_ktrace
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/none -o run --output-format csv -- python3 bench_prev.py $B > $O/none.json 2> $O/none.err || { tail $O/none.err; exit 1; }
QSMD_BENCH_DIST=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $O/dist -o run --output-format csv -- python3 bench_prev.py $B > $O/dist.json 2> $O/dist.err || { tail $O/dist.err; exit 1; }
for v in none dist; do python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v %.3e' % d['value'])"; grep enqueue_ms $O/$v.err; done
