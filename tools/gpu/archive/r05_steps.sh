#!/bin/bash
# The window's fixed cost: the driver's command at 10 / 20 / 40 / 80 / 160
# steps (time = fixed + K x per-step), with the host-time split, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
export QSMD_BENCH_HOSTTIME=1
O=gpurun_out/steps
mkdir -p $O
for r in 1 2; do
  for k in 10 20 40 80 160; do
    timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-extra --no-cpu-baseline > $O/b_${k}_$r.json 2> $O/b_${k}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${k}_$r.json')); print($k, $r, '%.3e' % d['value'], 'ms %.4f' % (d['ms_per_step'] * $k))"
    grep enqueue_ms $O/b_${k}_$r.err | tail -1
  done
done
