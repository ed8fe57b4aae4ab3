#!/bin/bash
# Round 6: the heavy stage's mode for one call at a time -- wave mode
# (heavy_mode 0) against lane mode (1) on heavy lists of ~160 to ~16k
# histories (config 2 at budget 20 on 10k / 100k / 1M histories; config 5's
# 100k at the automatic stage-0w budget), to set wave_max.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_wavemax
mkdir -p $O
run() {  # tag, bench args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -3 $O/$t.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/$t.json'))
print('$t', '%.3e' % d['value'], 'ms/call %.4f' % d['ms_per_step'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
}
for r in 1 2; do
  for m in 0 1; do
    run c2_1m_m$m.$r --steps 50 --warmup 5 --stage0-budget 20 --param heavy_mode=$m
    run c2_100k_m$m.$r --n-hist 100000 --steps 100 --warmup 5 --stage0-budget 20 --param heavy_mode=$m
    run c2_10k_m$m.$r --n-hist 10000 --steps 100 --warmup 5 --stage0-budget 20 --param heavy_mode=$m
    run c5_100k_m$m.$r --config bank_6x24 --n-hist 100000 --steps 50 --warmup 5 --stage0-budget -1 --param heavy_mode=$m
    run c3_100k_m$m.$r --config bank_4x16_bugs --n-hist 100000 --steps 50 --warmup 5 --stage0-budget -1 --param heavy_mode=$m
  done
done
