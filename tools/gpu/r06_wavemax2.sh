#!/bin/bash
# Round 6: wave (heavy_mode 0) against lane mode (1), one call at a time, at
# the small end and on config 1: config 1 (1M, the automatic budget),
# config 2 on 2000 and 300 histories, config 3 on 10k.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_wavemax2
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
    run c1_1m_m$m.$r --config ticket_2x10 --steps 50 --warmup 5 --stage0-budget -1 --param heavy_mode=$m
    run c2_2k_m$m.$r --n-hist 2000 --steps 200 --warmup 5 --stage0-budget -1 --param heavy_mode=$m
    run c2_300_m$m.$r --n-hist 300 --steps 200 --warmup 5 --stage0-budget -1 --param heavy_mode=$m
    run c3_10k_m$m.$r --config bank_4x16_bugs --n-hist 10000 --steps 100 --warmup 5 --stage0-budget -1 --param heavy_mode=$m
  done
done
