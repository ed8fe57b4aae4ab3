#!/bin/bash
# Round 6: lane mode for heavy lists of short searches (heavy_mode 2) --
# the GPU suite, then one call at a time with the library's defaults on
# configs 1 / 2 (1M, 2k, 300) / 3 (100k, 10k) / 5 (100k).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_short
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.txt 2>&1 &&
tail -1 $O/tests.txt || { tail -30 $O/tests.txt; exit 1; }
run() {  # tag, bench args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline --stage0-budget -1 "$@" > $O/$t.json 2> $O/$t.err || { tail -3 $O/$t.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/$t.json'))
print('$t', '%.3e' % d['value'], 'ms/call %.4f' % d['ms_per_step'], {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
}
run c2_1m --steps 50 --warmup 5
run c1_1m --config ticket_2x10 --steps 50 --warmup 5
run c2_2k --n-hist 2000 --steps 200 --warmup 5
run c2_300 --n-hist 300 --steps 200 --warmup 5
run c3_100k --config bank_4x16_bugs --n-hist 100000 --steps 50 --warmup 5
run c3_10k --config bank_4x16_bugs --n-hist 10000 --steps 100 --warmup 5
run c5_100k --config bank_6x24 --n-hist 100000 --steps 50 --warmup 5
