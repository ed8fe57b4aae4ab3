#!/bin/bash
# Round 6: lane mode's written-slot map plus an LDS fingerprint per slot (8 bits of the
# hash under the slot) against the map alone -- the lane-mode tests, the heavy stage's
# anatomy (HBM probe fraction), then A/B (ablib/base.so vs ablib/fp.so)
# at the driver's command and one call at a time, 3 rounds each.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_fp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lane_mode or resume or memo" > $O/tests.txt 2>&1 &&
tail -2 $O/tests.txt || exit 1
K="stage0_budget=20 heavy_mode=1 memo_lds=0"
for v in base fp; do
  QSMD_LIB_PATH=$PWD/ablib/$v.so timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms_c2_$v.json 2> $O/ms_c2_$v.err || exit 1
  python3 -c "
import json; d = json.load(open('$O/ms_c2_$v.json'))
print('$v', d['fraction_of_wave_iterations'], 'hits', d['memo_hits_total'], 'max it', d['max_iterations'], 'cyc', d['cycles_per_iteration'])
"
done
timeout -k 10 600 python tools/ab.py ablib/base.so ablib/fp.so 3 --steps 20 --warmup 5 --inflight 4 > $O/ab_driver.txt 2>&1 && tail -2 $O/ab_driver.txt &&
timeout -k 10 600 python tools/ab.py ablib/base.so ablib/fp.so 3 --steps 50 --warmup 5 --inflight 1 > $O/ab_one.txt 2>&1 && tail -2 $O/ab_one.txt
