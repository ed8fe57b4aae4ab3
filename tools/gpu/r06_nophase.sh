#!/bin/bash
# Round 6: the heavy stage's cycles per iteration without the phase stamps
# (tools/diag/memo_nophase.patch): tools/memo_stats.py on configs 2 and 3 at
# the bench's knobs with the stamps (ablib/fold.so) and without.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_nophase
mkdir -p $O
K="stage0_budget=20 heavy_mode=1 memo_lds=0"
for v in fold nophase; do
  QSMD_LIB_PATH=$PWD/ablib/$v.so timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms_c2_$v.json 2> $O/ms_c2_$v.err &&
  QSMD_LIB_PATH=$PWD/ablib/$v.so timeout -k 10 120 python tools/memo_stats.py bank_4x16_bugs 1250000 > $O/ms_c3_$v.json 2> $O/ms_c3_$v.err || exit 1
  python3 -c "
import json
for c in ('c2', 'c3'):
    d = json.load(open('$O/ms_' + c + '_$v.json'))
    print('$v', c, 'cycles/iter', d['cycles_per_iteration'], 'max it', d['max_iterations']['max'], 'span', d['stage_span_us'])
"
done
