#!/bin/bash
# Round 6: the memo slot from a register fold of the balances (LaneDFS::fold)
# -- the lane-mode parity tests, the heavy stage's anatomy (fold check: 0
# mismatches) on configs 2 and 3, then A/B against the previous build.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_fold
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lane_mode or resume or fold or memo or heavy or tail or bucket or stress or adversarial or wide" > $O/tests.txt 2>&1 &&
tail -2 $O/tests.txt &&
QSMD_LIB_PATH=$PWD/ablib/B.so timeout -k 10 120 python tools/memo_stats.py bank_4x16_bugs 1250000 > $O/ms_c3.json 2> $O/ms_c3.err &&
cat $O/ms_c3.json &&
bash tools/gpu/r06_ab.sh ablib/A.so ablib/B.so 3
