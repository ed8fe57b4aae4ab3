#!/bin/bash
# Round 6: the lane-mode heavy stage with the memo key computed once per node
# (pending entries, memo.hip) against round 5's build (ablib/base_r05.so):
# the GPU suite, the per-group anatomy (tools/memo_stats.py) of both builds
# at the bench's knobs, then A/B of the driver's command and of one call at
# a time (tools/ab.py).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_memo
mkdir -p $O
K="stage0_budget=20 heavy_mode=1 memo_lds=0"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/memo_stats_new.json 2> $O/memo_stats_new.err &&
for ma in 20 0; do timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K memo_after=$ma > $O/memo_stats_ma$ma.json 2> $O/memo_stats_ma$ma.err || exit 1; done
cat $O/memo_stats_new.json $O/memo_stats_ma20.json $O/memo_stats_ma0.json &&
timeout -k 10 400 python tools/ab.py ablib/base_r05.so quickcheck-state-machine-distributed_amd/lib/libqsmd.so 3 --steps 20 --warmup 5 --inflight 4 &&
timeout -k 10 300 python tools/ab.py ablib/base_r05.so quickcheck-state-machine-distributed_amd/lib/libqsmd.so 3 --steps 50 --warmup 5 --inflight 1
