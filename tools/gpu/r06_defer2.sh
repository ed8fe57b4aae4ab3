#!/bin/bash
# Round 6: the sharded deferred list with stage 0's list mode compiled out
# -- the cascade / fold / wide tests, then A/B against the build before the
# change (ablib/fold.so) at the driver's command, 4 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_defer2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "stage0w or cascade or wide or fold or stage0_budget or automatic or full_size or probe" > $O/tests.txt 2>&1 &&
tail -2 $O/tests.txt &&
timeout -k 10 600 python tools/ab.py ablib/fold.so ablib/cur.so 4 --steps 20 --warmup 5 --inflight 4 > $O/ab.txt 2>&1 &&
tail -2 $O/ab.txt
