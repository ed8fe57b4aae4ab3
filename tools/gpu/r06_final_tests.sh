#!/bin/bash
# Round 6 on the final tree: the GPU suite, smoke(), and the randomised
# parity sweep (random knobs per batch, incl. the round's tail_cap /
# tail_min / heavy_buckets and the early-exit flag; then the wide any-shape
# sweep), every history against the C oracle.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_final_tests}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python tools/stress_parity.py --batches 600 --seed 71 --knobs > $O/knobs.log 2>&1 || { tail -20 $O/knobs.log; exit 1; }
tail -1 $O/knobs.log
timeout -k 10 300 python tools/stress_parity.py --batches 200 --seed 72 --knobs --wide > $O/wide.log 2>&1 || { tail -20 $O/wide.log; exit 1; }
tail -1 $O/wide.log
