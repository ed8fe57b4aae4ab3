#!/bin/bash
# The randomised parity sweep on the round-5 tree (random knobs per batch,
# incl. fold, resume_cap and the early-exit flag), then the wide any-shape sweep.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_stress2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stress.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python tools/stress_parity.py --batches 600 --seed 61 --knobs > $O/knobs.log 2>&1 || { tail -20 $O/knobs.log; exit 1; }
tail -1 $O/knobs.log
timeout -k 10 400 python tools/stress_parity.py --batches 300 --seed 62 --knobs --wide > $O/wide.log 2>&1 || { tail -20 $O/wide.log; exit 1; }
tail -1 $O/wide.log
