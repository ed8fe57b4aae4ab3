#!/bin/bash
# The randomised parity sweep on the round-5 tree (random knobs per batch,
# incl. fold and resume_cap), then the wide any-shape sweep.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_stress
mkdir -p $O
timeout -k 10 500 python tools/stress_parity.py --batches 600 --seed 51 --knobs > $O/knobs.log 2>&1 || { tail -20 $O/knobs.log; exit 1; }
tail -1 $O/knobs.log
timeout -k 10 400 python tools/stress_parity.py --batches 300 --seed 52 --knobs --wide > $O/wide.log 2>&1 || { tail -20 $O/wide.log; exit 1; }
tail -1 $O/wide.log
