#!/bin/bash
# Round-end evidence: the -m gpu suite, smoke, the measurements
# (tools/gpu/measure.sh: driver command, 200-step default with CPU baselines
# and extra configs, one call at a time, the rocprofv3 passes), then a
# randomised parity sweep.  Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/final_suite.log 2>&1 || { tail -20 gpurun_out/final_suite.log; exit 1; }
tail -2 gpurun_out/final_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { cat gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash tools/gpu/measure.sh > gpurun_out/final_measure.log 2>&1 || { tail -30 gpurun_out/final_measure.log; exit 1; }
head -3 gpurun_out/final_measure.log
timeout -k 10 400 python -u tools/stress_parity.py --batches 60 --seed 31 --knobs > gpurun_out/final_stress.log 2>&1
rc=$?
tail -3 gpurun_out/final_stress.log
exit $rc
