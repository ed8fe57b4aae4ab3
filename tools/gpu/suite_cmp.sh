#!/bin/bash
# The whole -m gpu suite, then DAG vs DFS timings (tools/gpu/dagcmp.sh) and
# the config-4 host call.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/suite.log 2>&1 &&
rm -f gpurun_out/dagcmp.log && bash tools/gpu/dagcmp.sh > gpurun_out/dagcmp_out.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 40 "" > gpurun_out/c4.log 2>&1
rc=$?
tail -3 gpurun_out/suite.log; cat gpurun_out/dagcmp.log 2>/dev/null; grep -v amdgpu.ids gpurun_out/c4.log
exit $rc
