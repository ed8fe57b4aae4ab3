#!/bin/bash
# The whole -m gpu suite, then the config-4 host call (and its CPU point).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/suite.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 40 "" > gpurun_out/c4.log 2>&1 &&
timeout -k 10 120 python -u tools/overhead.py > gpurun_out/overhead.log 2>&1
rc=$?
tail -3 gpurun_out/suite.log; grep -v amdgpu.ids gpurun_out/c4.log; grep -v amdgpu.ids gpurun_out/overhead.log | tail -12
exit $rc
