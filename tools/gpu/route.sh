#!/bin/bash
# Host-entry routing: the parity tests that go through it (cascade, wide
# batches, config 4), then the config-4 timing.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 120 \
    --timeout-method thread -k "stage_cascade or mixed or packed or adversarial or ticket_8x64 or memo or kats or wire" \
    > gpurun_out/route_pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 40 "" > gpurun_out/route_c4.log 2>&1
rc=$?
tail -3 gpurun_out/route_pytest.log; grep -v amdgpu.ids gpurun_out/route_c4.log
exit $rc
