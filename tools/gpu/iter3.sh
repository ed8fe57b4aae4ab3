#!/bin/bash
# Wave-mode heavy stage: stats on config 2 and 3 (diagnostic), the heavy-stage
# parity tests, the config-4 single history.
set -o pipefail
mkdir -p gpurun_out/iter3
export PYTHONUNBUFFERED=1
O=gpurun_out/iter3
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 > $O/wave_stats.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 wave_min_rem=64 > $O/wave_stats_nomemo.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "wave or heavy or cascade or adversarial or memo or kats or budget or early or full_size" \
    > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py "" "heavy_mode=1" "wave_min_rem=0" > $O/config4.log 2>&1
rc=$?
cat $O/wave_stats.log $O/wave_stats_nomemo.log | grep -v amdgpu.ids | grep -v "call 0"
tail -3 $O/pytest.log; tail -5 $O/config4.log
exit $rc
