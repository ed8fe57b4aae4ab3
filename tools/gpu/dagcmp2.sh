#!/bin/bash
# wave-mode parity tests, then DAG vs DFS timings and the config-4 host call
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 120 \
    --timeout-method thread -k "wave_mode or heavy_any_shape or generated_configs or memo or stage_cascade or adversarial or dag" \
    > gpurun_out/dag_pytest.log 2>&1 &&
rm -f gpurun_out/dagcmp.log && bash tools/gpu/dagcmp.sh > gpurun_out/dagcmp_out.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 40 "" > gpurun_out/c4.log 2>&1
rc=$?
tail -2 gpurun_out/dag_pytest.log; cat gpurun_out/dagcmp.log 2>/dev/null | grep -v "call 5\|call 6"; grep -v amdgpu.ids gpurun_out/c4.log
exit $rc
