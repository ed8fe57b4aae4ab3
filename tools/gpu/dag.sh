#!/bin/bash
# State-DAG heavy stage: the wave-mode parity tests, then its statistics on
# configs 2 and 3 and the config-4 timing.  Every GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -v --timeout 120 \
    --timeout-method thread -k "wave_mode or heavy_any_shape or generated_configs or memo or stage_cascade or mixed" \
    > gpurun_out/dag_pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 > gpurun_out/dag_ws2.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 dag_states=0 > gpurun_out/dag_ws2_off.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16_bugs 1000000 wave_max=10000000 > gpurun_out/dag_ws3.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 20 "" "dag_states=0" > gpurun_out/dag_c4.log 2>&1
rc=$?
tail -5 gpurun_out/dag_pytest.log
for f in dag_ws2 dag_ws2_off dag_ws3 dag_c4; do echo "== $f"; grep -v amdgpu.ids gpurun_out/$f.log | tail -5; done
exit $rc
