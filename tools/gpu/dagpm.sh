#!/bin/bash
# State-DAG change check: the wave-mode parity tests, a wide stress sweep,
# config 4 (timing and phase cycles), config-2 DAG cycles, one call at a time.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 120 \
    --timeout-method thread -k "wave_mode or heavy_any_shape or generated_configs or memo or stage_cascade or adversarial or dag or lane_mode" \
    > gpurun_out/pm_pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/stress_parity.py --batches 20 --seed 53 --knobs --wide > gpurun_out/pm_stress.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 40 "" > gpurun_out/pm_c4.log 2>&1 &&
timeout -k 10 120 python -u tools/config4_phases.py > gpurun_out/pm_c4ph.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 > gpurun_out/pm_ws2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --inflight 1 --steps 200 --warmup 10 > gpurun_out/pm_if1.log 2>&1
rc=$?
tail -2 gpurun_out/pm_pytest.log; tail -1 gpurun_out/pm_stress.log
for f in pm_c4 pm_c4ph pm_ws2; do echo "== $f"; grep -v amdgpu.ids gpurun_out/$f.log | tail -3; done
tail -1 gpurun_out/pm_if1.log | cut -c1-300
exit $rc
