#!/bin/bash
# State-DAG phase timings (wave_stats) and the config-4 host/device times.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 > gpurun_out/dag_ws2.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16_bugs 200000 wave_max=10000000 > gpurun_out/dag_ws3.log 2>&1 &&
timeout -k 10 120 python -u tools/config4.py --reps 20 "" > gpurun_out/dag_c4.log 2>&1
rc=$?
for f in dag_ws2 dag_ws3 dag_c4; do echo "== $f"; grep -v amdgpu.ids gpurun_out/$f.log | tail -2; done
exit $rc
