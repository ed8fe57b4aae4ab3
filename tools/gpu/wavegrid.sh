#!/bin/bash
# Wave-mode heavy stage (state DAG) by grid size: workgroups resident at once
# vs histories per workgroup (config 2 and 5, no diagnostic timers).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/wavegrid.log
for cfg in "bank_4x16 1000000" "bank_6x24 100000"; do
  for g in 0 256 512 1024 2048; do
    echo "== $cfg wave_grid=$g" >> gpurun_out/wavegrid.log
    timeout -k 10 120 python -u tools/wave_stats.py $cfg wave_grid=$g --nostats 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/wavegrid.log || exit 1
  done
done
cat gpurun_out/wavegrid.log
