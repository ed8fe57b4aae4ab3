#!/bin/bash
# Heavy stage in wave mode, DAG vs DFS, without the diagnostic timers; then
# a kernel trace of the config-4 host call.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in "bank_4x16 1000000" "bank_4x16_bugs 200000 wave_max=10000000" "bank_6x24 100000"; do
  for dag in 128 0; do
    echo "== $cfg dag_states=$dag" >> gpurun_out/dagcmp.log
    timeout -k 10 120 python -u tools/wave_stats.py $cfg dag_states=$dag --nostats 2>&1 | grep -v amdgpu.ids | tail -3 >> gpurun_out/dagcmp.log || exit 1
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run --output-format csv -- python3 tools/config4.py --reps 20 "" > gpurun_out/c4prof.log 2>&1
rc=$?
cat gpurun_out/dagcmp.log
find gpurun_out/c4prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-160
exit $rc
