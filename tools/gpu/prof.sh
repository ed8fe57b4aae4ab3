#!/bin/bash
# Stage timings for configs 2 and 3, then a rocprofv3 kernel trace of the
# default bench (one call in flight and the default) -> gpurun_out/prof*.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
QSMD_SYNC_STAGES=1 timeout -k 10 120 python -u tools/stage_times.py bank_4x16 1000000 > gpurun_out/st2.log 2>&1 &&
QSMD_SYNC_STAGES=1 timeout -k 10 120 python -u tools/stage_times.py bank_4x16_bugs 1000000 > gpurun_out/st3.log 2>&1 &&
timeout -k 10 180 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --inflight 1 > gpurun_out/b1.json 2> gpurun_out/b1.err &&
timeout -k 10 180 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/prof3 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b3.json 2> gpurun_out/b3.err
rc=$?
grep -v amdgpu.ids gpurun_out/st2.log | tail -12; grep -v amdgpu.ids gpurun_out/st3.log | tail -12
find gpurun_out/prof1 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
exit $rc
