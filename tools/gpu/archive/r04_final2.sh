#!/bin/bash
# Round 4 evidence, part 2: the randomised parity sweep, one rank with and
# without the RCCL path at the driver's 20 steps, the 2-rank gloo rehearsal.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/rccl
timeout -k 10 400 python -u tools/stress_parity.py --batches 60 --seed 41 --knobs > gpurun_out/final_stress.log 2>&1 ||
    { tail -20 gpurun_out/final_stress.log; exit 1; }
tail -3 gpurun_out/final_stress.log
STEPS=20 bash tools/gpu/archive/rccl_sweep.sh 3 "none||" "dist|QSMD_BENCH_DIST=1|" "dist_noar|QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR=1|" \
    > gpurun_out/rccl/sweep20.log 2>&1 || { cat gpurun_out/rccl/sweep20.log; exit 1; }
cat gpurun_out/rccl/sweep20.log
bash tools/gpu/dist_rehearsal.sh
