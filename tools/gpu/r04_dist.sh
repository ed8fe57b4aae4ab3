#!/bin/bash
# Round 4: one rank's RCCL path at the driver's 20-step command after the
# closing barrier left the timed window (none / RCCL / RCCL without the
# all-reduce, 3 rounds each), the 2-rank gloo rehearsal on one GPU, and the
# full-size bench-knob parity test.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/rccl
STEPS=20 bash tools/gpu/rccl_sweep.sh 3 "none||" "dist|QSMD_BENCH_DIST=1|" "dist_noar|QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR=1|" \
    > gpurun_out/rccl/sweep20.log 2>&1 || { cat gpurun_out/rccl/sweep20.log; exit 1; }
cat gpurun_out/rccl/sweep20.log
bash tools/gpu/dist_rehearsal.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "bench_knobs" > gpurun_out/bk.log 2>&1; rc=$?; tail -3 gpurun_out/bk.log; exit $rc
