#!/bin/bash
# One-rank cost of the RCCL path (verdict r02 item 7): with and without the
# process group, with 8 hardware queues, with 2 calls in flight, without the
# all-reduce; then a kernel + HIP trace of one rank each way.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu/archive/rccl_sweep.sh 3 "none||" "dist|QSMD_BENCH_DIST=1|" "dist_q8|QSMD_BENCH_DIST=1|--hw-queues 8" \
    "dist_i2|QSMD_BENCH_DIST=1|--inflight 2" "dist_noar|QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR=1|" "none_i2||--inflight 2" \
    > gpurun_out/rccl/sweep.log 2>&1 || { cat gpurun_out/rccl/sweep.log; exit 1; }
cat gpurun_out/rccl/sweep.log
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/rccl/tr_none -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/rccl/tr_none.json 2> gpurun_out/rccl/tr_none.err &&
QSMD_BENCH_DIST=1 timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/rccl/tr_dist -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/rccl/tr_dist.json 2> gpurun_out/rccl/tr_dist.err
