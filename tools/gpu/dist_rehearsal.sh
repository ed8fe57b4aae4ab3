#!/bin/bash
# The bench's N > 1 path on one GPU (diagnostic): one rank over RCCL, then
# two ranks on the same device over gloo (RCCL refuses two ranks per GPU).
set -o pipefail
mkdir -p gpurun_out/dist
QSMD_BENCH_DIST=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra \
    > gpurun_out/dist/rccl1.json 2> gpurun_out/dist/rccl1.err || { tail -5 gpurun_out/dist/rccl1.err; exit 1; }
QSMD_BENCH_DEVICE=0 QSMD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
    > gpurun_out/dist/gloo2.json 2> gpurun_out/dist/gloo2.err || { tail -5 gpurun_out/dist/gloo2.err; exit 1; }
for f in gpurun_out/dist/rccl1.json gpurun_out/dist/gloo2.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['n_gpus'], '%.4g' % d['value'], d['verdicts'], d['config']['allreduce_every_steps'])" "$f"
done
