# the bench's all-reduce path on one rank (torchrun, nccl = RCCL), then plain
set -e
O=gpurun_out/dist1; mkdir -p $O
QSMD_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_dist.json 2> $O/bench_dist.err || { tail -20 $O/bench_dist.err; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python - <<'PY'
import json
for f in ("bench_dist", "bench"):
    d = json.loads(open(f"gpurun_out/dist1/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "%.4g" % d["value"], d["verdicts"])
PY
