set -e
O=gpurun_out/dist3; mkdir -p $O
QSMD_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 31 --warmup 4 --no-cpu-baseline > $O/bench_dist.json 2> $O/bench_dist.err || { tail -20 $O/bench_dist.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python - <<'PY'
import json
for f in ("bench_dist", "bench_default"):
    d = json.loads(open(f"gpurun_out/dist3/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "%.4g" % d["value"], d["verdicts"], d.get("mismatches_vs_oracle"), d["config"])
PY
