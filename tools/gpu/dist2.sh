set -e
O=gpurun_out/dist2; mkdir -p $O
for ar in side inline; do
QSMD_BENCH_AR=$ar QSMD_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/bench_$ar.json 2> $O/bench_$ar.err || { tail -20 $O/bench_$ar.err; exit 1; }
done
python - <<'PY'
import json
for f in ("bench_side", "bench_inline"):
    d = json.loads(open(f"gpurun_out/dist2/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "%.4g" % d["value"], d["device_ms"])
PY
