# hardware queues per process (GPU_MAX_HW_QUEUES, 4 by default) vs calls in
# flight, without and with the RCCL counter all-reduce (one rank)
set -e
O=gpurun_out/hwq; mkdir -p $O
run() {  # name, env..., -- bench args
  n=$1; shift
  timeout -k 10 200 env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
}
P=29600
for q in 4 8; do
  for s in 2 3 4; do
    run q${q}_s${s} GPU_MAX_HW_QUEUES=$q python bench.py --inflight $s --no-cpu-baseline
    P=$((P+1))
    run q${q}_s${s}_rccl GPU_MAX_HW_QUEUES=$q QSMD_BENCH_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --inflight $s --no-cpu-baseline
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/hwq/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "%.4g" % d["value"], d["config"]["calls_in_flight"])
PY
