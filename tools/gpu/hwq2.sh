# RCCL initialised but no collectives (QSMD_BENCH_NOAR=1) vs with, one rank:
# is the cost RCCL's queue or the per-round all-reduce?
set -e
O=gpurun_out/hwq2; mkdir -p $O
P=29700
for s in 2 3; do
  for v in ar noar; do
    E=""; [ $v = noar ] && E="QSMD_BENCH_NOAR=1"
    P=$((P+1))
    timeout -k 10 200 env QSMD_BENCH_DIST=1 $E python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --inflight $s --no-cpu-baseline > $O/s${s}_$v.json 2> $O/s${s}_$v.err || { tail -5 $O/s${s}_$v.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/hwq2/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "%.4g" % d["value"], d["config"]["calls_in_flight"])
PY
