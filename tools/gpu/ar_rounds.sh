# RCCL counter all-reduce every R rounds of in-flight steps (one rank, RCCL
# path forced), alternated, plus the plain one-GPU default
set -e
O=gpurun_out/ar_rounds; mkdir -p $O
P=29800
for rep in 1 2; do
  for r in 1 4 16; do
    P=$((P+1))
    timeout -k 10 200 env QSMD_BENCH_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $P bench.py --ar-rounds $r --no-cpu-baseline > $O/r${r}_$rep.json 2> $O/r${r}_$rep.err || { tail -5 $O/r${r}_$rep.err; exit 1; }
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/plain.json 2> $O/plain.err
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ar_rounds/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "%.4g" % d["value"], d["config"]["calls_in_flight"], d["config"]["allreduce_every_steps"], d["verdicts"]["checked"])
PY
