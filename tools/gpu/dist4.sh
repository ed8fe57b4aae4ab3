set -e
O=gpurun_out/dist4; mkdir -p $O
run() { env "$@" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1; }
echo "noar $(run QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR=1)" > $O/r.txt
echo "ar $(run QSMD_BENCH_DIST=1)" >> $O/r.txt
echo "ar_inflight1 $(QSMD_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --inflight 1 --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1)" >> $O/r.txt
echo "torchrun_nodist $(run QSMD_X=1)" >> $O/r.txt
python - <<'PY'
import json
for l in open("gpurun_out/dist4/r.txt"):
    k, j = l.split(" ", 1)
    d = json.loads(j)
    print(k, round(d["ms_per_step"], 4), "%.4g" % d["value"])
PY
