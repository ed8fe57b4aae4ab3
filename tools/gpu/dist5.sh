set -e
O=gpurun_out/dist5; mkdir -p $O
: > $O/r.txt
for q in 4 8; do
for inf in 2 3; do
  echo "q${q}_inf${inf}_ar $(GPU_MAX_HW_QUEUES=$q QSMD_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --inflight $inf --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1)" >> $O/r.txt
  echo "q${q}_inf${inf}_plain $(GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --inflight $inf --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1)" >> $O/r.txt
done
done
python - <<'PY'
import json
for l in open("gpurun_out/dist5/r.txt"):
    k, j = l.split(" ", 1)
    d = json.loads(j)
    print(k, round(d["ms_per_step"], 4), "%.4g" % d["value"])
PY
