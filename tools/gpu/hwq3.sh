# one GPU, no RCCL: 4 hardware queues x 3 in flight (default) vs 8 queues x 4-6
set -e
O=gpurun_out/hwq3; mkdir -p $O
for rep in 1 2; do
  for v in q4_s3 q8_s4 q8_s5 q8_s6 q6_s4; do
    q=${v%_*}; q=${q#q}; s=${v#*_s}
    timeout -k 10 200 env GPU_MAX_HW_QUEUES=$q python bench.py --inflight $s --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/hwq3/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "%.4g" % d["value"], d["device_ms"])
PY
