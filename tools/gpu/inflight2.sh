set -e
O=gpurun_out/inflight2; mkdir -p $O
for s in 3 4 6; do
  timeout -k 10 200 python bench.py --inflight $s --steps 40 --warmup 6 --no-cpu-baseline > $O/b_$s.json 2> $O/b_$s.err || { tail -5 $O/b_$s.err; exit 1; }
done
timeout -k 10 200 python bench.py --config bank_4x16_bugs --inflight 4 --steps 20 --warmup 4 --no-cpu-baseline > $O/bugs_4.json 2> $O/bugs_4.err
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/inflight2/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), "%.4g" % d["value"], d["device_ms"], d["roofline"]["frac"])
PY
