set -e
O=gpurun_out/inflight; mkdir -p $O
for c in bank_4x16 bank_4x16_bugs ticket_2x10; do
for s in 1 2 3; do
  timeout -k 10 200 python bench.py --config $c --inflight $s --steps 30 --warmup 4 --no-cpu-baseline > $O/${c}_$s.json 2> $O/${c}_$s.err || { tail -5 $O/${c}_$s.err; exit 1; }
done
done
timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --inflight 1 --steps 30 --warmup 4 --no-cpu-baseline > $O/bank_6x24_1.json 2> $O/bank_6x24_1.err
timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --inflight 2 --steps 30 --warmup 4 --no-cpu-baseline > $O/bank_6x24_2.json 2> $O/bank_6x24_2.err
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/inflight/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), "%.4g" % d["value"], d["verdicts"]["checked"], d["device_ms"])
PY
