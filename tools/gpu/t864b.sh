set -e
O=gpurun_out/t864b; mkdir -p $O
timeout -k 10 300 python bench.py --config ticket_8x64 --n-hist 100000 --inflight 1 --steps 5 --warmup 2 --cpu-seconds 3 > $O/b1.json 2> $O/b1.err
timeout -k 10 300 python bench.py --config ticket_8x64 --n-hist 100000 --steps 5 --warmup 2 --no-cpu-baseline > $O/b3.json 2> $O/b3.err
python - <<'PY'
import json
for f in ("b1", "b3"):
    d = json.loads(open(f"gpurun_out/t864b/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 3), "%.4g" % d["value"], d["verdicts"], d.get("mismatches_vs_oracle"), (d.get("cpu_baseline") or {}).get("value"))
PY
