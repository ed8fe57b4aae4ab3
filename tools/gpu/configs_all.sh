# full GPU suite, then every BASELINE config through bench.py (one line each)
set -e
O=${1:-gpurun_out/all}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for c in bank_4x16 ticket_2x10 bank_4x16_bugs; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 3 > $O/bench_$c.json 2> $O/bench_$c.err
done
timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 10 --warmup 3 --cpu-seconds 3 > $O/bench_bank_6x24.json 2> $O/bench_bank_6x24.err
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/all/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), "ms", "%.3g" % d["value"], d["unit"], "nodes/s %.3g" % d.get("nodes_per_sec", 0),
          "cpu", (d.get("cpu_baseline") or {}).get("value"), "mism", d.get("mismatches_vs_oracle"))
PY
