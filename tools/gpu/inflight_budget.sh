# fixed stage-0 budgets vs the adaptive cascade under the bench's default
# 3 calls in flight (the per-call sweep, budget_sweep.sh, measures one call
# at a time, where the memo stage's latency is not hidden by the next batch)
set -e
O=gpurun_out/inflight_budget; mkdir -p $O
for c in bank_4x16 ticket_2x10; do
  for b in auto 24 32 48 64 128; do
    if [ $b = auto ]; then A=""; else A="--stage0-budget $b"; fi
    timeout -k 10 200 python bench.py --config $c $A --steps 60 --warmup 6 --no-cpu-baseline > $O/${c}_$b.json 2> $O/${c}_$b.err || { tail -5 $O/${c}_$b.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/inflight_budget/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 4), "%.4g" % d["value"], d["device_ms"], d["verdicts"])
PY
