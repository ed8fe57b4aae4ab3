# fixed stage-0 budget (memo stage for the rest) vs the adaptive cascade, every config
set -e
O=gpurun_out/budget; mkdir -p $O
V='stage0_auto=1;stage0_budget=48;stage0_budget=64;stage0_budget=96;stage0_budget=128'
for c in bank_4x16 ticket_2x10 bank_4x16_bugs; do
  timeout -k 10 250 python tools/sweep_params.py --config $c --rounds 3 --reps 4 --variants "$V" > $O/$c.json 2> $O/$c.err
done
python - <<'PY'
import json
for f in ("bank_4x16", "ticket_2x10", "bank_4x16_bugs"):
    d = json.load(open(f"gpurun_out/budget/{f}.json"))
    print(f, {k: (round(v["call_median_ms"], 4), round(v["call_min_ms"], 4), v["parity_vs_first"]) for k, v in d["variants"].items()})
PY
