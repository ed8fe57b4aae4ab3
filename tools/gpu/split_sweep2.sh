set -e
timeout -k 10 250 python tools/sweep_params.py --config ticket_8x64 --n 100000 --rounds 2 --reps 3 --variants 'split_budget=4096;split_budget=1024;split_budget=256;split_budget=64' > gpurun_out/ss_t.json 2>/dev/null
timeout -k 10 250 python tools/sweep_params.py --config bank_4x16 --rounds 2 --reps 4 --variants 'split_budget=4096;split_budget=1024;split_budget=256' > gpurun_out/ss_b.json 2>/dev/null
timeout -k 10 250 python tools/sweep_params.py --config bank_4x16_bugs --rounds 2 --reps 3 --variants 'split_budget=4096;split_budget=1024;split_budget=256' > gpurun_out/ss_bb.json 2>/dev/null
python - <<'PY'
import json
for f in ("ss_t", "ss_b", "ss_bb"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, {k: (round(v["call_median_ms"], 3), v["parity_vs_first"]) for k, v in d["variants"].items()})
PY
