set -e
V='split_budget=4096;split_budget=2048;split_budget=1024;split_budget=512'
timeout -k 10 250 python tools/sweep_params.py --config ticket_8x64 --n 100000 --rounds 3 --reps 3 --variants "$V" > gpurun_out/s3_t864.json 2>/dev/null
for c in bank_4x16 bank_4x16_bugs ticket_2x10; do
timeout -k 10 250 python tools/sweep_params.py --config $c --rounds 3 --reps 5 --variants "$V" > gpurun_out/s3_$c.json 2>/dev/null
done
timeout -k 10 250 python tools/sweep_params.py --config bank_6x24 --n 100000 --rounds 3 --reps 5 --variants "$V" > gpurun_out/s3_bank_6x24.json 2>/dev/null
python - <<'PY'
import json
for f in ("t864", "bank_4x16", "bank_4x16_bugs", "ticket_2x10", "bank_6x24"):
    d = json.load(open(f"gpurun_out/s3_{f}.json"))
    print(f, {k: (round(v["call_median_ms"], 3), round(v["call_min_ms"], 3), v["parity_vs_first"]) for k, v in d["variants"].items()})
PY
