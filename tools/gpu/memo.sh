# memo stage: parity, then timing on configs 3, 5, 2
set -e
O=gpurun_out/memo; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "memo" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/sweep_params.py --config bank_4x16_bugs --rounds 2 --reps 3 --variants 'stage0_auto=1;stage0_auto=1,memo_stage=1;stage0_budget=64,memo_stage=1;stage0_budget=128,memo_stage=1;stage0_budget=32,memo_stage=1' > $O/sweep_bugs.json 2> $O/sweep_bugs.err
timeout -k 10 200 python tools/sweep_params.py --config bank_6x24 --n 100000 --variants 'stage0w_budget=0;stage0w_budget=256,memo_stage=1;stage0w_budget=64,memo_stage=1;stage0w_budget=32,memo_stage=1' > $O/sweep_6x24.json 2> $O/sweep_6x24.err
python - <<'PY'
import json
for f in ("sweep_bugs", "sweep_6x24"):
    d = json.load(open(f"gpurun_out/memo/{f}.json"))
    print(f, {k: (round(v["call_median_ms"], 4), v["parity_vs_first"]) for k, v in d["variants"].items()})
PY
