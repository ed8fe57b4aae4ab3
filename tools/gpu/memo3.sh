set -e
O=gpurun_out/memo3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "memo or budget or cascade" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 250 python tools/sweep_params.py --config bank_4x16_bugs --rounds 2 --reps 3 --variants 'stage0_budget=64;stage0_budget=64,memo_grid=4096;stage0_budget=64,memo_grid=1024;stage0_budget=48;stage0_budget=80' > $O/sweep_bugs.json 2> $O/sweep_bugs.err
python - <<'PY'
import json
d = json.load(open("gpurun_out/memo3/sweep_bugs.json"))
for k, v in d["variants"].items():
    print(k, round(v["stage0_median_ms"], 4), round(v["call_median_ms"], 4), v["parity_vs_first"])
PY
timeout -k 10 300 python tools/first_call.py > $O/first_call.json 2> $O/first_call.err
cat $O/first_call.json
