# stage 0r: parity, then the re-run budget on config 2 and config 5
set -e
O=gpurun_out/rerun; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/sweep_params.py --config bank_4x16 --variants 'rerun_budget=0;rerun_budget=16;rerun_budget=17;rerun_budget=18;rerun_budget=20;rerun_budget=24;rerun_budget=32' > $O/sweep_4x16.json 2> $O/sweep_4x16.err
timeout -k 10 200 python tools/sweep_params.py --config ticket_2x10 --variants 'rerun_budget=0;rerun_budget=8;rerun_budget=12;rerun_budget=16' > $O/sweep_t.json 2> $O/sweep_t.err
python - <<'PY'
import json
for f in ("sweep_4x16", "sweep_t"):
    d = json.load(open(f"gpurun_out/rerun/{f}.json"))
    print(f, {k: (round(v["call_median_ms"], 4), v["parity_vs_first"]) for k, v in d["variants"].items()})
PY
