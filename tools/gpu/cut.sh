set -e
O=gpurun_out/cut; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "straggler or memo" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
V='stage0_auto=1;stage0_auto=1,cut_k=1;stage0_auto=1,cut_k=2;stage0_auto=1,cut_k=4;stage0_auto=1,cut_k=2,cut_min=20;stage0_auto=1,cut_k=4,cut_min=24;stage0_auto=1,cut_k=8,cut_min=24'
for c in bank_4x16 bank_4x16_bugs ticket_2x10; do
  timeout -k 10 250 python tools/sweep_params.py --config $c --rounds 3 --reps 4 --variants "$V" > $O/$c.json 2> $O/$c.err
done
timeout -k 10 250 python tools/sweep_params.py --config bank_6x24 --n 100000 --rounds 3 --reps 4 --variants "$V" > $O/bank_6x24.json 2> $O/bank_6x24.err
python - <<'PY'
import json
for f in ("bank_4x16", "bank_4x16_bugs", "ticket_2x10", "bank_6x24"):
    d = json.load(open(f"gpurun_out/cut/{f}.json"))
    print(f, {k.replace("stage0_auto=1", "").strip(",") or "base": (round(v["call_median_ms"], 4), v["parity_vs_first"]) for k, v in d["variants"].items()})
PY
