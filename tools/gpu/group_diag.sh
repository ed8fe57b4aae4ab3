O=gpurun_out/ad1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; tail -4 $O/tests.log
timeout -k 10 200 python tools/spread_diag.py --config bank_4x16 --reps 5 --variants "stage0_auto=1;stage0_budget=0" 2>$O/c2.err | tee $O/c2.jsonl || exit 1
timeout -k 10 200 python tools/spread_diag.py --config bank_4x16_bugs --n 1000000 --reps 3 --variants "stage0_auto=1;stage0_budget=256,heavy_stage=1" 2>$O/c3.err | tee $O/c3.jsonl
