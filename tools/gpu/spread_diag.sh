O=gpurun_out/sd7; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
timeout -k 10 200 python tools/spread_diag.py --config bank_4x16 --variants "stage0_budget=0;stage0_budget=1024;stage0_budget=1024,coop_grid=512;stage0_budget=0" 2>$O/c2.err | tee $O/c2.jsonl || exit 1
timeout -k 10 200 python tools/spread_diag.py --config bank_4x16_bugs --n 1000000 --reps 2 --variants "stage0_budget=1024,spread_budget=1024;stage0_budget=256,spread_budget=1024,spread_grid=1024;stage0_budget=512,spread_budget=1024,spread_grid=1024" 2>$O/c3.err | tee $O/c3.jsonl
