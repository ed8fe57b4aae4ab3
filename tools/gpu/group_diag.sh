O=gpurun_out/gd4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; tail -4 $O/tests.log
timeout -k 10 200 python tools/spread_diag.py --config bank_4x16 --variants "stage0_kernel=0;stage0_kernel=1;stage0_kernel=1,share_nodes=48;stage0_kernel=1,share_idle=32;stage0_kernel=0" 2>$O/c2.err | tee $O/c2.jsonl || exit 1
timeout -k 10 200 python tools/spread_diag.py --config bank_4x16_bugs --n 1000000 --reps 2 --variants "stage0_kernel=1;stage0_kernel=1,group_budget=64;stage0_kernel=1,share_nodes=64" 2>$O/c3.err | tee $O/c3.jsonl
