set -e
O=gpurun_out/sp; mkdir -p $O
timeout -k 10 250 python tools/sweep_params.py --config bank_4x16 --rounds 3 --reps 5 --variants "stage0_budget=0;stage0_budget=64;stage0_budget=48,spread_budget=32;stage0_budget=64,spread_budget=64;stage0_budget=32,spread_budget=32;stage0_budget=64,spread_grid=512" > $O/s2.json 2> $O/s2.err
python -c "import json;d=json.load(open('$O/s2.json'));[print('cfg2',k,round(v['stage0_median_ms'],3),round(v['call_median_ms'],3),v['parity_vs_first']) for k,v in d['variants'].items()]"
timeout -k 10 250 python tools/sweep_params.py --config bank_4x16_bugs --rounds 1 --reps 2 --variants "stage0_budget=64,split_budget=16384;stage0_budget=64;stage0_budget=64,spread_budget=512;stage0_budget=64,spread_budget=32;stage0_budget=32,spread_budget=128,spread_grid=4096" > $O/s3.json 2> $O/s3.err
python -c "import json;d=json.load(open('$O/s3.json'));[print('cfg3',k,round(v['stage0_median_ms'],3),round(v['call_median_ms'],3),v['parity_vs_first']) for k,v in d['variants'].items()]"
