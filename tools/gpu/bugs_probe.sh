set -e
export TMPDIR=/tmp
O=gpurun_out/r3; mkdir -p $O
timeout -k 10 300 python tools/sweep_params.py --config bank_4x16_bugs --rounds 2 --reps 2 --variants 'split_budget=4096;split_budget=0;split_budget=65536;stage0_budget=64;stage0_budget=64,split_budget=0;stage0_budget=256,split_budget=16384;stage0_budget=64,split_budget=16384' > $O/sweep_bugs.json 2> $O/sweep_bugs.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config bank_4x16_bugs --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
cat $O/sweep_bugs.json
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-6 
