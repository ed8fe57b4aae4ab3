# memo stage tuning: grid x stage-0 budget on config 3, stage-0w budget on config 5, kernel trace of config 3
set -e
O=gpurun_out/memo_tune; mkdir -p $O
timeout -k 10 250 python tools/sweep_params.py --config bank_4x16_bugs --rounds 2 --reps 3 --variants 'stage0_budget=128;stage0_budget=128,memo_grid=1024;stage0_budget=128,memo_grid=2048;stage0_budget=128,memo_grid=4096;stage0_budget=64,memo_grid=2048;stage0_budget=32,memo_grid=2048;stage0_budget=64,memo_grid=2048,memo_lane_entries=64;stage0_budget=64,memo_grid=2048,memo_lane_entries=256' > $O/sweep_bugs.json 2> $O/sweep_bugs.err
timeout -k 10 200 python tools/sweep_params.py --config bank_6x24 --n 100000 --variants 'stage0w_budget=32;stage0w_budget=32,memo_grid=1024;stage0w_budget=32,memo_grid=2048;stage0w_budget=16,memo_grid=2048;stage0w_budget=48,memo_grid=2048' > $O/sweep_6x24.json 2> $O/sweep_6x24.err
python - <<'PY'
import json
for f in ("sweep_bugs", "sweep_6x24"):
    d = json.load(open(f"gpurun_out/memo_tune/{f}.json"))
    for k, v in d["variants"].items():
        print(f, k, round(v["stage0_median_ms"], 4), round(v["call_median_ms"], 4), v["parity_vs_first"])
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --config bank_4x16_bugs --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -12
