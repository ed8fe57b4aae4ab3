set -e
O=gpurun_out/r2; mkdir -p $O
timeout -k 10 200 python tools/sweep_params.py --config bank_4x16 --variants 'stage0_persistent_grid=0;stage0_persistent_grid=1024;stage0_persistent_grid=2048;stage0_persistent_grid=4096;stage0_persistent_grid=2048,refill_min=16;stage0_persistent_grid=2048,refill_min=4' > $O/sweep_persist.json 2> $O/sweep_persist.err
timeout -k 10 200 python bench.py --config bank_4x16_bugs --steps 5 --warmup 1 --cpu-seconds 5 > $O/bench_bugs.json 2> $O/bench_bugs.err
timeout -k 10 200 python bench.py --config bank_6x24 --n-hist 100000 --steps 5 --warmup 1 --cpu-seconds 5 > $O/bench_6x24.json 2> $O/bench_6x24.err
timeout -k 10 200 python bench.py --config ticket_2x10 --steps 5 --warmup 1 --cpu-seconds 5 > $O/bench_t2x10.json 2> $O/bench_t2x10.err
timeout -k 10 200 python tools/bench_single.py > $O/single.json 2> $O/single.err
cat $O/*.json
