# stage 0w + coop64: parity subset, then A/B on the 48-event config
set -e
O=gpurun_out/w64; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "stage_cascade or packed_uniform or mixed_sizes or budget or 6x24 or kats or encode" > $O/pytest.log 2>&1
timeout -k 10 200 python tools/sweep_params.py --config bank_6x24 --n 100000 --variants 'stage0w_budget=256;stage0w=0;stage0w_budget=0;stage0w_budget=64;stage0w_budget=128;stage0w_budget=512;stage0w_budget=256,coop64_grid=128;stage0w_budget=128,coop_budget=8;stage0w_budget=128,coop_budget=32' > $O/sweep_6x24.json 2> $O/sweep_6x24.err
timeout -k 10 200 python tools/sweep_params.py --config bank_4x16 --n 1000000 --variants 'stage0w=1;stage0w=0' > $O/sweep_4x16.json 2> $O/sweep_4x16.err
tail -3 $O/pytest.log; cat $O/*.json
