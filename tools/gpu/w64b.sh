# config 5 tail: the 48-event histories over the split budget go to the giant split
set -e
O=gpurun_out/w64b; mkdir -p $O
timeout -k 10 300 python tools/sweep_params.py --config bank_6x24 --n 100000 --variants 'split_budget=4096;split_budget=1024;split_budget=256;split_budget=128;split_budget=64;split_budget=256,stage0w=0' > $O/sweep_6x24.json 2> $O/sweep_6x24.err
cat $O/*.json
