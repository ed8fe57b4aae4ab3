# kernel trace of the 48-event config (which kernel holds the call)
set -e
O=gpurun_out/prof6x24; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python bench.py --config bank_6x24 --n-hist 100000 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
find $O -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -30
