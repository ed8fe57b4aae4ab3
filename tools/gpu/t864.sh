set -e
O=gpurun_out/t864; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --config ticket_8x64 --n-hist 100000 --inflight 1 --steps 2 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -12
