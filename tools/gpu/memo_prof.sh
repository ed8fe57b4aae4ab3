set -e
O=gpurun_out/memo_prof; mkdir -p $O
timeout -k 10 120 python tools/memo_stats.py > $O/stats.json 2> $O/stats.err
timeout -k 10 120 python tools/memo_stats.py --set memo_lane_entries=1024 >> $O/stats.json 2>> $O/stats.err
timeout -k 10 120 python tools/memo_stats.py --set memo_grid=3072 >> $O/stats.json 2>> $O/stats.err
cat $O/stats.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/memo_stats.py > $O/trace.log 2>&1
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -8
