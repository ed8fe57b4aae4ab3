set -e
O=gpurun_out/memo_prof2; mkdir -p $O
: > $O/stats.json
for e in 16 32 64 128; do
  timeout -k 10 120 python tools/memo_stats.py --set memo_lane_entries=$e >> $O/stats.json 2>> $O/stats.err
done
timeout -k 10 120 python tools/memo_stats.py --set memo_lane_entries=64,memo_grid=4096 >> $O/stats.json 2>> $O/stats.err
timeout -k 10 120 python tools/memo_stats.py --set memo_lane_entries=32,memo_grid=4096 >> $O/stats.json 2>> $O/stats.err
cat $O/stats.json
