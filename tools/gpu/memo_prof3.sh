set -e
O=gpurun_out/memo_prof3; mkdir -p $O
: > $O/stats.json
for m in 0 4 6 8 10 12 16; do
  timeout -k 10 120 python tools/memo_stats.py --set memo_min_rem=$m >> $O/stats.json 2>> $O/stats.err
done
timeout -k 10 120 python tools/memo_stats.py --config bank_6x24 --n 100000 --set memo_min_rem=0 >> $O/stats.json 2>> $O/stats.err
timeout -k 10 120 python tools/memo_stats.py --config bank_6x24 --n 100000 --set memo_min_rem=8 >> $O/stats.json 2>> $O/stats.err
timeout -k 10 120 python tools/memo_stats.py --config bank_6x24 --n 100000 --set memo_min_rem=12 >> $O/stats.json 2>> $O/stats.err
cat $O/stats.json
