#!/bin/bash
# Round 6: config 5 (Bank 6x24, 100k histories: every history 48 events, so
# stage 0w) -- the kernel trace of the bench's config-5 shape (3 calls in
# flight, the library's defaults), and the heavy stage's anatomy.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_c5}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --config bank_6x24 --n-hist 100000 --steps 20 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --stage0-budget -1 \
  > $O/bench.json 2> $O/bench.err &&
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; &&
cat $O/kernel_stats.csv | cut -d, -f1-8 | head -20 &&
timeout -k 10 120 python tools/memo_stats.py bank_6x24 100000 > $O/memo_stats.json 2> $O/memo_stats.err; cat $O/memo_stats.json; tail -3 $O/memo_stats.err
