#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/measure
mkdir -p $O
timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/bench_inflight1.json 2> $O/bench_inflight1.err &&
timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 > $O/bench_early.json 2> $O/bench_early.err
rc=$?
python3 -c "
import json; d=json.load(open('$O/bench_inflight1.json')); print('inflight1 %.3e' % d['value'], d['device_ms'])"
python3 -c "import json; d=json.load(open('$O/bench_early.json')); print('early', json.dumps(d['early_exit']))"
exit $rc
