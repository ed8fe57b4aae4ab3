#!/bin/bash
# Round 4: lane mode goes on from stage 0's saved state -- parity, then the
# driver's command against the stage-0 budget.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/rs; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread \
    -k "lane_mode or memo_after or generated_configs or sharded or bench_knobs or budget or early or witness or kats or model_error or handoff" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for b in ${DBUDGETS:-14 16 17 18 20}; do
  step drv_${b}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b
  python3 -c "import json; d=json.load(open('$O/drv_${b}_$r.out')); print('drv budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
timeout -k 10 300 python tools/memo_stats.py bank_4x16 1000000 stage0_budget=16 heavy_mode=1 memo_lds=0 > $O/ms16.json 2> $O/ms16.err && cat $O/ms16.json
