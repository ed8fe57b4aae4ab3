#!/bin/bash
# Round 4: stage 0b (stage 0's heavy list searched again by the compact DFS
# at budget B) -- a parity subset, then the driver's command and one call at
# a time against B (0 = off).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/s0b2; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "generated_configs or lane_mode or wave_mode or budget or early_exit or sharded or knobs or kats or witness" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in 1 2; do
for sb in ${SBS:-0 64 128 256 1024}; do
  for b in ${DBUDGETS:-16 20}; do
    step drv_${sb}_${b}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --stage0-budget $b --param stage0b_budget=$sb
    python3 -c "import json; d=json.load(open('$O/drv_${sb}_${b}_$r.out')); print('drv s0b $sb budget $b', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4), d['mismatches_vs_oracle'])"
  done
  step i1_${sb}_$r python bench.py --inflight 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --param stage0b_budget=$sb
  python3 -c "import json; d=json.load(open('$O/i1_${sb}_$r.out')); print('i1 s0b $sb', round(d['value']/1e9,3), 'call', round(d['device_ms']['alone']['call_mean'],4))"
done
done
