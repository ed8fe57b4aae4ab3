#!/bin/bash
# Round 4: stage 0's prefetch distance (knob stage0_prefetch, groups of 64
# ahead; 0 = off): a parity subset on the default, lone stage 0 per
# distance, then the driver's bench command per distance; ROUNDS rounds.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/pf; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "generated_configs or lane_mode or packed or value_ranges or encode or budget or early_exit or device_resident or grids" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for d in ${DISTS:-0 512 1024 2048 4096 8192}; do
    step lone_${d}_$r python tools/stage0_anatomy.py 1000000 26 stage0_prefetch=$d
    python3 -c "import json; d=json.load(open('$O/lone_${d}_$r.out')); x=d['stage0_ms_events'][2:]; print('lone $d', round(sum(x)/len(x),4))"
  done
  for d in ${BDISTS:-0 2048}; do
    step drv_${d}_$r python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --param stage0_prefetch=$d
    python3 -c "import json; d=json.load(open('$O/drv_${d}_$r.out')); print('drv $d', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
