#!/bin/bash
# Round 4 A/B over named builds: a parity subset on the product build, then
# lone stage 0 (and the driver's bench command unless LONE_ONLY=1) for each
# build named on the command line (prod = lib/libqsmd.so, NAME =
# ablib/NAME.so), ROUNDS rounds (default 2).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/abn; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "generated_configs or lane_mode or packed or value_ranges or encode or budget or early_exit or device_resident or wave_mode" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    L=ablib/$v.so; [ $v = prod ] && L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so
    step lone_${v}_$r env QSMD_LIB_PATH=$L python tools/stage0_anatomy.py 1000000 26
    python3 -c "import json; d=json.load(open('$O/lone_${v}_$r.out')); x=d['stage0_ms_events'][2:]; print('lone $v', round(sum(x)/len(x),4))"
    [ -n "$LONE_ONLY" ] && continue
    step drv_${v}_$r env QSMD_LIB_PATH=$L python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
    python3 -c "import json; d=json.load(open('$O/drv_${v}_$r.out')); print('drv $v', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"
  done
done
