#!/bin/bash
# Round 4: the synchronous caller (one call at a time) and the driver's command, A/B against HEAD's build
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/sync; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
pj() { python3 -c "import json,sys; d=json.load(open('$O/$1.out')); print('$1', round(d['value']/1e9,3), 'alone s0', round(d['device_ms']['alone']['stage0_mean'],4), 'call', round(d['device_ms']['alone']['call_mean'],4))"; }
for r in 1 2; do
  for v in head prod; do
    L=ablib/$v.so; [ $v = prod ] && L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so
    step i1_${v}_$r env QSMD_LIB_PATH=$L python bench.py --inflight 1 --steps 200 --warmup 10 --no-cpu-baseline --no-extra; pj i1_${v}_$r
    step drv_${v}_$r env QSMD_LIB_PATH=$L python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra; pj drv_${v}_$r
  done
done
step ws_prod python tools/wave_stats.py bank_4x16 1000000
tail -2 $O/ws_prod.out
