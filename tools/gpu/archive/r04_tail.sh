#!/bin/bash
# Round 4: the synchronous caller's tail after stage 0 -- per-stage device
# times of one call (QSMD_SYNC_STAGES=1) at the library's defaults and at the
# bench's knobs, and the one-call-at-a-time bench.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/tail; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
step st_default env QSMD_SYNC_STAGES=1 python tools/stage_times.py bank_4x16 1000000
tail -12 $O/st_default.err
step st_bench env QSMD_SYNC_STAGES=1 python tools/stage_times.py bank_4x16 1000000 stage0_budget=26 heavy_mode=1 memo_lds=0
tail -12 $O/st_bench.err
step i1 python bench.py --inflight 1 --steps 200 --warmup 10 --no-cpu-baseline --no-extra
python3 -c "import json; d=json.load(open('$O/i1.out')); print('i1', round(d['value']/1e9,3), d['ms_per_step'], d['device_ms'])"
step ws python tools/wave_stats.py bank_4x16 1000000
tail -3 $O/ws.out
