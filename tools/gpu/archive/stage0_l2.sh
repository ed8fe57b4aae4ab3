#!/bin/bash
# Round 4: stage 0 with its HBM reads turned into L2 hits (diagnostic builds),
# lone stage-0 times, one workgroup per group (stage0_persistent=0)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/ab3; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -15 $O/$name.out; tail -5 $O/$name.err; exit $rc; }; }
step stamp_l2 env QSMD_LIB_PATH=ablib/l2stamp.so QSMD_STAMPS_OUT=$O/stamps_l2.npy python tools/stage0_anatomy.py 1000000 26
step stamp_np env QSMD_LIB_PATH=ablib/s0stamp.so QSMD_STAMPS_OUT=$O/stamps_np.npy python tools/stage0_anatomy.py 1000000 26
for r in 1 2; do
for v in head prod l2 l2nos s0nosearch; do
  L=ablib/$v.so; [ $v = prod ] && L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so
  step lone_${v}_$r env QSMD_LIB_PATH=$L python tools/stage0_anatomy.py 1000000 26
  python3 -c "import json; d=json.load(open('$O/lone_${v}_$r.out')); x=d['stage0_ms_events'][2:]; print('$v', round(sum(x)/len(x),4), [round(y,4) for y in x])"
done
done
