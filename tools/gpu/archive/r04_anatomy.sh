#!/bin/bash
# Round 4: stage 0's anatomy on a lone call (config 2, bench knobs).
#   1. the stamped diagnostic build: per-group staging / search cycles, timeline
#   2. lone stage-0 event times of the product build and the no-search build
#   3. PMC of both builds over the same lone calls (SQ counters, FETCH_SIZE)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/anat; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 240 "$@" > $O/$name.out 2> $O/$name.err; local rc=$?;
         echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }; }
step stamp env QSMD_LIB_PATH=ablib/s0stamp.so python tools/stage0_anatomy.py
step lone_prod python tools/stage0_anatomy.py
step lone_nos env QSMD_LIB_PATH=ablib/s0nosearch.so python tools/stage0_anatomy.py
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
for lib in prod nos; do
  L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so; [ $lib = nos ] && L=ablib/s0nosearch.so
  export QSMD_LIB_PATH=$L
  step pmc_sq_$lib rocprofv3 --pmc $SQ -d $O/pmc_sq_$lib -o run --output-format csv -- python3 tools/stage0_anatomy.py
  step pmc_fetch_$lib rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$lib -o run --output-format csv -- python3 tools/stage0_anatomy.py
  step trace_$lib rocprofv3 --kernel-trace --stats -d $O/trace_$lib -o run --output-format csv -- python3 tools/stage0_anatomy.py
done
cat $O/stamp.out | head -40
