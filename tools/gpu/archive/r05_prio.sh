#!/bin/bash
# Round 5: the in-flight critical path is one stream's chain (stage 0, then
# its heavy stage beside the other two streams' stage 0s).  A/B at the
# driver's 20 steps, 3 rounds: the heavy stage's waves at issue priority 1 / 3
# (diagnostic builds ablib/prio*.so), 4 calls in flight (on the box's 4
# hardware queues, and on 8), and the RCCL path after the bench's fixes.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_prio
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in base prio1 prio3 if4 if4q8 dist; do
    E=""; A=""
    case $v in
      prio1) E="QSMD_LIB_PATH=$PWD/ablib/prio1.so";;
      prio3) E="QSMD_LIB_PATH=$PWD/ablib/prio3.so";;
      if4) A="--inflight 4";;
      if4q8) A="--inflight 4 --hw-queues 8";;
      dist) E="QSMD_BENCH_DIST=1";;
    esac
    env $E timeout -k 10 120 python bench.py $B $A > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('$v $r %.3e' % d['value'], 'alone', d['device_ms']['alone'])"
  done
done
