#!/bin/bash
# Round 5: calls in flight 3..6 (one context + stream each, the box's 4
# hardware queues), with and without the heavy stage at issue priority 3
# (ablib/prio3.so), the driver's 20 steps, 3 rounds; then the extra
# configs at 3 and 4 in flight.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_if
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for r in 1 2 3; do
  for v in 3 4 5 6 4p 5p; do
    E=""
    case $v in *p) E="QSMD_LIB_PATH=$PWD/ablib/prio3.so";; esac
    n=${v%p}
    env $E timeout -k 10 120 python bench.py $B --inflight $n > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('if$v $r %.3e' % d['value'])"
  done
done
for n in 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --inflight $n > $O/x$n.json 2> $O/x$n.err || { tail $O/x$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/x$n.json')); print('extra if$n %.3e' % d['value'], {k: (round(v.get('histories_per_sec', 0)/1e9, 3), v.get('mismatches_vs_oracle'), v.get('ms_per_history')) for k, v in d['extra']['configs'].items()})"
done
