#!/bin/bash
# A/B: stage 0's packed staging loads non-temporal (abtmp/nt.so, built with
# -DQSMD_NT_STAGE) against the plain loads (lib/), 3 rounds of the driver's
# command and the 200-step default.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_nt
mkdir -p $O
for r in 1 2 3 4 5; do
  for v in nt base; do
    E=""; [ $v = nt ] && E="QSMD_LIB_PATH=$PWD/abtmp/nt.so"
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('$v $r %.3e' % d['value'], {k: round(v*1e3,1) for k, v in d['device_ms']['alone'].items()})"
  done
done
for v in nt base; do
  E=""; [ $v = nt ] && E="QSMD_LIB_PATH=$PWD/abtmp/nt.so"
  env $E timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline > $O/d.json 2> $O/d.err || { tail $O/d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/d.json')); print('200 $v %.3e' % d['value'])"
done
