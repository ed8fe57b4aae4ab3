#!/bin/bash
# Round 5: why distinct resident batches are slower -- kernel traces of the
# driver's command with one batch and with five (--rotate 5).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_rot2
mkdir -p $O
B="--steps 20 --warmup 5 --no-extra --no-cpu-baseline"
for k in 1 5; do
  timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace -d $O/k$k -o run --output-format csv -- python3 bench.py $B --rotate $k > $O/k$k.json 2> $O/k$k.err || { tail $O/k$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/k$k.json')); print('rotate $k %.3e' % d['value'])"
done
