#!/bin/bash
# Lane mode's memo tables in LDS (memo_lds 2: forced; 1, the default: when
# the last call's heavy groups fit the CUs) for config 2 at budget 20, where
# the heavy groups (~257) sit at the CU count: the driver's command and one
# call at a time, 2 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/lt
mkdir -p $O
for r in 1 2; do
  for v in 1 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param memo_lds=$v > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline --param memo_lds=$v > $O/i_${v}_$r.json 2> $O/i_${v}_$r.err || exit 1
    python3 -c "
import json
for f in ('b', 'i'):
    d = json.load(open('$O/%s_${v}_$r.json' % f)); a = d['device_ms']['alone']
    print('$v', $r, f, '%.3e' % d['value'], 'stage0 %.4f heavy %.4f call %.4f' % (a['stage0_mean'], a['heavy_mean'], a['call_mean']), 'mism', d.get('mismatches_vs_oracle'))"
  done
done
