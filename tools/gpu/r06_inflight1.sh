#!/bin/bash
# Round 6: one call at a time (bench.py --inflight 1, the library's
# automatic budget: 16 on config 2, ~96k heavy histories) against the
# round's knobs: the giant stage's grid on folded calls, the tail launch,
# stage 0's bucketed heavy list.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_inflight1}
mkdir -p $O
for r in 1 2; do
  for v in default gg64 tc0 hb0 all0; do
    case $v in
      default) P="";; gg64) P="--param giant_grid=64";; tc0) P="--param tail_cap=0";; hb0) P="--param heavy_buckets=0";;
      all0) P="--param giant_grid=64 --param tail_cap=0 --param heavy_buckets=0";;
    esac
    timeout -k 10 200 python bench.py --inflight 1 --steps 50 --warmup 5 --no-extra --no-cpu-baseline $P > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/$v.$r.json'))
print('$v round $r', '%.3e' % d['value'], 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
