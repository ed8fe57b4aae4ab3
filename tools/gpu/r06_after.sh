#!/bin/bash
# Round 6: lane mode's memo_after (probes after this many nodes; failed
# subtrees are recorded from the start since round 6) at 0 / 8 / 16 / 32:
# the heavy stage's anatomy on config 2 at the bench's knobs, then the
# driver's command and one call at a time, 2 interleaved rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_after}
mkdir -p $O
for ma in 0 8 16 32; do
  timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 stage0_budget=20 heavy_mode=1 memo_lds=0 memo_after=$ma > $O/ms_ma$ma.json 2> $O/ms_ma$ma.err || { tail $O/ms_ma$ma.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/ms_ma$ma.json'))
print('memo_after $ma', 'span_us', d['stage_span_us'], 'max_it', d['max_iterations'], 'cyc/it', d['cycles_per_iteration'], 'hits', d['memo_hits_total'], 'probe frac', d.get('fraction_of_wave_iterations'))
"
done
for r in 1 2; do
  for ma in 0 16 32; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param memo_after=$ma > $O/d$ma.$r.json 2> $O/d$ma.$r.err || { tail $O/d$ma.$r.err; exit 1; }
    timeout -k 10 200 python bench.py --inflight 1 --steps 50 --warmup 5 --no-extra --no-cpu-baseline --param memo_after=$ma > $O/i$ma.$r.json 2> $O/i$ma.$r.err || { tail $O/i$ma.$r.err; exit 1; }
    python3 -c "
import json
d = json.load(open('$O/d$ma.$r.json')); i = json.load(open('$O/i$ma.$r.json'))
print('memo_after $ma round $r', 'driver %.3e' % d['value'], 'heavy %.4f' % d['device_ms']['alone']['heavy_mean'], 'one-at-a-time %.3e' % i['value'], 'call %.4f' % i['device_ms']['alone']['call_mean'])
"
  done
done
