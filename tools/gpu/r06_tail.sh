#!/bin/bash
# Round 6: lane mode's wave-mode tail launch (api.hip tail_cap / tail_min):
# the lane-mode and tail parity tests, then config 3's exhaustive call in
# bench.py's extra-config shape (1M, 3 in flight, the library's budget) at
# tail_cap 0 (off) / 128 / 192 / 256 / 384, then the driver's command
# (config 2: its heavy list stays under tail_min, no tail) at 0 and 256.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_tail}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lane_mode or tail or cascade or fold" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for tc in 0 128 192 256 384; do
  timeout -k 10 200 python bench.py --config bank_4x16_bugs --steps 10 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --param tail_cap=$tc > $O/c3_tc$tc.json 2> $O/c3_tc$tc.err || { tail $O/c3_tc$tc.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/c3_tc$tc.json'))
print('config3 tail_cap $tc', '%.3e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'mism', d.get('mismatches_vs_oracle'), 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
done
for r in 1 2; do
  for tc in 0 256; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param tail_cap=$tc > $O/c2_tc$tc.$r.json 2> $O/c2_tc$tc.$r.err || { tail $O/c2_tc$tc.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/c2_tc$tc.$r.json'))
print('config2 tail_cap $tc round $r', '%.3e' % d['value'], 'mism', d.get('mismatches_vs_oracle'))
"
  done
done
