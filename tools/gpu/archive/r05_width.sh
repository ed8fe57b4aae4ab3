#!/bin/bash
# Lane mode with fewer histories per wavefront (knob lane_width): parity,
# then one call at a time (lane mode forced) and the driver's command.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/width
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "lane_width or lane_mode or resume_cap or fold" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for w in 64 32 16 8; do
    timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline --param heavy_mode=1 --param lane_width=$w > $O/i_${w}_$r.json 2> $O/i_${w}_$r.err || exit 1
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param lane_width=$w > $O/b_${w}_$r.json 2> $O/b_${w}_$r.err || exit 1
    python3 -c "
import json
for f in ('i', 'b'):
    d = json.load(open('$O/%s_${w}_$r.json' % f)); a = d['device_ms']['alone']
    print('$w', $r, f, '%.3e' % d['value'], 'stage0 %.4f heavy %.4f call %.4f' % (a['stage0_mean'], a['heavy_mean'], a['call_mean']), 'mism', d.get('mismatches_vs_oracle'))"
  done
done
