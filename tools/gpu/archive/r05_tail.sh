#!/bin/bash
# Lane mode's tail hand-off (knob tail_cap): parity, then the driver's
# command and one call at a time across caps.  Every GPU step has its own limit.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/tail
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "tail_cap or lane_mode or resume_cap or fold or cascade" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
show() { python3 -c "
import json; d=json.load(open('$1')); r=d['roofline']
print('$2', '%.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], {k: (round(v['frac'], 4), v['kernel_ms']['mean']) for k, v in r['kernels'].items()}, 'alone', d['device_ms']['alone'], 'mism', d.get('mismatches_vs_oracle'))"; }
for cap in 0 24 16 32 48 0 24; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param tail_cap=$cap > $O/b_$cap.json 2> $O/b_$cap.err || exit 1
  show $O/b_$cap.json "cap $cap"
done
for cap in 0 24 16; do
  timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline --param tail_cap=$cap > $O/i1_$cap.json 2> $O/i1_$cap.err || exit 1
  show $O/i1_$cap.json "inflight1 cap $cap"
done
