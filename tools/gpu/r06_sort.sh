#!/bin/bash
# Round 6: the heavy stage's groups in order of predicted work (stage 0's
# heavy_key + memo.hip heavy_sort) -- the parity tests, config 3 with the
# ordering on / off and the tail at 256, and config 2 one call at a time and
# in the driver's command (no ordering: short lists).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_sort}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "buckets or tail or lane_mode or fold or cascade" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for hb in 0 1; do
    timeout -k 10 200 python bench.py --config bank_4x16_bugs --steps 10 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --param heavy_buckets=$hb > $O/c3_hb$hb.$r.json 2> $O/c3_hb$hb.$r.err || { tail $O/c3_hb$hb.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/c3_hb$hb.$r.json'))
print('config3 heavy_buckets $hb round $r', '%.3e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
timeout -k 10 120 python tools/memo_stats.py bank_4x16_bugs 1000000 heavy_mode=1 memo_lds=0 tail_cap=0 tail_min=0 heavy_buckets=1 > $O/ms_c3_sorted.json 2> $O/ms_c3_sorted.err || { tail $O/ms_c3_sorted.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/ms_c3_sorted.json'))
print('memo_stats sorted', 'span_us', d['stage_span_us'], 'util', d['lane_utilisation'], 'max_it', d['max_iterations'], 'stage0_us', d['stage0_us'], 'call_us', d['call_device_us'])
"
timeout -k 10 200 python bench.py --inflight 1 --steps 50 --warmup 5 --no-extra --no-cpu-baseline > $O/c2_inflight1.json 2> $O/c2_inflight1.err || { tail $O/c2_inflight1.err; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/c2_driver.json 2> $O/c2_driver.err || { tail $O/c2_driver.err; exit 1; }
python3 -c "
import json
for f in ('c2_inflight1', 'c2_driver'):
    d = json.load(open('$O/%s.json' % f)); print(f, '%.3e' % d['value'], 'alone', {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v}, 'mism', d.get('mismatches_vs_oracle'))
"
