#!/bin/bash
# tools/gpu/check.sh, then the default bench (200 steps, extra configs).
bash tools/gpu/check.sh && \
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_default.json'))
print('default', d['value'], d['device_ms'])
for k,v in d.get('extra',{}).get('configs',{}).items(): print(k, {x: v[x] for x in v if x in ('value','unit','mismatches_vs_oracle','device_ms_per_call','ms_per_history')})
" 2>/dev/null
exit $rc
