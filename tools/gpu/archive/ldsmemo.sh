#!/bin/bash
# In-flight bench A/B: lane-mode memo tables in HBM (the bench's default)
# vs in LDS with 16 / 32 / 64 entries per lane; then one GPU-parity slice.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/ldsmemo.log
: > $out
for r in 1 2; do
  for v in "" "--param memo_lds=1 --param memo_lds_entries=16" "--param memo_lds=1 --param memo_lds_entries=32" "--param memo_lds=1 --param memo_lds_entries=64"; do
    for st in "--steps 200 --warmup 10" "--steps 20 --warmup 5"; do
      line=$(timeout -k 10 120 python -u bench.py $st --no-extra --no-cpu-baseline $v 2>/dev/null | tail -1) || exit 1
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], sys.argv[3], round(d['value']/1e9,3), 'in_flight', d['device_ms']['in_flight'], 'alone', d['device_ms']['alone'])" "$line" "[$v]" "[$st]" >> $out
    done
  done
done
cat $out
