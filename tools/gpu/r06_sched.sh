#!/bin/bash
# Round 6: the compiler's machine scheduling strategy for the whole library
# (tools/build_variant.sh with -mllvm --amdgpu-sched-strategy=... /
# --amdgpu-use-amdgpu-trackers) -- the driver's command per variant, 3
# rounds in rotation: value and the roofline leg's lone stage 0 / heavy stage.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_sched
mkdir -p $O
for r in 1 2 3; do
  for v in base maxilp itilp trackers memclause; do
    QSMD_LIB_PATH=$PWD/ablib/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/$v.$r.json 2> $O/$v.$r.err || { tail -3 $O/$v.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/$v.$r.json'))
print('$v round $r', '%.3e' % d['value'], 'mism', d.get('mismatches_vs_oracle'), {k: round(v, 4) for k, v in d['device_ms']['alone'].items() if v})
"
  done
done
