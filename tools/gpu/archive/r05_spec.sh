#!/bin/bash
# A/B: stage 0's speculative first staging step (knob spec_stage, default 1)
# against none (spec_stage=0), same library: the parity tests of the compact
# stages first, then lone stage 0 and the driver's command, 3 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_spec
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --param spec_stage=$v > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('spec $v $r %.3e' % d['value'], 'mism', d.get('mismatches_vs_oracle'), {k: round(v*1e3,1) for k, v in d['device_ms']['alone'].items()})"
  done
done
for v in 1 0; do
  timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --param spec_stage=$v > $O/d.json 2> $O/d.err || { tail $O/d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/d.json')); print('200 steps spec $v %.3e' % d['value'])"
done
