#!/bin/bash
# Bank balances in registers (abtmp/balregs.so, -DQSMD_BAL_REGS=1) against
# LDS (lib/libqsmd.so): the lane-mode / cascade parity tests on the variant,
# then the driver's command and one call at a time, interleaved, 3 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/balregs
mkdir -p $O
QSMD_LIB_PATH=$PWD/abtmp/balregs.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in lds regs; do
    if [ $v = regs ]; then export QSMD_LIB_PATH=$PWD/abtmp/balregs.so; else unset QSMD_LIB_PATH; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/i_${v}_$r.json 2> $O/i_${v}_$r.err || exit 1
    python3 -c "
import json
for f in ('b', 'i'):
    d = json.load(open('$O/%s_${v}_$r.json' % f)); a = d['device_ms']['alone']
    print('$v', $r, f, '%.3e' % d['value'], 'stage0 %.4f heavy %.4f call %.4f' % (a['stage0_mean'], a['heavy_mean'], a['call_mean']), 'mism', d.get('mismatches_vs_oracle'))"
  done
done
