#!/bin/bash
# The round's measurements: the GPU suite, then the rocprofv3 evidence of the
# driver's command (profiles/profile.sh: kernel trace + FETCH_SIZE +
# WRITE_SIZE + SQ passes, summarised over the roofline leg's last 30 calls
# for stage 0 and the heavy stage; copied to $ROUND_DIR/stage0_pmc.json,
# which bench.py reads for the roofline's traffic), then the driver's bench
# command, the same over one resident batch (--rotate 1), the default bench
# (200 steps, CPU baselines, extra configs), one call at a time, and the
# early-exit leg.  Every GPU step has its own limit.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/measure
R=${ROUND_DIR:-profiles/r05}
mkdir -p $O $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
bash profiles/profile.sh $O/prof "--steps 20 --warmup 5 --no-cpu-baseline --no-extra" > $O/prof.log 2>&1 &&
cp $O/prof/summary.json $R/stage0_pmc.json &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --rotate 1 --no-extra --no-cpu-baseline > $O/bench_rotate1.json 2> $O/bench_rotate1.err &&
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/bench_inflight1.json 2> $O/bench_inflight1.err &&
timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 > $O/bench_early.json 2> $O/bench_early.err
rc=$?
for f in bench_driver bench_rotate1 bench_default bench_inflight1; do [ -s $O/$f.json ] && python3 -c "
import json; d=json.load(open('$O/$f.json')); r=d['roofline']
print('$f', '%.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], r['kernel'], 'frac %.4f' % r['frac'], {k: (round(v['frac'], 4), v['kernel_ms']['mean'], v['traffic']) for k, v in r['kernels'].items()}, 'alone', d['device_ms']['alone'], 'mism', d.get('mismatches_vs_oracle'))
"; done
[ -s $O/bench_early.json ] && python3 -c "import json; d=json.load(open('$O/bench_early.json')); print('early', json.dumps(d['early_exit']))"
tail -40 $O/prof.log
exit $rc
