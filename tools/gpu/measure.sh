#!/bin/bash
# The round's measurements: the rocprofv3 evidence of the driver's command
# (profiles/profile.sh: kernel trace + FETCH_SIZE + WRITE_SIZE + SQ passes,
# summarised over the roofline leg's 30 stage-0 launches; copied to
# $ROUND_DIR/stage0_pmc.json, which bench.py reads for roofline.traffic),
# then the driver's bench command, the default bench (200 steps, CPU
# baselines, extra configs) and one call at a time.  Every GPU step has its
# own time limit.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/measure
R=${ROUND_DIR:-profiles/r04}
mkdir -p $O $R
# the PMC evidence first: the benches below fill roofline.traffic from it
bash profiles/profile.sh $O/prof "--steps 20 --warmup 5 --no-cpu-baseline --no-extra" > $O/prof.log 2>&1 &&
cp $O/prof/summary.json $R/stage0_pmc.json &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 200 python bench.py --inflight 1 --no-extra --no-cpu-baseline > $O/bench_inflight1.json 2> $O/bench_inflight1.err
rc=$?
for f in bench_driver bench_default bench_inflight1; do [ -s $O/$f.json ] && python3 -c "
import json; d=json.load(open('$O/$f.json')); r=d['roofline']
print('$f', '%.3e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % r['frac'], 'traffic', r.get('traffic'), 'kernel_ms', r['kernel_ms']['mean'], 'alone', d['device_ms']['alone'], 'mism', d.get('mismatches_vs_oracle'))
"; done
tail -40 $O/prof.log
exit $rc
