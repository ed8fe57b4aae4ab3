#!/bin/bash
# Round 6: (1) config 4 through the host entry under a kernel + HIP API trace
# (the chain path; tools/config4.py, tools/trace_c4.py); (2) config 3's
# exhaustive call (bench.py's extra-config shape: 1M, 3 in flight) with the
# lane-mode hand-off to the giant stage after 64 x split_budget iterations,
# split_budget 1024 (default) / 8 / 6 / 4; (3) the driver's command with the
# giant stage on 2 workgroups per CU (giant_grid 512) against the default.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_c3c4}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/trace -o c4 -- python3 tools/config4.py --reps 100 > $O/c4_traced.log 2>&1 || { tail -20 $O/c4_traced.log; exit 1; }
python3 tools/trace_c4.py $O/trace > $O/c4_summary.txt 2>&1 || { tail $O/c4_summary.txt; exit 1; }
find $O/trace -name "*_trace.csv" -size +2M -delete
cat $O/c4_summary.txt
for sb in 1024 8 6 4; do
  timeout -k 10 200 python bench.py --config bank_4x16_bugs --steps 10 --warmup 3 --inflight 3 --no-extra --no-cpu-baseline --param split_budget=$sb > $O/c3_sb$sb.json 2> $O/c3_sb$sb.err || { tail $O/c3_sb$sb.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/c3_sb$sb.json'))
print('config3 split_budget $sb', '%.3e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'mism', d.get('mismatches_vs_oracle'), 'alone', d['device_ms']['alone'])
"
done
for r in 1 2 3; do
  for gg in 0 512; do
    P=""; [ $gg != 0 ] && P="--param giant_grid=$gg"
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline $P > $O/gg$gg.$r.json 2> $O/gg$gg.$r.err || { tail $O/gg$gg.$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/gg$gg.$r.json'))
print('giant_grid $gg round $r', '%.3e' % d['value'], 'alone', d['device_ms']['alone'])
"
  done
done
