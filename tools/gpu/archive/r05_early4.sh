#!/bin/bash
# The giant stage without giants (early exit): the whole GPU suite, then the
# early-exit step's floor and kernels, and the bench leg.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/early4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/micro/early_split.py > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
grep -v "rocprofv3\|simple_timer\|output_stream\|tool.cpp" $O/prof.log | tail -7
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | grep qsmd
for fc in 0 4096; do
  timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 --no-cpu-baseline --first-chunk $fc > $O/early_$fc.json 2> $O/early_$fc.err || exit 1
  python3 -c "import json; d=json.load(open('$O/early_$fc.json')); e=d['early_exit']; print($fc, '%.3e' % d['value'], 'ms %.4f' % d['ms_per_step'], e['searched'], e['rounds'])"
done
