#!/bin/bash
# Kernel-trace stats for two bench argument sets (one call in flight):
#   tools/gpu/prof_ab.sh "ARGS_A" "ARGS_B"   -> gpurun_out/pab_{a,b}/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for args in "$@"; do
  name=pab_$i
  timeout -k 10 180 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/$name -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --inflight 1 $args \
      > gpurun_out/$name.json 2> gpurun_out/$name.err || exit $?
  echo "== [$args]"
  find gpurun_out/$name -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-6 | cut -c1-160
  i=$((i+1))
done
