#!/bin/bash
# One-rank cost of the RCCL path (verdict r01 item 6) and the hardware-queue
# count: bench.py runs with and without RCCL initialised (QSMD_BENCH_DIST=1),
# with and without the all-reduce (QSMD_BENCH_NOAR=1), per in-flight depth
# and GPU_MAX_HW_QUEUES.  tools/gpu/archive/rccl_sweep.sh [rounds] "TAG|ENV|ARGS" ...
set -o pipefail
R=${1:-3}; shift
STEPS=${STEPS:-60}
mkdir -p gpurun_out/rccl
rm -f gpurun_out/rccl/*.json gpurun_out/rccl/*.err
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  for r in $(seq 1 "$R"); do
    env $envs timeout -k 10 150 python bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-extra $args \
        > "gpurun_out/rccl/$tag.$r.json" 2> "gpurun_out/rccl/$tag.$r.err" || exit $?
  done
done
python3 - <<'PY'
import glob, json, statistics
res = {}
for f in sorted(glob.glob("gpurun_out/rccl/*.json")):
    tag = f.split("/")[-1].rsplit(".", 2)[0]
    res.setdefault(tag, []).append(json.loads(open(f).read().strip().splitlines()[-1])["value"] / 1e9)
for k, v in res.items():
    print(k, [round(x, 3) for x in v], "median", round(statistics.median(v), 3))
PY
