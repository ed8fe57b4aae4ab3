#!/bin/bash
# The driver's bench command N times, then one call in flight (diagnostic).
set -o pipefail
N=${1:-3}
mkdir -p gpurun_out/drv
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/drv/drv$i.json 2> gpurun_out/drv/drv$i.err || exit 1
done
timeout -k 10 200 python bench.py --inflight 1 --steps 50 --no-cpu-baseline --no-extra > gpurun_out/drv/inflight1.json 2> gpurun_out/drv/inflight1.err || exit 1
for f in gpurun_out/drv/*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['device_ms'])" "$f"
done
