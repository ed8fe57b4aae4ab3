#!/bin/bash
# Round 5: the bench as the driver runs it (4 calls in flight), one batch
# against five distinct resident batches (--rotate 5), 3 alternating rounds;
# then the full default command once (CPU baselines, extra configs).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_val
mkdir -p $O
for r in 1 2 3; do
  for k in 1 5 3; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --rotate $k > $O/r.json 2> $O/r.err || { tail $O/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r.json')); print('rotate $k $r %.3e' % d['value'])"
  done
done
timeout -k 10 400 python bench.py > $O/default.json 2> $O/default.err || { tail -30 $O/default.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05_val/default.json"))
print("default %.3e" % d["value"], "mism", d.get("mismatches_vs_oracle"), "cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["multi_thread"]["value"])
r = d["roofline"]; print(r["kernel"], {k: (round(v["frac"], 4), round(v["kernel_ms"]["mean"], 4)) for k, v in r["kernels"].items()})
print({k: (round(v.get("histories_per_sec", 0) / 1e9, 3), v.get("mismatches_vs_oracle"), v.get("ms_per_history"), v.get("cpu_ms_per_history")) for k, v in d["extra"]["configs"].items()})
PY
