#!/bin/bash
# Round 5: the new tests (fold, resume cap, scoped host waits, the 9-bit
# value bounds, the device-resident sharded early exit), the new bench legs
# (two-kernel roofline, --rotate, --early-exit), and the heavy stage's
# cycles per DFS iteration without its memo / with LDS tables.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_check
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "dist or fold or resume_cap or host_waits or value_ranges or early_exit or timing" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/b20.json 2> $O/b20.err || { tail -20 $O/b20.err; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --rotate 4 --cpu-seconds 2 > $O/rot4.json 2> $O/rot4.err || { tail -20 $O/rot4.err; exit 1; }
timeout -k 10 200 python bench.py --early-exit --steps 5 --warmup 2 > $O/ee.json 2> $O/ee.err || { tail -20 $O/ee.err; exit 1; }
K="stage0_budget=18 heavy_mode=1"
for v in "memo_lds=0" "memo_lds=0 memo_after=1000000000" "memo_lds=2" "memo_lds=2 memo_lds_entries=16" "memo_lds=0 memo_after=18"; do
  timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K $v > $O/ms.json 2> $O/ms.err || { tail $O/ms.err; exit 1; }
  echo "$v: $(cat $O/ms.json)"
done
python3 - <<'PY'
import json
for f in ("b20", "rot4", "ee"):
    d = json.load(open(f"gpurun_out/r05_check/{f}.json"))
    print(f, "%.3e" % d["value"], json.dumps({k: d.get(k) for k in ("device_ms", "mismatches_vs_oracle", "checked_batch", "early_exit")})[:900])
    if "roofline" in d:
        r = d["roofline"]
        print("  roof", r["kernel"], "frac %.4f" % r["frac"], {k: (round(v["frac"], 4), v["kernel_ms"]["mean"]) for k, v in r["kernels"].items()}, "budget", r["stage0_budget_used"])
PY
