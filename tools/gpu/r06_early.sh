#!/bin/bash
# Round 6: the lane-mode heavy stage recording failed subtrees from its start
# (probes after memo_after), its backtrack reads batched, against HEAD's build
# (ablib/base_r06.so): the GPU suite, the heavy stage's anatomy
# (tools/memo_stats.py) of both builds on configs 2 and 3 at the bench's
# knobs, A/B of the driver's command and of one call at a time
# (tools/ab.py), then config 4 (the wave stage chain path) with and without the DAG.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_early}
mkdir -p $O
K="stage0_budget=20 heavy_mode=1 memo_lds=0"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for lib in base_r06 new; do
  if [ $lib = new ]; then L=quickcheck-state-machine-distributed_amd/lib/libqsmd.so; else L=ablib/$lib.so; fi
  QSMD_LIB_PATH=$L timeout -k 10 120 python tools/memo_stats.py bank_4x16 1000000 $K > $O/ms_c2_$lib.json 2> $O/ms_c2_$lib.err || { tail $O/ms_c2_$lib.err; exit 1; }
  QSMD_LIB_PATH=$L timeout -k 10 120 python tools/memo_stats.py bank_4x16_bugs 1250000 heavy_mode=1 memo_lds=0 > $O/ms_c3_$lib.json 2> $O/ms_c3_$lib.err || { tail $O/ms_c3_$lib.err; exit 1; }
done
python3 - <<EOF
import json
for c in ("c2", "c3"):
    for lib in ("base_r06", "new"):
        d = json.load(open("$O/ms_%s_%s.json" % (c, lib)))
        print(c, lib, "span_us", d["stage_span_us"], "max_it", d["max_iterations"], "cyc/it", d["cycles_per_iteration"],
              "hits", d["memo_hits_total"], "its", d["iterations_total"])
EOF
timeout -k 10 400 python tools/ab.py ablib/base_r06.so quickcheck-state-machine-distributed_amd/lib/libqsmd.so 3 --steps 20 --warmup 5 > $O/ab_inflight.txt 2>&1 || { tail $O/ab_inflight.txt; exit 1; }
tail -2 $O/ab_inflight.txt
timeout -k 10 300 python tools/ab.py ablib/base_r06.so quickcheck-state-machine-distributed_amd/lib/libqsmd.so 3 --steps 50 --warmup 5 --inflight 1 > $O/ab_alone.txt 2>&1 || { tail $O/ab_alone.txt; exit 1; }
tail -2 $O/ab_alone.txt
timeout -k 10 120 python3 tools/config4.py --reps 50 "" "dag_states=0" > $O/c4.log 2>&1 || { tail $O/c4.log; exit 1; }
cat $O/c4.log
