#!/bin/bash
# Heavy-stage and stage-0 measurements (diagnostic): wave-mode stats, a PMC
# pass over the wave kernel, the stage-0 budget sweep and a stage-0 grid sweep.
set -o pipefail
mkdir -p gpurun_out/iter2
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/iter2
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 > $O/wave_stats.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 wave_min_rem=64 > $O/wave_stats_nomemo.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    -d $O/pmc1 -o run --output-format csv -- python3 tools/wave_stats.py bank_4x16 1000000 > $O/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    -d $O/pmc2 -o run --output-format csv -- python3 tools/wave_stats.py bank_4x16 1000000 > $O/pmc2.log 2>&1 &&
bash tools/gpu/sweep_budget.sh "14 16 18 20 23 26 32" 100 > $O/sweep.log 2>&1
rc=$?
cat $O/wave_stats.log $O/wave_stats_nomemo.log | grep -v amdgpu.ids
python3 - <<'PY'
import csv, glob, collections
for name in ("pmc1", "pmc2"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(f"gpurun_out/iter2/{name}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0][-40:]
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    last = {}
    for (k, d), v in sorted(per.items(), key=lambda x: int(x[0][1])):
        last[k] = v
    for k, v in last.items():
        print(name, k, {c: int(x) for c, x in sorted(v.items())})
PY
cat $O/sweep.log
exit $rc
