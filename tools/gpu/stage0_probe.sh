#!/bin/bash
# Stage 0 anatomy (diagnostic): the no-search build (QSMD_DIAG_STAGE0=1) and
# the product build at several stage-0 grid caps, then SQ / TA counters of the
# no-search build.  tools/build_variant.sh diag0 "-DQSMD_DIAG_STAGE0=1" first.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/s0probe
mkdir -p $O
rocprofv3 -L > $O/counters_available.txt 2>&1 || true
bash tools/gpu/diag_stage0.sh "ablib/diag0.so" "ablib/diag0.so stage0_grid=4096" "ablib/diag0.so stage0_grid=2048" \
    "quickcheck-state-machine-distributed_amd/lib/libqsmd.so" "quickcheck-state-machine-distributed_amd/lib/libqsmd.so stage0_grid=4096" \
    "quickcheck-state-machine-distributed_amd/lib/libqsmd.so stage0_grid=2048" > $O/grid.log 2>&1 || { cat $O/grid.log; exit 1; }
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
            "TA_BUSY_avr TA_TA_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" ; do
  tag=$(echo $pass | cut -d' ' -f1)
  QSMD_LIB_PATH=ablib/diag0.so timeout -s KILL 90 rocprofv3 --pmc $pass -d $O/pmc_$tag -o run --output-format csv \
      -- python3 tools/stage_times.py bank_4x16 1000000 > $O/pmc_$tag.log 2>&1
  echo "pass $tag rc=$?"
done
cat $O/grid.log
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/s0probe/pmc_*")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "compact_search" in r["Kernel_Name"] and "G32" in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if per:
        k = sorted(per)[-1]
        print(d.split("/")[-1], {c: round(v) for c, v in sorted(per[k].items())})
PY
