#!/bin/bash
# SQ counters of stage 0 for several library builds (diagnostic):
#   tools/gpu/pmc_variants.sh lib.so ...   -> gpurun_out/pmcv/<lib>/<pass>/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcv
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
              "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD"; do
    p=$(echo $pass | cut -c1-12 | tr ' ' _)
    QSMD_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/pmcv/$tag/$p -o run --output-format csv \
        -- python3 tools/stage_times.py bank_4x16 1000000 > gpurun_out/pmcv/$tag.$p.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$tag $p rc=$rc"; tail -3 gpurun_out/pmcv/$tag.$p.log; exit $rc; fi
  done
done
python3 - <<'PY'
import csv, glob, os, collections
for d in sorted(glob.glob("gpurun_out/pmcv/*/")):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "compact_search" in r["Kernel_Name"] and "G32" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")), {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
