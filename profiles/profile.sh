#!/bin/bash
# Collect the rocprofv3 evidence for the dominant kernel (run on the GPU box
# from the repo root):  profiles/profile.sh <out_dir> [bench args...]
#   1. --kernel-trace --stats            per-kernel durations
#   2. --pmc FETCH_SIZE                   HBM read bytes   (own pass)
#   3. --pmc WRITE_SIZE                   HBM write bytes  (own pass)
#   4. --pmc SQ_* (two passes)            waves, busy/wait cycles, VALU/LDS
# then profiles/summarize_pmc.py writes <out_dir>/summary.json over the last
# 30 stage-0 dispatches: bench.py's roofline leg (30 synchronous calls after
# its timed region), the launches its roofline.kernel_ms times.
# Every pass has its own time limit; a pass that times out, aborts or
# crashes stops the script (nothing further runs on the GPU).
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=${@:-"--steps 20 --warmup 5 --no-cpu-baseline --no-extra"}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS \
      > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
  return 0
}
rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
python3 profiles/summarize_pmc.py "$OUT" --last 30 > "$OUT/summary.json"
cat "$OUT/summary.json"
