#!/bin/bash
# PMC passes over tools/stage_times.py (config 2, 4 calls): instruction mix
# and stall buckets of every kernel.  One pass per counter group.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${ARGS:-bank_4x16 1000000}
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc1 -o run -- python3 tools/stage_times.py $ARGS > gpurun_out/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU -d gpurun_out/pmc2 -o run -- python3 tools/stage_times.py $ARGS > gpurun_out/pmc2.log 2>&1
rc=$?
python3 tools/pmc_table.py gpurun_out/pmc1 gpurun_out/pmc2 --json gpurun_out/pmc.json 2>&1 | tail -80
exit $rc
