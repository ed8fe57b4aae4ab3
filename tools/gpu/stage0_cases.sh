#!/bin/bash
# tools/stage0_cases.py under a kernel trace; per-case median kernel durations.
#   tools/gpu/stage0_cases.sh CONFIG N REPS CASE...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/s0c
timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d gpurun_out/s0c -o run -- \
    python3 tools/stage0_cases.py "$@" > gpurun_out/s0c.log 2> gpurun_out/s0c.err || exit $?
cat gpurun_out/s0c.log
python3 tools/trace_cases.py gpurun_out/s0c "$3" "${@:4}"
