#!/bin/bash
# Stage-0 time of diagnostic builds (tools/build_variant.sh) and settings:
# per-launch device times from tools/stage_times.py, one process per case.
#   tools/gpu/archive/diag_stage0.sh "lib.so [param=value ...]" ...
set -o pipefail
mkdir -p gpurun_out/diag
i=0
for spec in "$@"; do
  set -- $spec; lib=$1; shift
  i=$((i+1)); tag=$i.$(basename "$lib" .so)
  QSMD_LIB_PATH=$lib QSMD_SYNC_STAGES=1 timeout -k 10 120 python -u tools/stage_times.py bank_4x16 1000000 "$@" \
      > gpurun_out/diag/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/diag/$tag.log; exit 1; }
  echo "== $tag $*"; grep -v amdgpu.ids gpurun_out/diag/$tag.log | grep -E "stage0 |lane " | tail -2
done
