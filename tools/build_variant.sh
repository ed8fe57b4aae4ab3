#!/bin/bash
# Build a variant of lib/libqsmd.so with extra compiler flags into
# ablib/NAME.so (diagnostic / A-B builds; ablib/ is git-ignored but travels
# to the GPU box):   tools/build_variant.sh NAME "-DQSMD_DIAG_STAGE0=1"
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/quickcheck-state-machine-distributed_amd
OUT=$ROOT/ablib/$NAME
mkdir -p "$OUT"
objs=()
for f in compact memo wave gen wellformed split api; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -I"$ROOT/include" -I"$PKG/csrc" $FLAGS \
    -c "$PKG/csrc/$f.hip" -o "$OUT/$f.o" &
  objs+=("$OUT/$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$ROOT/ablib/$NAME.so"
echo "ablib/$NAME.so"
